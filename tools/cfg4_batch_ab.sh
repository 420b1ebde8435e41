#!/bin/bash
# cfg4 batch-size A/B (FI_BENCH_CFG4_BATCH) -> gpurun_out/cfg4b/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cfg4b; mkdir -p $OUT
for b in ${BATCHES:-1024 2048 4096}; do
  FI_BENCH_CFG4_BATCH=$b timeout -k 10 400 python bench.py --workload cfg4 --steps 2 --warmup 1 --no-cpu-baseline \
    > $OUT/b$b.json 2> $OUT/b$b.err || { echo "batch $b rc=$?"; tail -3 $OUT/b$b.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/b$b.json'));s=d['stages_ms_per_step'];print($b, d['value'], d['ms_per_step'], d['roofline']['frac'], s.get('host_plan'), d.get('verified','')[:6])"
done
