#!/bin/bash
# Bench lines of the BASELINE configurations (one process each) -> gpurun_out/configs/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/configs; mkdir -p $OUT
for w in ${WORKLOADS:-cfg1 cfg3 cfg5}; do
  timeout -k 10 600 python bench.py --workload $w --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > $OUT/$w.json 2> $OUT/$w.err; rc=$?
  echo "$w rc=$rc"; tail -2 $OUT/$w.err
  python -c "import json;d=json.load(open('$OUT/$w.json'));print(d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d.get('verified'))" 2>/dev/null
  [ $rc -eq 0 ] || exit $rc
done
