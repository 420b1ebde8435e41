#!/bin/bash
# One more sample of the bench lines (no profiler) on whatever box this lands
# on -> gpurun_out/sample/ (box-to-box spread of the final tree's numbers)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sample; mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/cfg2.json 2> $OUT/cfg2.err || { echo "cfg2 rc=$?"; exit 3; }
for wl in cfg1 cfg3 cfg5; do
  timeout -k 10 600 python bench.py --workload $wl --no-cpu-baseline > $OUT/$wl.json 2> $OUT/$wl.err || { echo "$wl rc=$?"; exit 3; }
done
timeout -k 10 900 python bench.py --workload cfg4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err || { echo "cfg4 rc=$?"; exit 3; }
for wl in cfg2 cfg1 cfg3 cfg5 cfg4; do
  python3 -c "import json;d=json.load(open('$OUT/$wl.json'));print('$wl', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('verified','')[:5])"
done
