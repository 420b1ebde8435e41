#!/bin/bash
# A/B of library builds on one workload: the tree's libflyimg_hip.so vs tools/bin/lib<NAME>.so (FI_LIB_PATH)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
for rep in 1 2; do
for name in base ${NAMES:-}; do
  lib=""; [ "$name" != base ] && lib=$PWD/tools/bin/lib$name.so
  FI_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 3 ${WL:+--workload $WL} ${NOV:+--no-verify} > $OUT/ab_$name.json 2> $OUT/ab_$name.err || { echo "$name failed"; tail -3 $OUT/ab_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/ab_$name.json'));s=d['stages_ms_per_step'];print('$name', d['value'], d['ms_per_step'], 'resize', s['resize'], 'launch', d['roofline']['avg_launch_ms'], d['verified'][:5])"
done; done
