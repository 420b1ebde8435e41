#!/bin/bash
# k_rs_vr FI_VR_VARIANT A/B on one workload: VARIANTS="0 4" WL=cfg2 bash tools/gpu_vr_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vrv; mkdir -p $OUT
for wl in ${WL:-cfg2}; do
for v in ${VARIANTS:-0 4}; do
  FI_VR_VARIANT=$v timeout -k 10 200 python bench.py --workload $wl --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-verify \
    > $OUT/${wl}_v$v.json 2> $OUT/${wl}_v$v.err || { echo "$wl v$v failed"; tail -3 $OUT/${wl}_v$v.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/${wl}_v$v.json'));print('$wl variant $v', d['ms_per_step'], d['stages_ms_per_step']['resize'], d['roofline']['frac'])"
done
done
