#!/bin/bash
# k_rs_vr ablations on cfg2 (FI_VR_VARIANT, wrong pixels: --no-verify): resize ms/step per variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
for v in ${VARIANTS:-0 1 3}; do
  FI_VR_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-verify --steps 10 --warmup 2 > $OUT/abl_$v.json 2> $OUT/abl_$v.err || { echo "variant $v failed"; tail -3 $OUT/abl_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/abl_$v.json'));s=d['stages_ms_per_step'];print('variant $v', d['ms_per_step'], 'resize', s['resize'], 'launch', d['roofline']['avg_launch_ms'])"
done
