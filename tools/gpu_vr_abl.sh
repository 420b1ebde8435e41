#!/bin/bash
# k_rs_vr profiling ablations (FI_VR_VARIANT, wrong pixels except 0/5/6/9) on a
# bench workload, two rounds: VARIANTS="0 4" WL=cfg2 bash tools/gpu_vr_abl.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vrabl; mkdir -p $OUT
for rep in 1 2; do
for v in ${VARIANTS}; do
  FI_VR_VARIANT=$v timeout -k 10 200 python bench.py --workload ${WL:-cfg2} --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
    --no-verify > $OUT/v$v.json 2> $OUT/v$v.err || { echo "$v failed"; tail -3 $OUT/v$v.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/v$v.json'));s=d['stages_ms_per_step'];print('variant $v', d['ms_per_step'], 'resize', s['resize'])"
done
done
