#!/bin/bash
# A/B of one environment switch on a bench workload: AB_VAR=FI_SC_GROUPED AB_VALS="1 0" WL=cfg2 bash tools/gpu_ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab; mkdir -p $OUT
for rep in 1 2; do
for v in ${AB_VALS}; do
  env ${AB_VAR}=$v timeout -k 10 200 python bench.py --workload ${WL:-cfg2} --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
    > $OUT/${AB_VAR}_$v.json 2> $OUT/${AB_VAR}_$v.err || { echo "$v failed"; tail -3 $OUT/${AB_VAR}_$v.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/${AB_VAR}_$v.json'));s=d['stages_ms_per_step'];print('${AB_VAR}=$v', d['ms_per_step'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')), d['verified'][:5])"
done
done
