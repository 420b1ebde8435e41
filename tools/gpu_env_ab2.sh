#!/bin/bash
# Bench A/B of environment settings on the tree's library, twice:
#   ENVS="FI_VR_PF=0 FI_VR_PF=64" WL=cfg2 bash tools/gpu_env_ab2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/envab; mkdir -p $OUT
for rep in 1 2; do
for e in ${ENVS}; do
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --workload ${WL:-cfg2} ${BENCH_ARGS:-} > $OUT/run.json 2> $OUT/run.err || { echo "$e failed"; tail -3 $OUT/run.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/run.json'));s=d['stages_ms_per_step'];print('$e', d['ms_per_step'], d['value'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')), 'frac', d['roofline']['frac'], d['verified'][:5])"
done
done
