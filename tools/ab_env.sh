#!/bin/bash
# A/B of an environment switch on one workload: ENVS="A=1 A=0" (each a space-free VAR=VALUE list joined by ,)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
for rep in $(seq ${REPS:-1}); do
for e in $ENVS; do
  tag=$(echo $e | tr ',=' '__')
  env $(echo $e | tr ',' ' ') timeout -k 10 600 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup ${WARM:-3} ${WL:+--workload $WL} > $OUT/env_$tag.json 2> $OUT/env_$tag.err || { echo "$e failed"; tail -3 $OUT/env_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/env_$tag.json'));s=d['stages_ms_per_step'];print('$e', d['value'], d['ms_per_step'], 'resize', s['resize'], 'frac', d['roofline']['frac'], d['verified'][:5])"
done; done
