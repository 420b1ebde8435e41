#!/bin/bash
# A/B of one environment switch on the bench workload: runs with "$AB_ENV"
# (e.g. FI_VR_RS=0) exported (B) and without (A), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/envab
mkdir -p $OUT
for i in ${AB_ROUNDS-1 2 3}; do
  for v in A B; do
    if [ $v = B ]; then ENVV="$AB_ENV"; else ENVV=""; fi
    env $ENVV timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$v$i.json 2> $OUT/$v$i.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/$v$i.json')); s=d['stages_ms_per_step']; print('$v$i', 'step', d['ms_per_step'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')))"
  done
done
