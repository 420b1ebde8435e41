#!/bin/bash
# A/B of two library builds on the bench workload: tools/bin/libA.so (FI_LIB_PATH)
# vs the in-tree build, alternating, each run under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p $OUT
for i in ${AB_ROUNDS-1 2 3}; do
  for v in A B; do
    if [ $v = A ]; then export FI_LIB_PATH=$PWD/tools/bin/libA.so; else unset FI_LIB_PATH; fi
    timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$v$i.json 2> $OUT/$v$i.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/$v$i.json')); s=d['stages_ms_per_step']; print('$v$i', 'step', d['ms_per_step'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')))"
  done
done
