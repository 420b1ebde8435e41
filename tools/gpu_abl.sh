#!/bin/bash
# Bench each tools/bin/lib<V>.so named in $LIBS (FI_LIB_PATH), one run each,
# printing the stage times -> gpurun_out/abl/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abl
mkdir -p $OUT
for v in ${LIBS}; do
  if [ $v = tree ]; then unset FI_LIB_PATH; else export FI_LIB_PATH=$PWD/tools/bin/lib$v.so; fi
  timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$v.json 2> $OUT/$v.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); s=d['stages_ms_per_step']; print('$v', 'step', d['ms_per_step'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')))"
done
