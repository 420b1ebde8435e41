#!/bin/bash
# Bench A/B of tools/bin/lib<A>.so against the tree's library, twice (FI_LIB_PATH)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lab; mkdir -p $OUT
for rep in 1 2; do
for v in ${LIB_A:-base} tree; do
  if [ $v = tree ]; then unset FI_LIB_PATH; else export FI_LIB_PATH=$PWD/tools/bin/lib$v.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$v.json 2> $OUT/$v.err || { echo "$v failed"; tail -3 $OUT/$v.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/$v.json'));s=d['stages_ms_per_step'];print('$v', d['ms_per_step'], d['value'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')), d['verified'][:5])"
done
done
