#!/bin/bash
# Two bench variants back to back, twice: ARGS_A / ARGS_B (e.g. ARGS_B=--timed-stages)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bab; mkdir -p $OUT
for rep in 1 2; do
for v in A B; do
  if [ $v = A ]; then a=${ARGS_A:-}; else a=${ARGS_B:-}; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline $a > $OUT/$v.json 2> $OUT/$v.err || { echo "$v failed"; tail -3 $OUT/$v.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/$v.json'));s=d['stages_ms_per_step'];print('$v', d['ms_per_step'], d['value'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')), d['verified'][:5])"
done
done
