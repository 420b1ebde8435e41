#!/bin/bash
# cfg4 under two environments back to back: ENV_A / ENV_B (e.g. ENV_B="FI_VR_MAX_CLASSES=100000")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c4ab; mkdir -p $OUT
for v in A B; do
  if [ $v = A ]; then e=${ENV_A:-}; else e=${ENV_B:-}; fi
  env $e timeout -k 10 400 python bench.py --workload cfg4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/$v.json 2> $OUT/$v.err || { echo "$v failed"; tail -3 $OUT/$v.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/$v.json'));s=d['stages_ms_per_step'];print('$v', '$e', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'][:160], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply','host_plan')), d['verified'][:5])"
done
