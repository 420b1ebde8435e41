#!/bin/bash
# k_rs_vs ablations (FI_VS_VARIANT, wrong pixels; timing only) on one workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vs_variants
mkdir -p $OUT
for v in ${VARIANTS:-0 1 2 3}; do
  FI_VS_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/v$v.json 2> $OUT/v$v.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/v$v.json')); print('variant $v', d['stages_ms_per_step']['resize'], d['ms_per_step'])"
done
