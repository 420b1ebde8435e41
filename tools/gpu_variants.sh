#!/bin/bash
# Ablation runs of the fused resample kernel (FI_FUSED_VARIANT), one process each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/variants; mkdir -p $OUT
for v in ${VARIANTS:-base d16 noepi noflops}; do
  FI_FUSED_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$v.json 2> $OUT/$v.err; rc=$?
  echo "$v rc=$rc $(python -c "import json;d=json.load(open('$OUT/$v.json'));print(d['stages_ms_per_step'], d['value'])" 2>/dev/null)"
  [ $rc -le 1 ] || exit $rc
done
