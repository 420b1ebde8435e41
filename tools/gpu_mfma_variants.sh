#!/bin/bash
# Ablations of k_rs_mfma (FI_MFMA_VARIANT): resize-stage ms per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mvariants; mkdir -p $OUT
for v in ${VARIANTS:-0 1 2 3}; do
  FI_MFMA_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$v.json 2> $OUT/$v.err; rc=$?
  echo "variant $v rc=$rc $(python -c "import json;d=json.load(open('$OUT/$v.json'));print(d['stages_ms_per_step']['resize'])" 2>/dev/null)"
  [ $rc -le 1 ] || exit $rc
done
