#!/bin/bash
# SQ counters of the GPU JPEG decode kernels on a short jpeg_bench run -> gpurun_out/pmc_jpeg/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_jpeg
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
NIMG=${NIMG:-64} REPS=1 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  --kernel-include-regex "k_jpeg" --output-format csv -d "$OUT/sq" -o run -- \
  python3 "$ROOT/tools/jpeg_bench.py" > "$OUT/sq.json" 2> "$OUT/sq.err" || exit $?
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
