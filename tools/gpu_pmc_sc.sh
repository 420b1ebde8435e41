#!/bin/bash
# SQ counter pass (instruction mix, waits) for the smartcrop kernels on a
# reduced cfg2 bench run -> gpurun_out/pmc_sc/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_sc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
REGEX=${REGEX:-k_sc_|k_crop}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  --kernel-include-regex "$REGEX" --output-format csv -d "$OUT/sq" -o run -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 1 --images 512 --no-cpu-baseline > "$OUT/sq.bench.json" 2> "$OUT/sq.err" || exit $?
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
