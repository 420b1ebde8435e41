#!/bin/bash
# PMC passes for k_rs_vp on a reduced bench run (one pass per counter group),
# plus the counter list of this gfx950 box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_${TAG:-vp}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export FI_VP_RS=${FI_VP_RS:-1}
REGEX=${REGEX:-k_rs_vp}
ARGS=${PMC_BENCH_ARGS:---steps 1 --warmup 1 --no-cpu-baseline --no-verify}
[ -n "${LIST:-}" ] && { timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; grep -o "SQ_[A-Z_0-9]*" "$OUT/counters.txt" | sort -u | tr '\n' ' ' > "$OUT/sq_names.txt"; }
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$REGEX" --output-format csv -d "$OUT/$name" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.bench.json" 2> "$OUT/$name.err"; local rc=$?
  echo "pass $name rc=$rc"; return $rc
}
for spec in ${PASSES:-"sq:SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"}; do
  pass "${spec%%:*}" $(echo "${spec#*:}" | tr ',' ' ') || exit $?
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT"
