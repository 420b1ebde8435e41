#!/bin/bash
# PMC passes (counters only + kernel trace; no sys/runtime trace) for the
# resample kernel (k_rs_vr by default) on a reduced bench run.  One pass per counter group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc/${PMC_TAG:-run}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
REGEX=${REGEX:-k_rs_vr}
ARGS=${PMC_BENCH_ARGS:---steps 1 --warmup 1 --images 512 --no-cpu-baseline}
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$REGEX" --output-format csv -d "$OUT/$name" -o run -- \
    python "$ROOT/bench.py" $ARGS > "$OUT/$name.bench.json" 2> "$OUT/$name.err"; local rc=$?
  echo "pass $name rc=$rc"; return $rc
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES || exit $?
pass fetch FETCH_SIZE || exit $?
pass write WRITE_SIZE TCC_HIT_sum || exit $?
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
ls "$OUT"
