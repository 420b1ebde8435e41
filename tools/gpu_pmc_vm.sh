#!/bin/bash
# PMC passes for one kernel (REGEX) on a reduced bench run; one pass per counter group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_${TAG:-vm}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
REGEX=${REGEX:-k_rs_vm}
ARGS=${PMC_BENCH_ARGS:---steps 1 --warmup 1 --images 512 --no-cpu-baseline}
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$REGEX" --output-format csv -d "$OUT/$name" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.bench.json" 2> "$OUT/$name.err"; local rc=$?
  echo "pass $name rc=$rc"; return $rc
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS || exit $?
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
pass fetch FETCH_SIZE || exit $?
pass write WRITE_SIZE || exit $?
python3 "$ROOT/tools/pmc_summary.py" "$OUT"
