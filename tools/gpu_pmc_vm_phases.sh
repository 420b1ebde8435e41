#!/bin/bash
# LDS bank-conflict / LDS-wait counters of k_rs_vm per ablation (FI_VM_VARIANT,
# fi_vm.hip MODE): which phase the conflicts come from.  One pass per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_vm_phases
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-0 1 2 4 5}; do
  FI_VM_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex k_rs_vm --output-format csv -d "$OUT/v$v" -o run -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --images 512 --no-cpu-baseline > "$OUT/v$v.bench.json" 2> "$OUT/v$v.err" || { echo "variant $v failed"; exit 1; }
  echo "variant $v done"
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT"
