#!/bin/bash
# k_rs_vr LDS / issue counters on cfg2 (512 images), per FI_VR_VARIANT in $VARIANTS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_vr
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-0}; do
  export FI_VR_VARIANT=$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    --kernel-include-regex k_rs_vr --output-format csv -d "$OUT/v$v" -o run -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --images 512 --no-cpu-baseline --no-verify > "$OUT/v$v.json" 2> "$OUT/v$v.err" || { echo "pmc v$v rc=$?"; exit 5; }
  python3 - "$OUT/v$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
tot = collections.defaultdict(float); disp = set()
for r in rows:
    tot[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r.get("Dispatch_Id"))
n = max(1, len(disp))
print(sys.argv[1].split("/")[-1], "dispatches", n, " ".join(f"{k}={v/n:.4g}" for k, v in sorted(tot.items())))
PY
done
