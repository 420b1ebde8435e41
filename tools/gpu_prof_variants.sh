#!/bin/bash
# rocprofv3 kernel-trace stats of bench runs with the k_rs_mfma ablations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-0 3}; do
  FI_MFMA_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/pv$v" -o run -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/pv$v.json" 2> "$ROOT/gpurun_out/pv$v.err" || exit $?
  python3 - "$ROOT/gpurun_out/pv$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:50]:50s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:9.1f} us")
PY
done
