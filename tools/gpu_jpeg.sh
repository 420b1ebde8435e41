#!/bin/bash
# GPU JPEG decode throughput + rocprofv3 kernel stats -> gpurun_out/jpeg/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/jpeg
mkdir -p "$OUT"
timeout -k 10 300 python tools/jpeg_bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { cat "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/tools/jpeg_bench.py" > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || exit $?
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
