#!/bin/bash
# Kernel + memory-copy trace of a short bench run (no PMC): per-step timeline
# gaps between batches (tools/trace_gaps.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/trace
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT" -o run -- \
  python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
python "$ROOT/tools/trace_gaps.py" "$OUT"
