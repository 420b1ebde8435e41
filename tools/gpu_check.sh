#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test/assert failure, not a fault
STEPS=${STEPS:-all}
if [[ $STEPS == *all* || $STEPS == *test* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; ok $rc || exit $rc
fi
if [[ $STEPS == *all* || $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; ok $rc || exit $rc
fi
if [[ $STEPS == *all* || $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
  echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; ok $rc || exit $rc
fi
if [[ $STEPS == *all* || $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_bench.json" 2> "$OUT/prof.err"; rc=$?
  echo "rocprof rc=$rc"; tail -3 "$OUT/prof.err"
  find "$OUT/prof" -name "*stats*" | head
  exit $rc
fi
