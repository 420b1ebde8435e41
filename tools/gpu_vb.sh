#!/bin/bash
# k_rs_vs iteration loop on the GPU box: smoke, vs-path parity tests, phase
# stamps, bench (each step under its own limit; a fault ends the script).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vs1
mkdir -p $OUT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
FI_VB_RS=1 timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "${PYK:-vb}" --timeout 120 --timeout-method thread > $OUT/pytest_vs.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/pytest_vs.log; ok $rc || exit $rc
timeout -k 10 300 python -u tools/vb_timing.py > $OUT/timing.log 2>&1; rc=$?
echo "timing rc=$rc"; cat $OUT/timing.log; ok $rc || exit $rc
FI_VB_RS=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['stages_ms_per_step'])"
