#!/bin/bash
# Round-end evidence in one GPU session -> gpurun_out/final/: parity tests,
# smoke, the default bench line, rocprofv3 kernel stats, PMC traffic of the
# dominant kernel, GPU JPEG decode and the end-to-end codec bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/final
mkdir -p "$OUT"
ok() { [ "$1" -eq 0 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; ok $rc || exit $rc
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "bench rc=$rc"; cat "$OUT/bench.json"; ok $rc || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/profile_bench.json" 2> "$OUT/prof.err"; rc=$?
echo "rocprof rc=$rc"; ok $rc || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "k_rs_vr" --output-format csv -d "$OUT/pmc_$c" -o run -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --images 512 --no-cpu-baseline > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err" || exit $?
done
python3 "$ROOT/tools/pmc_to_json.py" "$OUT" k_rs_vr 512 "$OUT/traffic_cfg2_k_rs_vr.json"
cd "$ROOT"
NIMG=1024 timeout -k 10 300 python tools/jpeg_bench.py > "$OUT/jpeg_bench.json" 2> "$OUT/jpeg_bench.err"; rc=$?
echo "jpeg rc=$rc"; cat "$OUT/jpeg_bench.json"; ok $rc || exit $rc
timeout -k 10 300 python tools/codec_bench.py --images 512 --batch 128 > "$OUT/codec_bench.json" 2> "$OUT/codec_bench.err"; rc=$?
echo "codec rc=$rc"; cat "$OUT/codec_bench.json"
exit $rc
