#!/bin/bash
# Round evidence on the current tree -> gpurun_out/ev/: full GPU tests, smoke, the
# default bench line (CPU baseline), rocprofv3 kernel stats of the bench, PMC
# traffic of k_rs_vr on cfg2 / cfg3 (separate FETCH_SIZE / WRITE_SIZE passes),
# the other configs' bench lines.  STAGES selects steps (default all).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/ev
mkdir -p "$OUT"
want() { [ -z "${STAGES:-}" ] || [[ " $STAGES " == *" $1 "* ]]; }
if want tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if want bench; then
  timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
  echo "bench rc=$rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
fi
if want prof; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/profile_bench.json" 2> "$OUT/prof.err"; rc=$?
  echo "rocprof cfg2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof3" -o run -- \
    python3 "$ROOT/bench.py" --workload cfg3 --steps 6 --warmup 2 --no-cpu-baseline > "$OUT/profile_bench3.json" 2> "$OUT/prof3.err"; rc=$?
  echo "rocprof cfg3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$ROOT"
fi
if want pmc; then
  cd /tmp && export TMPDIR=/tmp
  for wl in cfg2 cfg3; do
    n=512; [ $wl = cfg3 ] && n=256
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "k_rs_vr" --output-format csv -d "$OUT/pmc_${wl}_$c" -o run -- \
        python3 "$ROOT/bench.py" --workload $wl --steps 1 --warmup 1 --images $n --no-cpu-baseline > "$OUT/pmc_${wl}_$c.json" 2> "$OUT/pmc_${wl}_$c.err" || exit $?
    done
    mkdir -p "$OUT/pmc_$wl"; cp -r "$OUT"/pmc_${wl}_FETCH_SIZE "$OUT"/pmc_${wl}_WRITE_SIZE "$OUT/pmc_$wl/"
    python3 "$ROOT/tools/pmc_to_json.py" "$OUT/pmc_$wl" k_rs_vr $n "$OUT/traffic_${wl}_k_rs_vr.json"
  done
  cd "$ROOT"
fi
if want configs; then
  for wl in cfg1 cfg3 cfg5; do
    timeout -k 10 600 python bench.py --workload $wl > "$OUT/$wl.json" 2> "$OUT/$wl.err" || { echo "$wl failed"; tail -3 "$OUT/$wl.err"; exit 3; }
    python3 -c "import json;d=json.load(open('$OUT/$wl.json'));print('$wl', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('verified','')[:5])"
  done
  timeout -k 10 900 python bench.py --workload cfg4 --steps 1 --warmup 1 > "$OUT/cfg4.json" 2> "$OUT/cfg4.err" || { echo "cfg4 failed"; tail -3 "$OUT/cfg4.err"; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/cfg4.json'));print('cfg4', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('verified','')[:5])"
fi
