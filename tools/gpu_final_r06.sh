#!/bin/bash
# Round-6 final evidence, in up to three gpurun calls (each under the 1200 s limit):
#   PART=1: full GPU tests + smoke, then PMC traffic (FETCH_SIZE / WRITE_SIZE,
#           separate passes) of k_rs_vr on cfg2 / cfg3 / cfg1 / cfg5 and of the
#           smartcrop prescale k_sc_fd on cfg2, plus one SQ pass on k_sc_fd
#           -> gpurun_out/final/ (copy traffic_*.json into profiles/ before
#           PART=2, so the bench lines report them)
#   PART=3: the cfg4 PMC passes (every resample kernel) -> traffic_cfg4_resize.json
#   PART=4: cfg4's kernel stats and bench line alone
#   PART=2: rocprofv3 kernel stats of cfg2 / cfg3 / cfg4 / cfg5, the default
#           bench line, the cfg1 / cfg3 / cfg4 / cfg5 lines -> gpurun_out/final/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/final
mkdir -p "$OUT"
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --durations=10 --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
  cd /tmp && export TMPDIR=/tmp
  for wl in cfg2 cfg3 cfg1 cfg5; do
    n=512; [ $wl = cfg3 ] && n=256
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "k_rs_vr" --output-format csv -d "$OUT/pmc_${wl}/$c" -o run -- \
        python3 "$ROOT/bench.py" --workload $wl --steps 1 --warmup 1 --images $n --no-cpu-baseline \
        > "$OUT/pmc_${wl}_$c.json" 2> "$OUT/pmc_${wl}_$c.err" || { echo "pmc $wl $c rc=$?"; exit 5; }
    done
    python3 "$ROOT/tools/pmc_to_json.py" "$OUT/pmc_$wl" k_rs_vr $n "$OUT/traffic_${wl}_k_rs_vr.json" || exit 4
    echo "pmc $wl ok"
  done
  # the smartcrop prescale: HBM traffic and one SQ pass
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "k_sc_fd" --output-format csv -d "$OUT/pmc_sc/$c" -o run -- \
      python3 "$ROOT/bench.py" --steps 1 --warmup 1 --images 512 --no-cpu-baseline \
      > "$OUT/pmc_sc_$c.json" 2> "$OUT/pmc_sc_$c.err" || { echo "pmc sc $c rc=$?"; exit 5; }
  done
  python3 "$ROOT/tools/pmc_to_json.py" "$OUT/pmc_sc" k_sc_fd 512 "$OUT/traffic_cfg2_k_sc_fd.json" || exit 4
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM \
    --kernel-include-regex "k_sc_fd" --output-format csv -d "$OUT/pmc_sc_sq" -o run -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --images 512 --no-cpu-baseline \
    > "$OUT/pmc_sc_sq.json" 2> "$OUT/pmc_sc_sq.err" || { echo "pmc sc sq rc=$?"; exit 5; }
  python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmc_sc_sq" > "$OUT/pmc_k_sc_fd_cfg2.txt"
  echo "pmc sc ok"
  cd "$ROOT"
fi
if [ "${PART:-1}" = 3 ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 500 rocprofv3 --pmc $c --kernel-include-regex "k_rs_" --output-format csv -d "$OUT/pmc_cfg4/$c" -o run -- \
      python3 "$ROOT/bench.py" --workload cfg4 --steps 1 --warmup 1 --no-cpu-baseline --no-verify \
      > "$OUT/pmc_cfg4_$c.json" 2> "$OUT/pmc_cfg4_$c.err" || { echo "pmc cfg4 $c rc=$?"; exit 5; }
  done
  # every resample dispatch of the warm-up and the timed step: 2 x the shard
  n4=$(python3 -c "import json; d=json.load(open('$OUT/pmc_cfg4_FETCH_SIZE.json')); print(2 * d['shard_images'][0])")
  python3 "$ROOT/tools/pmc_to_json.py" "$OUT/pmc_cfg4" k_rs_ total:$n4 "$OUT/traffic_cfg4_resize.json" || exit 4
  echo "pmc cfg4 ok ($n4 images)"
  cd "$ROOT"
fi
if [ "${PART:-1}" = 4 ]; then
  # cfg4 alone (after the bench's batch size changed): kernel stats + the line
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg4" -o run -- \
    python3 "$ROOT/bench.py" --workload cfg4 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_cfg4.json" 2> "$OUT/prof_cfg4.err" || exit 6
  cd "$ROOT"
  timeout -k 10 900 python bench.py --workload cfg4 --steps 1 --warmup 1 > "$OUT/cfg4.json" 2> "$OUT/cfg4.err" || { echo "cfg4 failed"; tail -3 "$OUT/cfg4.err"; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/cfg4.json'));print('cfg4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('verified','')[:5])"
fi
if [ "${PART:-1}" = 2 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_cfg2.json" 2> "$OUT/prof_cfg2.err" || exit 6
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- \
    python3 "$ROOT/bench.py" --workload cfg3 --steps 6 --warmup 2 --no-cpu-baseline > "$OUT/prof_cfg3.json" 2> "$OUT/prof_cfg3.err" || exit 6
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg4" -o run -- \
    python3 "$ROOT/bench.py" --workload cfg4 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_cfg4.json" 2> "$OUT/prof_cfg4.err" || exit 6
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg5" -o run -- \
    python3 "$ROOT/bench.py" --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_cfg5.json" 2> "$OUT/prof_cfg5.err" || exit 6
  echo "rocprof ok"
  cd "$ROOT"
  python3 tools/trace_gaps.py "$OUT/prof_cfg2" > "$OUT/timeline_cfg2.txt" || true
  timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
  echo "bench rc=$rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
  for wl in cfg1 cfg3 cfg5; do
    timeout -k 10 600 python bench.py --workload $wl > "$OUT/$wl.json" 2> "$OUT/$wl.err" || { echo "$wl failed"; tail -3 "$OUT/$wl.err"; exit 3; }
    python3 -c "import json;d=json.load(open('$OUT/$wl.json'));print('$wl', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('verified','')[:5])"
  done
  timeout -k 10 900 python bench.py --workload cfg4 --steps 1 --warmup 1 > "$OUT/cfg4.json" 2> "$OUT/cfg4.err" || { echo "cfg4 failed"; tail -3 "$OUT/cfg4.err"; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/cfg4.json'));print('cfg4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('verified','')[:5])"
fi
