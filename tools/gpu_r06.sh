#!/bin/bash
# Round-6 iteration run (one gpurun call).  STEP selects what runs:
#   tests  : the new stream-ordering tests + the smartcrop / pipeline parity subset
#   bench  : cfg2 bench line (stage split) with FI_SC_CX=1 and =0 (CXS)
#   trace  : rocprofv3 kernel trace + stats of a short cfg2 bench
# default: tests bench trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r06; mkdir -p "$OUT"
for s in ${STEP:-tests bench trace}; do
  case $s in
  full)
    rm -f "$OUT/exact.tsv"
    FI_EXACT_LOG="$OUT/exact.tsv" timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --durations=25 \
      --timeout 300 --timeout-method thread > "$OUT/pytest_full.log" 2>&1; rc=$?
    echo "pytest full rc=$rc"; tail -30 "$OUT/pytest_full.log" | grep -E "passed|failed|s call" | head -30
    [ $rc -eq 0 ] || exit $rc ;;
  tests)
    timeout -k 10 500 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_parity.py -m gpu -x -q -rf \
      -k "${TESTK:-streams or smartcrop or score3 or pipelined or baseline_geometries}" \
      --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
    echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc ;;
  bench)
    # FI_SC_CX=1: smartcrop prescale beside the next resample (default); 0: k_sc_fd serial
    for cx in ${CXS:-1 0}; do
      FI_SC_CX=$cx timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-20} ${WL:+--workload $WL} \
        > "$OUT/bench_cx$cx.json" 2> "$OUT/bench_cx$cx.err"; rc=$?
      [ $rc -eq 0 ] || { echo "bench cx=$cx rc=$rc"; tail -5 "$OUT/bench_cx$cx.err"; exit $rc; }
      python3 -c "import json;d=json.load(open('$OUT/bench_cx$cx.json'));print('cx=$cx', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms_per_step'], d['smartcrop_kernels'], d['verified'][:5])"
    done ;;
  cfg4)
    timeout -k 10 600 python bench.py --workload cfg4 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/cfg4.json" \
      2> "$OUT/cfg4.err"; rc=$?
    [ $rc -eq 0 ] || { echo "cfg4 rc=$rc"; tail -5 "$OUT/cfg4.err"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/cfg4.json'));print('cfg4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified'][:5]); print({k: v for k, v in d['stages_ms_per_step'].items() if k.startswith('host') or k in ('resize','sc_prep','sc_score','batch')})" ;;
  trace)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-verify > "$OUT/trace.json" 2> "$OUT/trace.err"; rc=$?
    cd "$ROOT"
    [ $rc -eq 0 ] || { echo "trace rc=$rc"; tail -5 "$OUT/trace.err"; exit $rc; }
    f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
" ;;
  esac
done
