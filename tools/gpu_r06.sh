#!/bin/bash
# Round-6 iteration run (one gpurun call).  STEP selects what runs:
#   tests  : the new stream-ordering tests + the smartcrop / pipeline parity subset
#   bench  : cfg2 bench line (stage split) with FI_SC_FT=1 and =0
#   trace  : rocprofv3 kernel trace + stats of a short cfg2 bench
# default: tests bench trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r06; mkdir -p "$OUT"
for s in ${STEP:-tests bench trace}; do
  case $s in
  tests)
    timeout -k 10 500 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_parity.py -m gpu -x -q -rf \
      -k "${TESTK:-streams or smartcrop or score3 or pipelined or baseline_geometries}" \
      --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
    echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc ;;
  bench)
    for ft in 1 0; do
      FI_SC_FT=$ft timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-20} > "$OUT/bench_ft$ft.json" \
        2> "$OUT/bench_ft$ft.err"; rc=$?
      [ $rc -eq 0 ] || { echo "bench ft=$ft rc=$rc"; tail -5 "$OUT/bench_ft$ft.err"; exit $rc; }
      python3 -c "import json;d=json.load(open('$OUT/bench_ft$ft.json'));print('ft=$ft', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms_per_step'], d['smartcrop_kernels'], d['verified'][:5])"
    done ;;
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
