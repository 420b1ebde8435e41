#!/bin/bash
# bench cfg4's host side (prebuilt descriptor arrays, column-wise records):
# the stream / gather GPU tests, then cfg4 lines -> gpurun_out/cfg4h/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cfg4h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 600 python bench.py --workload cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/cfg4_$i.json 2> $OUT/cfg4_$i.err || { echo "cfg4 rc=$?"; tail -3 $OUT/cfg4_$i.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/cfg4_$i.json'));s=d['stages_ms_per_step'];print('cfg4', d['value'], d['ms_per_step'], d['roofline']['frac'], s['resize'], s['host_wait'], d.get('verified','')[:6])"
done
