#!/bin/bash
# k_rs_vr second launch on a forked stream (FI_VR_FORK) A/B on cfg4 -> gpurun_out/fork/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fork; mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_vr.py tests/test_gpu_streams.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for f in ${FORKS:-0 1 0 1}; do
  FI_VR_FORK=$f timeout -k 10 400 python bench.py --workload cfg4 --steps 2 --warmup 1 --no-cpu-baseline \
    > $OUT/f$f.json 2> $OUT/f$f.err || { echo "fork $f rc=$?"; tail -3 $OUT/f$f.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/f$f.json'));s=d['stages_ms_per_step'];print('fork', $f, d['value'], d['ms_per_step'], d['roofline']['frac'], s.get('resize'), d.get('verified','')[:6])"
done
