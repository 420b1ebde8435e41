#!/bin/bash
# Last check of the final tree: full GPU suite + smoke -> gpurun_out/final/,
# then two cfg4 lines -> gpurun_out/cfg4h/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final gpurun_out/cfg4h
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --durations=10 --timeout 300 --timeout-method thread \
  > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/final/smoke.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 600 python bench.py --workload cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg4h/q_$i.json 2> gpurun_out/cfg4h/q_$i.err || { echo "cfg4 rc=$?"; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/cfg4h/q_$i.json'));print('cfg4', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('verified','')[:6])"
done
