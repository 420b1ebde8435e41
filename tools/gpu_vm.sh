#!/bin/bash
# k_rs_vm iteration: vm-path parity tests, bench, ablation variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
if [ "${TESTK:-vm}" != none ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "${TESTK:-vm}" > $OUT/vm_test.log 2>&1; rc=$?
tail -4 $OUT/vm_test.log; [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/vm_bench.json 2> $OUT/vm_bench.err || exit 1
python -c "import json;d=json.load(open('$OUT/vm_bench.json'));print('value', d['value'], 'ms/step', d['ms_per_step'], d['stages_ms_per_step'], d['roofline']['frac'])"
for v in ${VARIANTS:-}; do
  FI_VM_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/vmv$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/vmv$v.json'));print('variant', $v, d['stages_ms_per_step']['resize'])"
done
