#!/bin/bash
# k_rs_vm strip-width sweep (FI_VM_MAXNX) on a bench workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for nx in ${NXS:-32 48 64}; do
  FI_VM_MAXNX=$nx timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/nx$nx.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/nx$nx.json'));print('nx', $nx, 'value', d['value'], 'resize', d['stages_ms_per_step']['resize'], 'frac', d['roofline']['frac'])"
done
