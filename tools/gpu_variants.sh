#!/bin/bash
# Resize-stage time of each profiling ablation of k_rs_vm (FI_VM_VARIANT) on
# the bench workload; each run under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/variants
mkdir -p $OUT
for v in ${VM_VARIANTS-0 1 2 3 4 5 6 7}; do
  FI_VM_VARIANT=$v timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/vm$v.json 2> $OUT/vm$v.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/vm$v.json')); print('vm variant $v resize', d['stages_ms_per_step']['resize'])"
done
