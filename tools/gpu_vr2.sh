#!/bin/bash
# k_rs_vr change check: its GPU tests, the resample parity tests, then cfg2 / cfg3 bench lines and stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vr2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vr.py tests/test_gpu_batch.py \
  tests/test_gpu_parity.py -k "${PYK:-vr or batch or baseline or resize or smartcrop or full_size}" \
  > $OUT/pytest.log 2>&1; rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys; d=json.load(open('$1')); s=d['stages_ms_per_step']; print('$2', 'step', d['ms_per_step'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')), 'frac', d['roofline']['frac'], d.get('verified'))"; }
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/cfg2.json 2> $OUT/cfg2.err || exit 3
summ $OUT/cfg2.json cfg2
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload cfg3 --images 1024 > $OUT/cfg3.json 2> $OUT/cfg3.err || exit 3
summ $OUT/cfg3.json cfg3
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload cfg1 > $OUT/cfg1.json 2> $OUT/cfg1.err || exit 3
summ $OUT/cfg1.json cfg1
[ -n "${STAMPS:-}" ] || exit 0
timeout -k 10 200 python -u tools/vr_timing.py > $OUT/t2.log 2>&1 || exit 4
cat $OUT/t2.log
