#!/bin/bash
# k_rs_vr per-role stamps (MODE 9) on cfg2 and cfg3 geometries + bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stamps
mkdir -p $OUT
summ() { python3 -c "import json,sys; d=json.load(open('$1')); s=d['stages_ms_per_step']; print('$2', 'step', d['ms_per_step'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')), 'frac', d['roofline']['frac'], d.get('verified'))"; }
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/cfg2.json 2> $OUT/cfg2.err || exit 3
summ $OUT/cfg2.json cfg2
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload cfg3 --images 1024 > $OUT/cfg3.json 2> $OUT/cfg3.err || exit 3
summ $OUT/cfg3.json cfg3
timeout -k 10 200 python -u tools/vr_timing.py > $OUT/t2.log 2>&1 || exit 4
cat $OUT/t2.log
VP_W=3840 VP_H=2160 VP_OPTS=w_512,h_512,c_1 NIMG=1024 timeout -k 10 200 python -u tools/vr_timing.py > $OUT/t3.log 2>&1 || exit 4
cat $OUT/t3.log
