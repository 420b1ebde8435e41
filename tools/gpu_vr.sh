#!/bin/bash
# k_rs_vr bring-up on the GPU box: bitwise check against k_rs_vm, then cfg2 /
# cfg3 bench lines with k_rs_vr (FI_VR_RS=1) and k_rs_vm, optional stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vr
mkdir -p $OUT
timeout -k 10 200 python -u tools/vr_check.py > $OUT/check.log 2>&1
rc=$?
cat $OUT/check.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "${CHECK_ONLY:-}" ] && exit $rc
summ() { python3 -c "import json,sys; d=json.load(open('$1')); s=d['stages_ms_per_step']; print('$2', 'step', d['ms_per_step'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')), 'frac', d['roofline']['frac'], d.get('verified'))"; }
for v in ${VR_RUNS:-vr2 vm2 vr3 vm3}; do
  case $v in
    vr2) e="FI_VR_RS=1"; a="" ;;
    vm2) e="FI_VR_RS=0"; a="" ;;
    vr3) e="FI_VR_RS=1"; a="--workload cfg3 --images 1024" ;;
    vm3) e="FI_VR_RS=0"; a="--workload cfg3 --images 1024" ;;
    vr1) e="FI_VR_RS=1"; a="--workload cfg1" ;;
    vr5) e="FI_VR_RS=1"; a="--workload cfg5" ;;
  esac
  env $e timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $a > $OUT/$v.json 2> $OUT/$v.err || { echo "bench $v rc $?"; tail -5 $OUT/$v.err; exit 3; }
  summ $OUT/$v.json $v
done
if [ -n "${VR_TIMING:-}" ]; then
  timeout -k 10 200 python -u tools/vr_timing.py > $OUT/timing.log 2>&1; rc=$?; cat $OUT/timing.log; [ $rc -eq 0 ] || exit $rc
fi
