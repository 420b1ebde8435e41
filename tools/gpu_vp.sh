#!/bin/bash
# k_rs_vp bring-up on the GPU box: bitwise check against k_rs_vm, then the
# cfg2 bench with k_rs_vp, k_rs_vm and the k_rs_vp ablations (FI_VP_VARIANT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vp
mkdir -p $OUT
timeout -k 10 150 python -u tools/vp_check.py > $OUT/check.log 2>&1
rc=$?
cat $OUT/check.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
summ() { python3 -c "import json,sys; d=json.load(open('$1')); s=d['stages_ms_per_step']; print('$2', 'step', d['ms_per_step'], ' '.join(f'{k} {s[k]}' for k in ('resize','sc_prep','sc_score','crop_apply')), 'frac', d['roofline']['frac'])"; }
for v in ${VP_RUNS:-vp vm a1 a2 vp}; do
  case $v in
    vp) e="FI_VP_RS=1" ;;
    vm) e="FI_VP_RS=0" ;;
    a1) e="FI_VP_RS=1 FI_VP_VARIANT=1" ;;
    a2) e="FI_VP_RS=1 FI_VP_VARIANT=2" ;;
    a3) e="FI_VP_RS=1 FI_VP_VARIANT=3" ;;
    a4) e="FI_VP_RS=1 FI_VP_VARIANT=4" ;;
    a5) e="FI_VP_RS=1 FI_VP_VARIANT=5" ;;
    a6) e="FI_VP_RS=1 FI_VP_VARIANT=6" ;;
  esac
  nv=""; case $v in a*) nv="--no-verify" ;; esac
  env $e timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $nv ${BENCH_ARGS:-} > $OUT/$v.json 2> $OUT/$v.err || { echo "bench $v rc $?"; tail -5 $OUT/$v.err; exit 3; }
  summ $OUT/$v.json $v
done
if [ -n "${VP_TIMING:-}" ]; then
  timeout -k 10 200 python -u tools/vp_timing.py > $OUT/timing.log 2>&1; rc=$?; cat $OUT/timing.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${VP_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread $VP_TESTS > $OUT/tests.log 2>&1
  rc=$?; tail -15 $OUT/tests.log; exit $rc
fi
