#!/bin/bash
# Quick GPU check: smoke + the default bench line (+ optional extra workloads in $WL)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quick; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench.json; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
for wl in ${WL:-}; do
  timeout -k 10 500 python bench.py --workload $wl --no-cpu-baseline > $OUT/$wl.json 2> $OUT/$wl.err || { echo "$wl failed"; tail -3 $OUT/$wl.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/$wl.json'));print('$wl', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('stages_ms_per_step'), d.get('verified','')[:5])"
done
