#!/bin/bash
# rocprofv3 kernel statistics of each BASELINE configuration's bench run ->
# gpurun_out/prof_cfg/<workload>/ (kernel trace + stats only, no counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_cfg
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for w in ${WORKLOADS:-cfg1 cfg3 cfg5 cfg4}; do
  s=3; [ "$w" = cfg4 ] && s=1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$w" -o run -- \
    python3 "$ROOT/bench.py" --workload $w --steps $s --warmup 1 --no-cpu-baseline > "$OUT/$w.json" 2> "$OUT/$w.err" \
    || { echo "$w rc=$?"; tail -3 "$OUT/$w.err"; exit 3; }
  echo "$w ok"
done
