#!/bin/bash
# HBM traffic (rocprofv3 PMC FETCH_SIZE and WRITE_SIZE, one pass each, kernel
# filter on the resize kernel) per BASELINE configuration ->
# gpurun_out/pmc_cfg/traffic_<workload>_<kernel>.json (bench.py reads the
# committed copies under profiles/ for roofline.traffic).
#   WORKLOADS="cfg2 cfg1 cfg3 cfg5" KERNEL=k_rs_vr bash tools/gpu_pmc_configs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_cfg
mkdir -p "$OUT"
K=${KERNEL:-k_rs_vr}
cd /tmp && export TMPDIR=/tmp
for w in ${WORKLOADS:-cfg2 cfg1 cfg3 cfg5}; do
  n=512; [ "$w" = cfg3 ] && n=1024
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "$K" --output-format csv -d "$OUT/${w}_$c" -o run -- \
      python3 "$ROOT/bench.py" --workload $w --steps 1 --warmup 1 --images $n --no-cpu-baseline \
      > "$OUT/${w}_$c.json" 2> "$OUT/${w}_$c.err" || { echo "$w $c rc=$?"; tail -3 "$OUT/${w}_$c.err"; exit 3; }
  done
  mkdir -p "$OUT/$w" && mv "$OUT/${w}_FETCH_SIZE" "$OUT/${w}_WRITE_SIZE" "$OUT/$w/"
  python3 "$ROOT/tools/pmc_to_json.py" "$OUT/$w" $K $n "$OUT/traffic_${w}_$K.json" || exit 4
done
