#!/bin/bash
# Round profile of the default bench: bench line, rocprofv3 kernel stats, PMC
# traffic (FETCH_SIZE / WRITE_SIZE passes) of the resample kernel -> gpurun_out/profile/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/profile
mkdir -p "$OUT"
KERNEL=${KERNEL:-k_rs_vm}
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/stats_bench.json" 2> "$OUT/stats.err" || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "$KERNEL" --output-format csv -d "$OUT/pmc_$c" -o run -- \
    python3 "$ROOT/bench.py" --steps 1 --warmup 1 --images 512 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err" || exit $?
done
python3 "$ROOT/tools/pmc_to_json.py" "$OUT" "$KERNEL" 512 "$OUT/traffic.json"
find "$OUT" -name "*kernel_stats.csv" | head -2
