cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06; mkdir -p $OUT
for cx in ${CXS:-1 0}; do
FI_SC_CX=$cx timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace4_$cx" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload cfg4 --steps 1 --warmup 1 --no-cpu-baseline --no-verify > "$OUT/trace4_$cx.json" 2> "$OUT/trace4_$cx.err" || exit 1
f=$(find "$OUT/trace4_$cx" -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print('$cx', r['Name'][:50], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2), 'ms tot', round(float(r['MaxNs'])/1e3,1), 'us max')
"
done
