cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06; mkdir -p $OUT
for u in 1 0; do
FI_UP_SYNC=$u timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/up$u" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-verify > "$OUT/up$u.json" 2> "$OUT/up$u.err" || exit 1
python3 $GRAFT_REPO_ROOT/tools/trace_gaps.py "$OUT/up$u" > "$OUT/up$u.txt"
python3 - "$OUT/up$u.txt" $u <<'PY'
import sys, re
L=[l for l in open(sys.argv[1]) if 'k_synth' not in l and 'copyBuffer' not in l]
ev=[]
for l in L:
    m=re.match(r'\s*([\d.]+) \.\.\s*([\d.]+) us\s+([\d.]+) us\s+gap\s+(-?[\d.]+) us\s+(.*)', l)
    if m: ev.append((float(m.group(1)), float(m.group(2)), m.group(5)[:20]))
sc=[e for e in ev if 'k_sc_score3' in e[2]]; rs=[e for e in ev if 'k_rs_vr' in e[2]]
gaps=[]
for s in sc:
    nxt=[r[0] for r in rs if r[0] > s[1]]
    if nxt: gaps.append(min(nxt)-s[1])
print('FI_UP_SYNC', sys.argv[2], 'score3 end -> next k_rs_vr start (us):', [round(g,1) for g in gaps][2:])
PY
done
