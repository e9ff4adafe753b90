# round-5 GPU iteration z: warm-step head durations (step_diag) beside the cold step's tail
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --step-diag --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/b.json 2> $O/b.err || { tail -30 $O/b.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/b.json')); c=d['cold_first_step']
print('cold', round(c['ms']), c['last_to_end'][:3])
for s in d['step_diag']:
    print('warm span', round(s['span_ms']), 'longest', s['longest'][:6])
    for r in sorted(s['head'], key=lambda r: -r[1])[:6]: print('  head', r[:6])
"
