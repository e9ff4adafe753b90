# round-5 GPU iteration aa: the cold step's tail with and without handoffs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05aa; mkdir -p $O
for v in 0 32768; do
HASTAR_HANDOFF_POPS=$v timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/b_$v.json 2> $O/b_$v.err || { tail -30 $O/b_$v.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/b_$v.json')); c=d['cold_first_step']
print('$v cold', round(c['ms']), c['handoffs']); [print('  ', x) for x in c['last_to_end'][:4]]"
done
