# round-5 GPU iteration y: what bounds the cold step (its last-ending searches)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05y; mkdir -p $O
for i in 1 2; do
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/b_$i.json 2> $O/b_$i.err || { tail -30 $O/b_$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_$i.json')); c=d['cold_first_step']; print(round(d['value']/1e6,3), round(c['value']/1e6,3), round(c['ms']), c['handoffs'], d['step_balance']['pool']); [print(x) for x in c['last_to_end']]"
done
