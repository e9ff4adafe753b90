# round-5 GPU iteration s: handoff threshold on the cold step of the deferred-tree build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05s; mkdir -p $O
for v in 32768 16384 8192 32768 16384 8192; do
  HASTAR_HANDOFF_POPS=$v timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/b_$v.json 2> $O/b_$v.err || { tail -30 $O/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', round(d['value']/1e6,3), 'cold', round(d['cold_first_step']['value']/1e6,3), d['cold_first_step']['handoffs'], 'order', round(d['cold_order_step']['value']/1e6,3))"
  cat $O/b_$v.json >> $O/sweep.jsonl
done
