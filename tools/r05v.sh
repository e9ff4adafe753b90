# round-5 GPU iteration v: latency CUs in the head vs the cold step (deferred-tree build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05v; mkdir -p $O
for h in 16 24 32 16 24 32; do
  HASTAR_HEAD_CUS=$h timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/h_$h.json 2> $O/h_$h.err || { tail -30 $O/h_$h.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/h_$h.json')); print('$h', round(d['value']/1e6,3), 'cold', round(d['cold_first_step']['value']/1e6,3), d['cold_first_step']['handoffs'], 'order', round(d['cold_order_step']['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']])"
  cat $O/h_$h.json >> $O/head.jsonl
done
