# round-5 GPU iteration ad: issue priority of the queue head (HASTAR_PRIO_N) on the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05ad; mkdir -p $O
for p in 242 0 1000 242 0 1000; do
  HASTAR_PRIO_N=$p timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/p_$p.json 2> $O/p_$p.err || { tail -30 $O/p_$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/p_$p.json')); print('$p', round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']], 'busy', round(d['step_balance']['slot_busy_mean_ms']), 'longest', round(d['step_balance']['longest_search_under_load_ms']))"
  cat $O/p_$p.json >> $O/prio.jsonl
done
