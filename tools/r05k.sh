# round-5 GPU iteration k: handoff of long batch-kernel searches to free latency CUs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
HASTAR_HANDOFF_POPS=1024 timeout -k 10 600 python -u bench.py --steps 2 --warmup 2 --cpu-seconds 5 --latency-queries 1 > $O/bench_ho1024.json 2> $O/bench_ho1024.err || { tail -30 $O/bench_ho1024.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_ho1024.json')); print('ho1024', round(d['value']/1e6,3), d['cold_first_step']['handoffs'], d['step_balance']['handoffs'], d['parity_sample']['bit_exact'], d['parity_sample'].get('last_timed_step',{}).get('bit_exact'))"
for v in 32768 0 32768 0; do
  HASTAR_HANDOFF_POPS=$v timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --latency-queries 1 > $O/bench_ab_$v.json 2> $O/bench_ab_$v.err || { tail -30 $O/bench_ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_ab_$v.json')); print('$v', round(d['value']/1e6,3), 'cold', round(d['cold_first_step']['value']/1e6,3), d['cold_first_step']['handoffs'], 'order', round(d['cold_order_step']['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']], d['step_balance']['handoffs'])"
  cat $O/bench_ab_$v.json >> $O/ab.jsonl
done
