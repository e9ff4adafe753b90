# round-5 GPU iteration r: final build (deferred inner tree): driver-length bench with whole-batch
# parity, cfg5, cfg4 with whole-batch parity, round profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 1000 python -u bench.py --steps 20 --warmup 5 --parity-all > $O/bench_drv.json 2> $O/bench_drv.err || { tail -30 $O/bench_drv.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_drv.json')); print('drv', round(d['value']/1e6,3), 'cold', round(d['cold_first_step']['value']/1e6,3), d['cold_first_step']['handoffs'], 'order', round(d['cold_order_step']['value']/1e6,3), min(d['kernel_ms_per_step']), max(d['kernel_ms_per_step']), d['plan_latency_ms'], d['parity_sample']['bit_exact'], d['parity_sample']['last_timed_step']['bit_exact'], {k: v for k, v in d['parity_all'].items() if k != 'note'})"
timeout -k 10 600 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', d['tick_ms'], d['cpu_baseline']['tick_ms_16_threads'], [(s['pair'], round(s['ms'])) for s in d['slowest_search_per_tick']], d['parity_sample']['bit_exact'])"
timeout -k 10 1100 python -u bench.py --workload cfg4 --parity-all > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -30 $O/bench_cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); print('cfg4', round(d['value']/1e6,3), d['parity_sample']['bit_exact'], {k: v for k, v in d['parity_all'].items() if k != 'note'})"
bash tools/prof_round.sh r05r || exit 1
