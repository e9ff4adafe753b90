# round-5 GPU iteration n: final build (handoffs): GPU suite, driver-length bench, cfg5, round profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench_drv.json 2> $O/bench_drv.err || { tail -30 $O/bench_drv.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_drv.json')); print('drv', round(d['value']/1e6,3), 'cold', round(d['cold_first_step']['value']/1e6,3), d['cold_first_step']['handoffs'], 'order', round(d['cold_order_step']['value']/1e6,3), min(d['kernel_ms_per_step']), max(d['kernel_ms_per_step']), d['plan_latency_ms'], d['parity_sample']['bit_exact'], d['parity_sample']['last_timed_step']['bit_exact'])"
timeout -k 10 600 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', d['tick_ms'], d['cpu_baseline']['tick_ms_16_threads'], d['parity_sample']['bit_exact'])"
bash tools/prof_round.sh r05n || exit 1
