# round-6 GPU iteration v: the final build (branch hints): GPU suite, smoke, driver-length bench
# with whole-batch parity, round profile (trace + PMC + SQ counters, hash-matched)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06v; mkdir -p $O
bash tools/gpu_iter.sh r06v test smoke || exit 1
timeout -k 10 1000 python -u bench.py --steps 20 --warmup 5 --parity-all > $O/bench_drv.json 2> $O/bench_drv.err || { tail -30 $O/bench_drv.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_drv.json')); print('drv', round(d['value']/1e6,3), 'cold', round(d['cold_first_step']['value']/1e6,3), 'order', round(d['cold_order_step']['value']/1e6,3), min(d['kernel_ms_per_step']), max(d['kernel_ms_per_step']), d['plan_latency_ms'], d['parity_sample']['bit_exact'], d['parity_sample']['last_timed_step']['bit_exact'], d['parity_all']['bit_exact'], d['parity_all']['queries'], d['parity_all']['path_poses_checked'])"
