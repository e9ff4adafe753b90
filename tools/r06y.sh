# round-6 GPU iteration y: the final (hinted) build's cfg5 (20 ticks) and cfg4 (whole-batch parity) lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 900 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); c=d['cpu_baseline']; print('cfg5', d['steps'], round(d['tick_ms'],1), sorted([(round(s['ms']), s['pair']) for s in d['slowest_search_per_tick']])[-3:], 'cpu', round(c['tick_ms_one_core_per_pair'],1), d['parity_sample']['bit_exact'], d['parity_sample']['searches'], d['relaxed_mode']['tick_ms'])"
timeout -k 10 1100 python -u bench.py --workload cfg4 --parity-all > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -30 $O/bench_cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); print('cfg4', round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']], d['parity_sample']['bit_exact'], d['parity_all']['bit_exact'], d['parity_all']['queries'], d['parity_all']['path_poses_checked'])"
