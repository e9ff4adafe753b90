# round-5 GPU iteration ag: final build's cfg5 and cfg4 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05ag; mkdir -p $O
timeout -k 10 600 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); c=d['cpu_baseline']; print('cfg5', round(d['tick_ms'],1), [(s['pair'], round(s['ms'])) for s in d['slowest_search_per_tick']], 'cpu', round(c['tick_ms_one_core_per_pair'],1), [round(x) for x in c['tick_max_ms']], d['parity_sample']['bit_exact'], d['relaxed_mode']['tick_ms'])"
timeout -k 10 1100 python -u bench.py --workload cfg4 --parity-all > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -30 $O/bench_cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); print('cfg4', round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']], d['parity_sample']['bit_exact'], d['parity_all']['bit_exact'], d['parity_all']['queries'])"
