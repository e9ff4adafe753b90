# round-5 GPU iteration x: cfg5 with the CPU tick over the same timed ticks; smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); c=d['cpu_baseline']; print('cfg5', round(d['tick_ms'],1), [(s['pair'], round(s['ms'])) for s in d['slowest_search_per_tick']], 'cpu', round(c['tick_ms_one_core_per_pair'],1), [round(x) for x in c['tick_max_ms']], round(c['tick_ms_16_threads'],1), d['parity_sample']['bit_exact'])"
