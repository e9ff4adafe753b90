# round-6 GPU iteration ak: the cfg4 line of the final tree (map build local / row-sharded and the
# heuristic-field leg beside the search)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ak; mkdir -p $O
timeout -k 10 1000 python -u bench.py --workload cfg4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -30 $O/bench_cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); m=d['map_build']; print(round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']], d['parity_sample']['bit_exact'], m['parity'], round(m['local_ms_per_map'],2), round(m['sharded_ms_per_map'],2)); print(json.dumps(m['heuristic_field']))"
