# round-5 GPU iteration o: every query of the cfg3 and cfg4 batches against the oracle
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 900 python -u bench.py --parity-all > $O/bench_cfg3_parity_all.json 2> $O/bench_cfg3_parity_all.err || { tail -30 $O/bench_cfg3_parity_all.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg3_parity_all.json')); print('cfg3', round(d['value']/1e6,3), {k: v for k, v in d['parity_all'].items() if k != 'note'})"
timeout -k 10 1100 python -u bench.py --workload cfg4 --parity-all > $O/bench_cfg4_parity_all.json 2> $O/bench_cfg4_parity_all.err || { tail -30 $O/bench_cfg4_parity_all.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg4_parity_all.json')); print('cfg4', round(d['value']/1e6,3), {k: v for k, v in d['parity_all'].items() if k != 'note'})"
