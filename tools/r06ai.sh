# round-6 GPU iteration ai: the default bench line of the final tree (the driver's N=1 command
# shape), with the roofline's PMC traffic now matching the built sources' hash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ai; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print(round(d['value']/1e6,3), d['steps'], d['warmup'], round(r['achieved'],2), r['frac'], r['traffic'], d['plan_latency_ms']['gpu_median'], d['parity_sample']['bit_exact'])"
