# round-5 GPU iteration u: latency kernel's inner ring keeps f (rank queries without the index hop)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
for L in lib_pre lib lib_pre lib; do
  HASTAR_LIB=path_planning_pkg_amd/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --relaxed-batch 0 > $O/lat_$L.json 2> $O/lat_$L.err || { tail -20 $O/lat_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lat_$L.json')); print('$L latency', [round(x,1) for x in d['plan_latency_ms']['gpu']], d['longest_query']['gpu_ms_alone'])"
  cat $O/lat_$L.json >> $O/lat.jsonl
  HASTAR_LIB=path_planning_pkg_amd/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --workload cfg5 --no-cpu-baseline --no-relaxed > $O/cfg5_$L.json 2> $O/cfg5_$L.err || { tail -20 $O/cfg5_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg5_$L.json')); print('$L cfg5', round(d['tick_ms'],1), [(s['pair'], round(s['ms'])) for s in d['slowest_search_per_tick']])"
  cat $O/cfg5_$L.json >> $O/cfg5.jsonl
done
