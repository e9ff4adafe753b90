# round-5 GPU iteration w: the always-on deferral as a constant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05ae; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
bash tools/ab_bench.sh r05ae path_planning_pkg_amd/lib_pre path_planning_pkg_amd/lib path_planning_pkg_amd/lib_pre path_planning_pkg_amd/lib || exit 1
for L in lib_pre lib; do
  HASTAR_LIB=path_planning_pkg_amd/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --relaxed-batch 0 > $O/lat_$L.json 2> $O/lat_$L.err || { tail -20 $O/lat_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lat_$L.json')); print('$L latency', [round(x,1) for x in d['plan_latency_ms']['gpu']], d['longest_query']['gpu_ms_alone'])"
done
