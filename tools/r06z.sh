# round-6 GPU iteration z: compiler-flag sweep of the kernels object (tools/flag_variants.sh):
# short cfg3 benches alternating with the main build, then plan latency per build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06z; mkdir -p $O
P=path_planning_pkg_amd
V="$*"
L="$P/lib"; for v in $V; do L="$L $P/lib_$v"; done
bash tools/ab_bench.sh r06z $L || exit 1
for l in lib $(for v in $V; do echo lib_$v; done); do
  HASTAR_LIB=$P/$l/libhastar_amd.so timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --relaxed-batch 0 > $O/lat_$l.json 2> $O/lat_$l.err || { tail -20 $O/lat_$l.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lat_$l.json')); print('$l latency', [round(x,1) for x in d['plan_latency_ms']['gpu']], d['longest_query']['gpu_ms_alone'])"
done
bash tools/ab_bench.sh r06z2 $L || exit 1
