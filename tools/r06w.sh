# round-6 GPU iteration w: hints by measured branch frequency (lib_hint5: no hint on the insert branch, the closed re-pop unlikely) against the hinted build (lib)
# (lib): cfg3 short benches alternating, plan latency, 5-tick cfg5
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06w; mkdir -p $O
P=path_planning_pkg_amd
bash tools/ab_bench.sh r06w $P/lib $P/lib_hint5 $P/lib $P/lib_hint5 || exit 1
for L in lib lib_hint5 lib lib_hint5; do
  HASTAR_LIB=$P/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --relaxed-batch 0 > $O/lat_$L.json 2> $O/lat_$L.err || { tail -20 $O/lat_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lat_$L.json')); print('$L latency', [round(x,1) for x in d['plan_latency_ms']['gpu']], d['longest_query']['gpu_ms_alone'])"
done
for L in lib lib_hint5; do
  HASTAR_LIB=$P/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-relaxed > $O/cfg5_$L.json 2> $O/cfg5_$L.err || { tail -20 $O/cfg5_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg5_$L.json')); print('$L cfg5 tick', round(d['tick_ms'],1))"
done
