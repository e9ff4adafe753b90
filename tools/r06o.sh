# round-6 GPU iteration o: (1) the per-search shader-clock stamps cost nothing (A/B against the
# previous kernels: plan latency, cfg5); (2) the split-launch outlier: 20-step runs with 8 and 16
# latency CUs and per-step schedules, each head search's shader clock included
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06o; mkdir -p $O
P=path_planning_pkg_amd
for L in lib_prev lib lib_prev lib; do
  HASTAR_LIB=$P/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --relaxed-batch 0 > $O/lat_$L.json 2> $O/lat_$L.err || { tail -20 $O/lat_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lat_$L.json')); print('$L latency', [round(x,1) for x in d['plan_latency_ms']['gpu']], d['longest_query']['gpu_ms_alone'])"
done
for L in lib_prev lib; do
  HASTAR_LIB=$P/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-relaxed > $O/cfg5_$L.json 2> $O/cfg5_$L.err || { tail -20 $O/cfg5_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg5_$L.json')); print('$L cfg5 tick', round(d['tick_ms'],1))"
done
for hc in 8 16 8; do
  HASTAR_HEAD_CUS=$hc timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --step-diag --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/bench_h$hc.json 2> $O/bench_h$hc.err || { tail -30 $O/bench_h$hc.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_h$hc.json')); print($hc, round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']])"
  cat $O/bench_h$hc.json >> $O/bench_h$hc.all.jsonl
done
