# round-6 GPU iteration p: the split-launch outlier with per-search shader clocks (experimental
# build path_planning_pkg_amd/lib_clk: s_memtime at each search's start and end in cycles[38..39];
# the stamps cost the latency kernel 3-4 %, so they stay out of the product build).  lib_clk is
# hastar_kernels.hip with tools/clk_stamps.patch applied, compiled as the Makefile does and linked
# with the product build's other objects.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06p; mkdir -p $O
export HASTAR_LIB=path_planning_pkg_amd/lib_clk/libhastar_amd.so
timeout -k 10 200 python tools/clk_probe.py || exit 1
for hc in 8 8 8; do
  HASTAR_HEAD_CUS=$hc timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --step-diag --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/bench_h$hc.json 2> $O/bench_h$hc.err || { tail -30 $O/bench_h$hc.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_h$hc.json')); print($hc, round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']])"
  cat $O/bench_h$hc.json >> $O/bench_h$hc.all.jsonl
done
