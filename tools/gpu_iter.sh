#!/bin/bash
# One GPU iteration on the box:  tools/gpu_iter.sh <tag> <stage>...   (stops at the first failure)
#   test      pytest -m gpu (the parity suite, through the C-ABI)      -> gpurun_out/<tag>/pytest_gpu.txt
#   smoke     __graft_entry__.smoke()                                   -> smoke.txt
#   bench     python bench.py (defaults: cfg3, the headline line)       -> bench.json
#   benchlong bench.py --steps 8 --step-diag (per-step kernel times and schedules), no CPU/latency/relaxed legs -> bench_long.json
#   benchlong0 the same with HASTAR_SPLIT=0 (no latency CUs)   -> bench_long_nosplit.json
#   benchdrv  bench.py --steps 20 --warmup 5 (the driver's command line)  -> bench_drv.json
#   headcus   16-step benches: split mode 1 / 2 with 8 head CUs, mode 1 with 16 -> bench_mode*_head*.json
#   head20    20-step benches alternating 8 and 16 latency CUs (x2)  -> bench_h{8,16}.all.jsonl
#   cfg4      bench.py --workload cfg4                              -> bench_cfg4.json
#   cfg5      bench.py --workload cfg5                                  -> bench_cfg5.json
#   stamps    single-query phase stamps (lib_stamps build) of the bench's longest query and seed 1
#   prof      tools/prof_round.sh <tag>: rocprofv3 trace + PMC passes   -> trace_summary.json, pmc_*, counters_*
#   single    tools/prof_single.sh <tag> 1 3: SQ instruction mix of single queries on the latency kernel
#   relaxed   tools/gpu_relaxed.sh <tag>: relaxed-mode GPU tests + settings sweep  -> pytest.log, sweep.json
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p $O
for st in "$@"; do
  echo "== $st"
  case $st in
    test)  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
             || { tail -40 $O/pytest_gpu.txt; exit 1; }; tail -2 $O/pytest_gpu.txt ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
           tail -1 $O/smoke.txt ;;
    bench) timeout -k 10 900 python -u bench.py --dump-timings $O/timings.npz > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
           cut -c1-400 $O/bench.json ;;
    benchlong) timeout -k 10 900 python -u bench.py --steps 8 --warmup 1 --step-diag --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/bench_long.json 2> $O/bench_long.err || { tail -30 $O/bench_long.err; exit 1; }
           python -c "import json,sys; d=json.load(open('$O/bench_long.json')); print(d['value'], d['kernel_ms_per_step'])" ;;
    benchlong0) HASTAR_SPLIT=0 timeout -k 10 900 python -u bench.py --steps 8 --warmup 1 --step-diag --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/bench_long_nosplit.json 2> $O/bench_long_nosplit.err || { tail -30 $O/bench_long_nosplit.err; exit 1; }
           python -c "import json,sys; d=json.load(open('$O/bench_long_nosplit.json')); print(d['value'], d['kernel_ms_per_step'])" ;;
    benchdrv) timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --dump-timings $O/timings_drv.npz > $O/bench_drv.json 2> $O/bench_drv.err || { tail -30 $O/bench_drv.err; exit 1; }
           cut -c1-400 $O/bench_drv.json ;;
    headcus) for cfg in "1 8" "2 8" "1 16"; do set -- $cfg
             HASTAR_SPLIT_MODE=$1 HASTAR_HEAD_CUS=$2 timeout -k 10 600 python -u bench.py --steps 16 --warmup 2 --step-diag --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/bench_mode$1_head$2.json 2> $O/bench_mode$1_head$2.err || { tail -30 $O/bench_mode$1_head$2.err; exit 1; }
             python -c "import json; d=json.load(open('$O/bench_mode$1_head$2.json')); print('mode $1 head $2', d['value'], [round(k) for k in d['kernel_ms_per_step']])"; done ;;
    head20) for hc in 8 16 8 16; do HASTAR_HEAD_CUS=$hc timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --step-diag --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/bench_h$hc.json 2> $O/bench_h$hc.err || { tail -30 $O/bench_h$hc.err; exit 1; }
             python -c "import json; d=json.load(open('$O/bench_h$hc.json')); print($hc, d['value'], [round(k) for k in d['kernel_ms_per_step']])"; cat $O/bench_h$hc.json >> $O/bench_h$hc.all.jsonl; done ;;
    cfg4)  timeout -k 10 900 python -u bench.py --workload cfg4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -30 $O/bench_cfg4.err; exit 1; }
           cut -c1-400 $O/bench_cfg4.json ;;
    cfg5)  timeout -k 10 600 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
           cut -c1-400 $O/bench_cfg5.json ;;
    stamps) HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 300 python -u tools/profile_search.py --seeds 2396 1 2 3 > $O/stamps.jsonl 2>&1 \
             || { tail -20 $O/stamps.jsonl; exit 1; }; cut -c1-300 $O/stamps.jsonl ;;
    prof)  bash tools/prof_round.sh $TAG || exit 1 ;;
    single) bash tools/prof_single.sh $TAG 1 3 || exit 1 ;;
    relaxed) bash tools/gpu_relaxed.sh $TAG || exit 1 ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
