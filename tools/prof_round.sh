#!/bin/bash
# Round profile (run on the GPU box):  tools/prof_round.sh <tag>
#   1. bench.py under rocprofv3 --kernel-trace --stats  -> gpurun_out/<tag>/bench.json,
#      kernel_stats.csv, trace_summary.json (search-kernel dispatch durations)
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE) over the search kernel of a 1-step bench
#      -> gpurun_out/<tag>/pmc_search_summary.json
# Big raw traces stay in /tmp on the box.
set -o pipefail
TAG=${1:-prof}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
R=/tmp/rp_$TAG
rm -rf $R && mkdir -p $R
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/trace -o run -- python3 bench.py --warmup 2 --steps 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 tools/prof_summary.py trace $R/trace $OUT/trace_summary.json --warmup 2 --steps 3 || exit 1
find $R/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
# the PMC passes run the batch kernel alone (HASTAR_SPLIT=0: under counter collection the
# profiler serialises the split launch's two kernels, and a 1-step bench then ran > 3 min)
export HASTAR_SPLIT=0
B=$(python3 -c "import json;print(json.load(open('$OUT/bench.json'))['config']['queries_per_gpu'])")
for C in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
  n=${C%% *}
  timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv --kernel-include-regex hastar_search_kernel -d $R/$n -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $OUT/pmc_$n.log 2>&1 || { tail -5 $OUT/pmc_$n.log; exit 1; }
done
python3 tools/prof_summary.py pmc $R/FETCH_SIZE $R/WRITE_SIZE $OUT/pmc_search_summary.json --rdreq $R/TCC_EA0_RDREQ_sum --batch $B --grid 1024 || exit 1
cat $OUT/pmc_search_summary.json
# 3. SQ instruction mix / wait states of the batch kernel (one 1-step bench per pass)
for pass in "SQA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
            "SQB SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
            "SQC SQC_ICACHE_HITS SQC_ICACHE_MISSES TCC_HIT_sum TCC_MISS_sum"; do
  set -- $pass
  name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" --output-format csv --kernel-include-regex hastar_search_kernel -d $R/$name -o pmc \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $OUT/pmc_$name.log 2>&1 || { tail -5 $OUT/pmc_$name.log; exit 1; }
done
python3 tools/prof_summary.py counters $OUT/counters_search.json $R/SQA $R/SQB $R/SQC --batch $B --dispatch -1 || exit 1
