#!/bin/bash
# Round-2 profile (run on the GPU box):  tools/prof_r02.sh <tag>
#   1. bench.py (defaults) under rocprofv3 --kernel-trace --stats -> bench.json, kernel_stats.csv,
#      trace_summary.json (search-kernel dispatch durations of the timed steps)
#   2. separate --pmc passes over a 1-step bench (timed dispatch = index 1): FETCH_SIZE, WRITE_SIZE,
#      two SQ passes, one TCC pass -> pmc_search_summary.json, counters_search.json
set -o pipefail
TAG=${1:-prof}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
R=/tmp/rp_$TAG
rm -rf $R && mkdir -p $R
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/trace -o run -- python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 tools/prof_summary.py trace $R/trace $OUT/trace_summary.json --warmup 1 --steps 3 || exit 1
find $R/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
B=$(python3 -c "import json;print(json.load(open('$OUT/bench.json'))['config']['queries_per_gpu'])")
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --latency-queries 0"
timeout -s KILL 120 rocprofv3 -L > $OUT/avail_counters.txt 2>&1 || true
pass() {  # pass <name> <counters...>: counters this device does not list are dropped
  local name=$1; shift
  local use=()
  for c in "$@"; do
    base=${c%_sum}
    if grep -qw "$base" $OUT/avail_counters.txt; then use+=("$c"); else echo "  (counter $c not listed: skipped)"; fi
  done
  [ ${#use[@]} -eq 0 ] && return 0
  echo "pmc pass $name: ${use[*]}"
  timeout -s KILL 400 rocprofv3 --pmc "${use[@]}" --output-format csv --kernel-include-regex hastar_search_kernel -d $R/$name -o pmc -- python3 bench.py $ARGS > $OUT/pmc_$name.log 2>&1 || { tail -5 $OUT/pmc_$name.log; exit 1; }
}
pass FETCH FETCH_SIZE
pass WRITE WRITE_SIZE
pass SQA SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU
pass SQB SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH
pass TCC TCC_HIT_sum TCC_MISS_sum
python3 tools/prof_summary.py pmc $R/FETCH $R/WRITE $OUT/pmc_search_summary.json --batch $B --grid 1024 --dispatch 1 || exit 1
python3 tools/prof_summary.py counters $OUT/counters_search.json $R/SQA $R/SQB $R/TCC --batch $B --grid 1024 --dispatch 1 || exit 1
cat $OUT/pmc_search_summary.json | head -12
