#!/bin/bash
# HBM read-counter calibration on the box: tools/prof_fetch_calib.sh <tag>
#   1. tools/bin/fetch_calib's known patterns under three --pmc passes (FETCH_SIZE; the EA read
#      requests by size; DRAM requests and L2 hits/misses)
#   2. the same passes over the batch search kernel (a 1-step bench, HASTAR_SPLIT=0)
#   -> gpurun_out/<tag>/fetch_calib.jsonl (patterns), calib_pmc.json, search_pmc.json
set -o pipefail
TAG=${1:-calib}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=/tmp/rpc_$TAG; rm -rf $R; mkdir -p $R
timeout -k 10 300 tools/bin/fetch_calib > $OUT/fetch_calib.jsonl || exit 1
cat $OUT/fetch_calib.jsonl
P1="FETCH_SIZE"
P2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
P3="TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $R/c$i -o pmc -- tools/bin/fetch_calib > $OUT/calib_pass$i.log 2>&1 || { tail -5 $OUT/calib_pass$i.log; exit 1; }
done
python3 tools/pmc_table.py $OUT/calib_pmc.json $R/c1 $R/c2 $R/c3 --kernel-regex "k_stream16|k_scatter|k_probe" || exit 1
export HASTAR_SPLIT=0
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $P --output-format csv --kernel-include-regex hastar_search_kernel -d $R/s$i -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $OUT/search_pass$i.log 2>&1 || { tail -5 $OUT/search_pass$i.log; exit 1; }
done
python3 tools/pmc_table.py $OUT/search_pmc.json $R/s1 $R/s2 $R/s3 --kernel-regex hastar_search_kernel || exit 1
