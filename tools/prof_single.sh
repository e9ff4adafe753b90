#!/bin/bash
# Instruction mix of ONE exact search on the latency kernel (run on the GPU box):
#   tools/prof_single.sh <tag> <seed>...   -> gpurun_out/<tag>/single_<seed>.json
# Separate rocprofv3 --pmc passes over tools/profile_search.py (normal library, one query per
# process) restricted to hastar_search_wide_kernel; tools/prof_summary.py counters sums them.
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
R=/tmp/rps_$TAG
rm -rf $R && mkdir -p $R
for s in "$@"; do
  for pass in "SQA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
              "SQB SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
    set -- $pass
    name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv --kernel-include-regex hastar_search_wide_kernel \
      -d $R/${name}_$s -o pmc -- python3 tools/profile_search.py --seeds $s > $OUT/pmc_${name}_$s.log 2>&1 \
      || { tail -5 $OUT/pmc_${name}_$s.log; exit 1; }
  done
  python3 tools/prof_summary.py counters $OUT/single_$s.json $R/SQA_$s $R/SQB_$s --batch 1 --dispatch -1 \
    --kernel hastar_search_wide_kernel || exit 1
  cat $OUT/single_$s.json
done
