#!/bin/bash
# A/B of library builds on one box: tools/ab_bench.sh <tag> <libdir>... (each: a short cfg3 bench)
#   HASTAR_LIB=<libdir>/libhastar_amd.so python bench.py --steps 3 --warmup 1 (no CPU/latency/relaxed legs)
# AB_SPLIT=0 runs them with HASTAR_SPLIT=0 (the batch kernel alone).
# -> gpurun_out/<tag>/ab_<libdir basename>_<i>.json, one summary line per run
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG; mkdir -p $O
i=0
for L in "$@"; do
  i=$((i+1))
  n=$(basename $L)
  if [ -n "$AB_SPLIT" ]; then export HASTAR_SPLIT=$AB_SPLIT; fi
  HASTAR_LIB=$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/ab_${n}_$i.json 2> $O/ab_${n}_$i.err || { tail -20 $O/ab_${n}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab_${n}_$i.json')); sb=d['step_balance']; print('$n split=${AB_SPLIT:-default}', round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']], 'busy', round(sb['slot_busy_mean_ms']), 'longest', round(sb['longest_search_under_load_ms']), 'parity', d.get('parity_sample',{}).get('bit_exact'))"
done
