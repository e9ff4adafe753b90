# round-6 GPU iteration aj: plan latency with and without the latency kernel's helper waves
# (HASTAR_WIDE_DBG=4 runs the kernel without them): do idle helpers slow the inner A*?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06aj; mkdir -p $O
for M in default nohelp default nohelp; do
  if [ $M = nohelp ]; then export HASTAR_WIDE_DBG=4; else unset HASTAR_WIDE_DBG; fi
  timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --relaxed-batch 0 --batch 2048 > $O/lat_$M.json 2> $O/lat_$M.err || { tail -20 $O/lat_$M.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lat_$M.json')); print('$M latency', [round(x,1) for x in d['plan_latency_ms']['gpu']], round(d['longest_query']['gpu_ms_alone'],1))"
done
