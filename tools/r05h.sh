# round-5 GPU iteration h: 12 vs 16 latency CUs over 20 steps (outliers?), cfg4 line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05h; mkdir -p $O
for hc in 12 16 12; do
  HASTAR_HEAD_CUS=$hc timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --step-diag --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/bench_h$hc.json 2> $O/bench_h$hc.err || { tail -30 $O/bench_h$hc.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_h$hc.json')); print($hc, round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']])"
  cat $O/bench_h$hc.json >> $O/bench_h$hc.all.jsonl
done
timeout -k 10 900 python -u bench.py --workload cfg4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -30 $O/bench_cfg4.err; exit 1; }
cut -c1-400 $O/bench_cfg4.json
