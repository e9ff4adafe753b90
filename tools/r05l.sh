# round-5 GPU iteration l: handoff only for cold batches; threshold sweep on the cold step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v -k "split or handoff or park" --timeout 300 --timeout-method thread > $O/pytest_split.txt 2>&1 || { tail -40 $O/pytest_split.txt; exit 1; }
tail -2 $O/pytest_split.txt
for v in 32768 16384 65536 32768; do
  HASTAR_HANDOFF_POPS=$v timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --latency-queries 1 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -30 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', round(d['value']/1e6,3), 'cold', round(d['cold_first_step']['value']/1e6,3), d['cold_first_step']['handoffs'], 'order', round(d['cold_order_step']['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']], d['step_balance']['handoffs'])"
  cat $O/bench_$v.json >> $O/sweep.jsonl
done
