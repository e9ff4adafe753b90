# round-5 GPU iteration ab: claims take the most advanced offer (vs the oldest)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v -k "handoff or split" --timeout 300 --timeout-method thread > $O/pytest_split.txt 2>&1 || { tail -40 $O/pytest_split.txt; exit 1; }
tail -1 $O/pytest_split.txt
for L in lib_pre lib lib_pre lib; do
  HASTAR_LIB=path_planning_pkg_amd/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --latency-queries 0 --relaxed-batch 0 > $O/b_$L.json 2> $O/b_$L.err || { tail -30 $O/b_$L.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b_$L.json')); c=d['cold_first_step']
print('$L', round(d['value']/1e6,3), [round(k) for k in d['kernel_ms_per_step']], 'busy', round(d['step_balance']['slot_busy_mean_ms']), 'cold', round(c['value']/1e6,3), round(c['ms']), c['handoffs'], 'order', round(d['cold_order_step']['value']/1e6,3), c['last_to_end'][0])"
  cat $O/b_$L.json >> $O/ab.jsonl
done
