# round-6 GPU iteration ad: cfg4's heuristic-field leg (bench.py:field_phase): one rank (whole
# field + 4 stand-in ranks), then 2 and 4 gloo ranks on the one GPU (the sharded protocol with
# real collectives; the driver's multi-GPU runs use RCCL)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ad; mkdir -p $O
timeout -k 10 500 python -u bench.py --workload cfg4 --batch 256 --map-queries 4 --steps 1 --warmup 1 --latency-queries 0 --relaxed-batch 0 --cpu-seconds 3 > $O/cfg4_1rank.json 2> $O/cfg4_1rank.err || { tail -30 $O/cfg4_1rank.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg4_1rank.json')); print(json.dumps(d['map_build']['heuristic_field']))"
export HASTAR_BENCH_DEVICE=0 HASTAR_ARENA_FRAC=0.3
for G in 2 4; do
  timeout -k 10 500 python -u bench.py --gpus $G --backend gloo --workload cfg4 --batch 128 --map-queries 2 --steps 1 --warmup 1 --latency-queries 0 --relaxed-batch 0 --cpu-seconds 3 > $O/cfg4_${G}ranks.json 2> $O/cfg4_${G}ranks.err || { tail -30 $O/cfg4_${G}ranks.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg4_${G}ranks.json')); print($G, json.dumps(d['map_build']['heuristic_field']))"
done
