# round-6 GPU iteration i: multi-rank rehearsal of bench.py on a one-GPU box (2 ranks on cuda:0,
# gloo for the collectives; the driver's 8-GPU runs use RCCL): cfg3, cfg5 and cfg4 paths, small sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06i; mkdir -p $O
export HASTAR_BENCH_DEVICE=0 HASTAR_ARENA_FRAC=0.3
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --batch 2048 --steps 2 --warmup 1 --latency-queries 0 --relaxed-batch 0 --cpu-seconds 3 > $O/cfg3_2ranks.json 2> $O/cfg3_2ranks.err || { tail -30 $O/cfg3_2ranks.err; exit 1; }
cut -c1-600 $O/cfg3_2ranks.json
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --workload cfg5 --pairs 16 --steps 3 --warmup 1 > $O/cfg5_2ranks.json 2> $O/cfg5_2ranks.err || { tail -30 $O/cfg5_2ranks.err; exit 1; }
cut -c1-600 $O/cfg5_2ranks.json
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --workload cfg4 --batch 256 --map-queries 4 --steps 1 --warmup 1 --latency-queries 0 --relaxed-batch 0 --cpu-seconds 3 > $O/cfg4_2ranks.json 2> $O/cfg4_2ranks.err || { tail -30 $O/cfg4_2ranks.err; exit 1; }
cut -c1-600 $O/cfg4_2ranks.json
