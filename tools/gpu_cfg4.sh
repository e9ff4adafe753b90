#!/bin/bash
# cfg4 GPU pass (run on the GPU box):  tools/gpu_cfg4.sh <tag> [batch]
#   GPU parity tests -> bench.py --workload cfg4 (2048^2 queries + row-sharded map build).
set -o pipefail
TAG=${1:-cfg4}
BATCH=${2:-2048}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 600 python -u bench.py --workload cfg4 --batch $BATCH --steps 2 --warmup 1 > gpurun_out/$TAG/bench_cfg4.json 2> gpurun_out/$TAG/bench_cfg4.err || { tail -20 gpurun_out/$TAG/bench_cfg4.err; exit 1; }
cat gpurun_out/$TAG/bench_cfg4.json
