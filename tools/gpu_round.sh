#!/bin/bash
# Round GPU pass (run on the GPU box):  tools/gpu_round.sh <tag>
#   parity tests -> cfg5 replan-loop bench line -> tools/prof_round.sh <tag> (cfg3 bench under
#   rocprofv3 + PMC passes).  Stops at the first failing step.
set -o pipefail
TAG=${1:-round}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 18 --warmup 2 > gpurun_out/$TAG/bench_cfg5.json 2> gpurun_out/$TAG/bench_cfg5.err || { tail -20 gpurun_out/$TAG/bench_cfg5.err; exit 1; }
cat gpurun_out/$TAG/bench_cfg5.json
bash tools/prof_round.sh $TAG
