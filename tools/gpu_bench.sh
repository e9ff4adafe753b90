#!/bin/bash
# tools/gpu_bench.sh <tag> [bench args...] — one bench.py run on the GPU box -> gpurun_out/<tag>/bench.json
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
