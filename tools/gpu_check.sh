#!/bin/bash
# GPU iteration check (run on the GPU box): parity tests, then single-query phase profiles
# of the straggler seed and seed 1 (diagnostic stamps build), then optionally a batch run.
#   tools/gpu_check.sh [batch]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 200 python -u tools/profile_search.py --seeds 10227 1 > gpurun_out/prof.txt 2>&1 || { tail -20 gpurun_out/prof.txt; exit 1; }
cat gpurun_out/prof.txt
if [ -n "$1" ]; then
  timeout -k 10 400 python -u tools/batch_scaling.py --batches $1 --repeat 2 > gpurun_out/bs.txt 2>&1 || { tail -20 gpurun_out/bs.txt; exit 1; }
  cat gpurun_out/bs.txt
fi
