#!/bin/bash
# GPU iteration check with a batch-size sweep: parity tests, straggler phase profile, then
# tools/batch_scaling.py at the given batches with HASTAR_ARENA_FRAC=$FRAC (default 0.8).
#   FRAC=0.92 tools/gpu_check2.sh 16384 18432
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 200 python -u tools/profile_search.py --seeds 10227 > gpurun_out/prof.txt 2>&1 || { tail -20 gpurun_out/prof.txt; exit 1; }
cut -c1-700 gpurun_out/prof.txt
HASTAR_ARENA_FRAC=${FRAC:-0.8} timeout -k 10 600 python -u tools/batch_scaling.py --batches "$@" --repeat 2 > gpurun_out/bs.txt 2>&1 || { tail -20 gpurun_out/bs.txt; exit 1; }
cat gpurun_out/bs.txt
