set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r02b/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02b/pytest_gpu.log
