set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02d/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r02d/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02d/pytest_gpu.log
timeout -k 10 900 python -u bench.py > gpurun_out/r02d/bench.json 2> gpurun_out/r02d/bench.err || { tail -30 gpurun_out/r02d/bench.err; exit 1; }
cat gpurun_out/r02d/bench.json
