set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02e/pytest_gpu.log 2>&1 || { grep -E "PASSED|FAILED|Error|error" gpurun_out/r02e/pytest_gpu.log | tail -30; exit 1; }
tail -3 gpurun_out/r02e/pytest_gpu.log
timeout -k 10 900 python -u bench.py > gpurun_out/r02e/bench.json 2> gpurun_out/r02e/bench.err || { tail -30 gpurun_out/r02e/bench.err; exit 1; }
cut -c1-700 gpurun_out/r02e/bench.json
