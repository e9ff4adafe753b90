set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02a/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02a/pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --cpu-seconds 5 > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err || { tail -20 gpurun_out/r02a/bench.err; exit 1; }
cat gpurun_out/r02a/bench.json
