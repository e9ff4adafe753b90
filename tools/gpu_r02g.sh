set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02g/pytest_gpu.log 2>&1 || { grep -E "PASSED|FAILED|Error|error" gpurun_out/r02g/pytest_gpu.log | tail -30; exit 1; }
tail -2 gpurun_out/r02g/pytest_gpu.log
timeout -k 10 900 python -u bench.py > gpurun_out/r02g/bench.json 2> gpurun_out/r02g/bench.err || { tail -30 gpurun_out/r02g/bench.err; exit 1; }
cut -c1-400 gpurun_out/r02g/bench.json
timeout -k 10 900 python -u bench.py --workload cfg4 > gpurun_out/r02g/cfg4.json 2> gpurun_out/r02g/cfg4.err || { tail -30 gpurun_out/r02g/cfg4.err; exit 1; }
cut -c1-400 gpurun_out/r02g/cfg4.json
