# Pool-carved resume arenas beside a queue pass: park/resume tests, then the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02y
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_scale.py -k "park or pool or statuses" > $O/quick.txt 2>&1 || { tail -40 $O/quick.txt; exit 1; }
tail -9 $O/quick.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
