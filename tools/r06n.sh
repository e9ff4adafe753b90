# round-6 GPU iteration n: randomised planner configurations on both kernels against the oracle
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest_fuzz.txt 2>&1 || { tail -40 $O/pytest_fuzz.txt; exit 1; }
grep -E "PASSED|FAILED|seed" $O/pytest_fuzz.txt | cut -c1-300
