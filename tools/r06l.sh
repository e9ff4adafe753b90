# round-6 GPU iteration l: the relaxed mode's reversing model (Reeds-Shepp): relaxed GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_relaxed.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest_relaxed.txt 2>&1 || { tail -60 $O/pytest_relaxed.txt; exit 1; }
grep -E "PASSED|FAILED|reversals|goal behind|forward" $O/pytest_relaxed.txt | cut -c1-300 | tail -40
