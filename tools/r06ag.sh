# round-6 GPU iteration ag: the field's GPU tests with the small-block cases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ag; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_field.py > $O/pytest_field.txt 2>&1 || { tail -40 $O/pytest_field.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/pytest_field.txt | tail -16
