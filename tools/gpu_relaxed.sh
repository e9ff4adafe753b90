set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rlx
timeout -k 10 300 python -u tools/relaxed_sweep.py --out gpurun_out/rlx/sweep.json > gpurun_out/rlx/sweep.log 2>&1 || { tail -30 gpurun_out/rlx/sweep.log; exit 1; }
cat gpurun_out/rlx/sweep.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_relaxed.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/rlx/pytest.log 2>&1
rc=$?
grep -E "relaxed .* ms vs exact|passed|failed|Error" gpurun_out/rlx/pytest.log | tail -20
exit $rc
