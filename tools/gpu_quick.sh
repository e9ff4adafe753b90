set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/q
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/q/smoke.txt 2>&1 || { tail -20 gpurun_out/q/smoke.txt; exit 1; }
cat gpurun_out/q/smoke.txt
timeout -k 10 600 python -u -m pytest tests/test_cxx_dropin.py tests/test_gpu_scale.py::test_cfg3_survey_reference_cases tests/test_gpu_relaxed.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/q/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error" gpurun_out/q/pytest.log | tail -15
exit $rc
