set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/dbg1
mkdir -p $O
timeout -k 10 120 python -u -m pytest -x -v --timeout 40 --timeout-method thread tests/test_gpu_parity.py::test_libm_ports_on_gpu tests/test_cxx_units.py::test_units_match_golden_and_oracle > $O/t1.txt 2>&1 || { tail -40 $O/t1.txt; exit 1; }
tail -3 $O/t1.txt
timeout -k 10 120 python -u -m pytest -x -v --timeout 40 --timeout-method thread tests/test_gpu_parity.py::test_harness_search_parity_and_golden > $O/t2.txt 2>&1 || { tail -40 $O/t2.txt; exit 1; }
tail -3 $O/t2.txt
