# Colour bits in a VGPR: quick parity checks first, then the suite, stamps and the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 120 python -u -m pytest -x -v --timeout 40 --timeout-method thread tests/test_cxx_units.py::test_units_match_golden_and_oracle tests/test_gpu_parity.py::test_harness_search_parity_and_golden > $O/quick.txt 2>&1 || { tail -40 $O/quick.txt; exit 1; }
tail -2 $O/quick.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 300 python -u tools/profile_search.py --grid 1024 --seeds 2396 1 2 3 --replan > $O/stamps.jsonl 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cut -c1-160 $O/stamps.jsonl
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
