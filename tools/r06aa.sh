# round-6 GPU iteration aa: 12 search waves per CU (lib_occ12w: 3 per SIMD under a 168-VGPR
# budget, 512-node inner LDS pools, 12-wave workgroups) against the main build: parity of the
# batch kernel first, then short cfg3 benches alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06aa; mkdir -p $O
P=path_planning_pkg_amd
HASTAR_LIB=$P/lib_occ12w/libhastar_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fuzz.py::test_random_configurations_both_kernels tests/test_gpu_parity.py > $O/pytest_occ12w.txt 2>&1 || { tail -30 $O/pytest_occ12w.txt; exit 1; }
tail -3 $O/pytest_occ12w.txt
bash tools/ab_bench.sh r06aa $P/lib $P/lib_occ12w $P/lib $P/lib_occ12w || exit 1
