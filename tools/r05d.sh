# round-5 GPU iteration d: SGPR -> VGPR pointer pins and 32-bit counters (batch kernel alone, then split), f64 bit parity
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05d; mkdir -p $O
AB_SPLIT=0 bash tools/ab_bench.sh r05d path_planning_pkg_amd/lib_vc path_planning_pkg_amd/lib_v1 path_planning_pkg_amd/lib_v3 path_planning_pkg_amd/lib_v4 path_planning_pkg_amd/lib_vc &&
bash tools/ab_bench.sh r05d path_planning_pkg_amd/lib_v4 path_planning_pkg_amd/lib_vc &&
HASTAR_LIB=path_planning_pkg_amd/lib_v4/libhastar_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -v --timeout 300 --timeout-method thread > $O/pytest_f64.txt 2>&1; tail -30 $O/pytest_f64.txt | cut -c1-200
