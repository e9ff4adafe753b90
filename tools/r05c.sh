# round-5 GPU iteration c: device libm ports against glibc; A/B of the inner-tree header cache
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 tools/bin/libm64_fingerprint 2e8 1 16 > $O/libm64_gm64.jsonl 2> $O/libm64.err && cut -c1-200 $O/libm64_gm64.jsonl &&
bash tools/ab_bench.sh r05c path_planning_pkg_amd/lib_base path_planning_pkg_amd/lib path_planning_pkg_amd/lib_vc path_planning_pkg_amd/lib_base path_planning_pkg_amd/lib
