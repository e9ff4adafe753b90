# round-5 GPU iteration g: statistics in VGPR lanes (lib_s1) and windowed rank queries (lib_r1):
# parity of lib_r1, A/B benches, batch-kernel single-query stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05g; mkdir -p $O
HASTAR_LIB=path_planning_pkg_amd/lib_r1/libhastar_amd.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_r1.txt 2>&1 || { tail -30 $O/pytest_r1.txt; exit 1; }
tail -2 $O/pytest_r1.txt
bash tools/ab_bench.sh r05g path_planning_pkg_amd/lib path_planning_pkg_amd/lib_s1 path_planning_pkg_amd/lib_r1 path_planning_pkg_amd/lib path_planning_pkg_amd/lib_r1 || exit 1
for L in lib_stamps lib_r1s; do
  HASTAR_WIDE=0 HASTAR_LIB=path_planning_pkg_amd/$L/libhastar_amd.so timeout -k 10 300 python -u tools/profile_search.py --seeds 1 3 > $O/stamps_batchk_$L.jsonl 2>&1 || { tail -20 $O/stamps_batchk_$L.jsonl; exit 1; }
  python3 -c "
import json
for l in open('$O/stamps_batchk_$L.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$L', d['seed'], round(d['kernel_ms'],1), round(d['cyc_per_apop_lds']), d['lds_astar_per_apop'])"
done
