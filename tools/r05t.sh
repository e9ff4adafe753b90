# round-5 GPU iteration t: phase stamps of single searches with the deferred inner tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05t; mkdir -p $O
HASTAR_WIDE=0 HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 300 python -u tools/profile_search.py --seeds 1 3 > $O/stamps_batchk.jsonl 2>&1 || { tail -20 $O/stamps_batchk.jsonl; exit 1; }
HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 300 python -u tools/profile_search.py --seeds 1 3 > $O/stamps_latk.jsonl 2>&1 || { tail -20 $O/stamps_latk.jsonl; exit 1; }
grep -v amdgpu.ids $O/stamps_batchk.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('batchk', d['seed'], d['kernel_ms'], d['cyc_per_apop_lds'], d['lds_astar_per_apop'], d['lds_astar_parts_per_apop'])"
grep -v amdgpu.ids $O/stamps_latk.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('latk', d['seed'], d['kernel_ms'], d['cyc_per_apop_lds'], d['lds_astar_per_apop'], d['lds_astar_parts_per_apop'])"
