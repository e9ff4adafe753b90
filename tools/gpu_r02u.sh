# Phase stamps of the longest search under load (the bench batch, stamps build), to compare
# with the same search alone (profiles/r02p_stamps_single_query.jsonl).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02u
mkdir -p $O
HASTAR_ARENA_FRAC=0.95 HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 400 python -u tools/tail_analysis.py --steps 2 --clock > $O/tail_stamps.jsonl 2> $O/tail_stamps.err || { tail -20 $O/tail_stamps.err; exit 1; }
cat $O/tail_stamps.jsonl
