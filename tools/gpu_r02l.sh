# Step balance of the bench batch: slot busy fraction and the longest search under load
# (release build), then the shader clock of the searches under load (stamps build).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02l
mkdir -p $O
timeout -k 10 400 python -u tools/tail_analysis.py --steps 2 > $O/tail.jsonl 2> $O/tail.err || { tail -20 $O/tail.err; exit 1; }
cat $O/tail.jsonl
HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 400 python -u tools/tail_analysis.py --steps 2 --clock > $O/tail_stamps.jsonl 2> $O/tail_stamps.err || { tail -20 $O/tail_stamps.err; exit 1; }
cat $O/tail_stamps.jsonl
