# round-6 GPU iteration ae: the final tree (heuristic field added): the whole GPU suite and smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_iter.sh r06ae test smoke || exit 1
