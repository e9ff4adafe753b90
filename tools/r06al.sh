# round-6 GPU iteration al: the whole GPU suite and smoke on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_iter.sh r06al test smoke || exit 1
