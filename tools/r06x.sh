# round-6 GPU iteration x: round profile of the final (hinted) sources
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/prof_round.sh r06x || exit 1
