# round-6 GPU iteration af: round profile of the final sources (trace + PMC + SQ counters, hash-matched)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/prof_round.sh r06af || exit 1
