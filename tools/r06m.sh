# round-6 GPU iteration m: the final build (relaxed reversing model added): GPU suite, smoke, the
# round profile (trace + PMC + SQ counters, hash-matched to this build) and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06m; mkdir -p $O
bash tools/gpu_iter.sh r06m test smoke || exit 1
bash tools/prof_round.sh r06m || exit 1
