# round-6 GPU iteration q: the final tree: the whole GPU suite (fuzz and reversing tests included),
# smoke, and the driver's default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06q; mkdir -p $O
bash tools/gpu_iter.sh r06q test smoke bench || exit 1
