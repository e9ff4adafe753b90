set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03g
timeout -k 10 400 python -u tools/dbg_case.py rowshard2048 > gpurun_out/r03g/dbg.txt 2>&1; cat gpurun_out/r03g/dbg.txt
bash tools/gpu_iter.sh r03g test
