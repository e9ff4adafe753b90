set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cfg4
timeout -k 10 900 python -u bench.py --workload cfg4 --steps 3 --warmup 1 > gpurun_out/cfg4/bench.json 2> gpurun_out/cfg4/bench.err || { tail -30 gpurun_out/cfg4/bench.err; exit 1; }
cut -c1-1500 gpurun_out/cfg4/bench.json
