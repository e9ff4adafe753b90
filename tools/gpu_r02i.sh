set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02i
timeout -k 10 900 python -u bench.py > gpurun_out/r02i/bench.json 2> gpurun_out/r02i/bench.err || { tail -30 gpurun_out/r02i/bench.err; exit 1; }
cut -c1-300 gpurun_out/r02i/bench.json
timeout -k 10 900 python -u bench.py --workload cfg5 > gpurun_out/r02i/cfg5.json 2> gpurun_out/r02i/cfg5.err || { tail -30 gpurun_out/r02i/cfg5.err; exit 1; }
cut -c1-300 gpurun_out/r02i/cfg5.json
