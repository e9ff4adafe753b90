# cfg5 (20 Hz replan loop) and cfg4 (2048^2) lines with the 8-waves-per-CU build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02s
mkdir -p $O
timeout -k 10 600 python -u bench.py --workload cfg5 > $O/cfg5.json 2> $O/cfg5.err || { tail -30 $O/cfg5.err; exit 1; }
cut -c1-300 $O/cfg5.json
timeout -k 10 900 python -u bench.py --workload cfg4 > $O/cfg4.json 2> $O/cfg4.err || { tail -30 $O/cfg4.err; exit 1; }
cut -c1-300 $O/cfg4.json
