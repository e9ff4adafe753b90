# cfg4 is bound by its longest search (slots busy 23 % of the step at B = 6144): larger batches
# trade idle arenas for planners.  B = 7680 and 8192, CPU baseline skipped.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02w
mkdir -p $O
for B in 7680 8192; do
  timeout -k 10 600 python -u bench.py --workload cfg4 --batch $B --no-cpu-baseline > $O/cfg4_b$B.json 2> $O/cfg4_b$B.err || { tail -30 $O/cfg4_b$B.err; exit 1; }
  cut -c1-200 $O/cfg4_b$B.json
done
