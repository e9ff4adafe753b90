# cfg3 batch beyond 23552 (queries 23552..24575 need at most 95,057 pops, so the longest search
# stays query 2395): B = 24064 and 24576, CPU baseline skipped.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02z
mkdir -p $O
for B in 24064 24576; do
  timeout -k 10 600 python -u bench.py --batch $B --no-cpu-baseline > $O/b$B.json 2> $O/b$B.err || { tail -30 $O/b$B.err; exit 1; }
  cut -c1-160 $O/b$B.json
done
