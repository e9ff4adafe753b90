# Fewer resident searches than arenas (HASTAR_SLOTS): less load on the memory system for the
# longest search, more work per slot.  cfg3 default bench, CPU baseline skipped.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02aa
mkdir -p $O
for S in 1700 1850; do
  HASTAR_SLOTS=$S timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/s$S.json 2> $O/s$S.err || { tail -30 $O/s$S.err; exit 1; }
  cut -c1-160 $O/s$S.json
done
