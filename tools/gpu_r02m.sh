# Per-wave cost vs occupancy: the bench batch with 1024 / 1280 / 1536 resident slots
# (sum of search durations = total wave time; constant if waves do not slow each other).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02m
mkdir -p $O
export HASTAR_ARENA_FRAC=0.95
for S in 1024 1280 1536; do
  HASTAR_SLOTS=$S timeout -k 10 300 python -u tools/tail_analysis.py --steps 2 > $O/tail_$S.jsonl 2> $O/tail_$S.err || { tail -20 $O/tail_$S.err; exit 1; }
  echo "slots=$S"; tail -1 $O/tail_$S.jsonl
done
