# round-6 GPU iteration e: tiled, XCD-banded relocation by inversion: relocation tests, A/B
# against the claim passes at 1024^2 and 2048^2 (rocprofv3 kernel stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06e}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "relocation or map_upkeep or batched_map" > $O/pytest_reloc.txt 2>&1 || { tail -40 $O/pytest_reloc.txt; exit 1; }
tail -2 $O/pytest_reloc.txt
for g in 1024 2048; do
for m in invert claim; do
  n=$((1024 * 1024 * 1024 / g / g))
  HASTAR_RELOC=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${m}_$g -o reloc -- python3 -u tools/reloc_bench.py --grid $g --n $n --reps 5 > $O/reloc_${m}_$g.json 2> $O/reloc_${m}_$g.err
  rc=$?; [ $rc -ne 0 ] && { tail -20 $O/reloc_${m}_$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/reloc_${m}_$g.json')); print('$m $g', round(d['wall_ms_median'],3), round(d['alg_TBps_wall'],2))"
  find $O/prof_${m}_$g -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/reloc_kernel_stats_${m}_$g.csv
  head -4 $O/reloc_kernel_stats_${m}_$g.csv | cut -c1-160
done
done
