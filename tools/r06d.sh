# round-6 GPU iteration d: relocation by inversion (A/B against the claim passes, rocprofv3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "relocation or map_upkeep or batched_map" > $O/pytest_reloc.txt 2>&1 || { tail -40 $O/pytest_reloc.txt; exit 1; }
tail -2 $O/pytest_reloc.txt
for m in invert claim; do
  HASTAR_RELOC=$m timeout -k 10 120 python -u tools/reloc_bench.py --n 1024 --reps 5 > $O/reloc_$m.json 2> $O/reloc_$m.err || { tail -20 $O/reloc_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/reloc_$m.json')); print('$m', round(d['wall_ms_median'],2), round(d['alg_TBps_wall'],2))"
  HASTAR_RELOC=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o reloc -- python3 -u tools/reloc_bench.py --n 1024 --reps 5 > $O/reloc_prof_$m.json 2> $O/reloc_prof_$m.err
  rc=$?; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
  find $O/prof_$m -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/reloc_kernel_stats_$m.csv
  head -4 $O/reloc_kernel_stats_$m.csv
done
