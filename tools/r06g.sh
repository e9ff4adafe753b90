# round-6 GPU iteration g: relocation chunk size (scratch bytes per launch pair: does the copy-back
# read the scratch from the Infinity Cache when the chunk fits in it?)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
for mb in 1024 128 64 32 16; do
  HASTAR_RELOC_CHUNK_MB=$mb timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$mb -o reloc -- python3 -u tools/reloc_bench.py --grid 1024 --n 1024 --reps 5 > $O/reloc_$mb.json 2> $O/reloc_$mb.err
  rc=$?; [ $rc -ne 0 ] && { tail -20 $O/reloc_$mb.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/reloc_$mb.json')); print('chunk MB $mb', round(d['wall_ms_median'],3), round(d['alg_TBps_wall'],2))"
  find $O/prof_$mb -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/reloc_kernel_stats_$mb.csv
  head -3 $O/reloc_kernel_stats_$mb.csv | cut -c1-130
done
