# round-6 GPU iteration c: where the in-place relocation's time goes (diagnostic modes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06c; mkdir -p $O
for m in 0 1 2 4 6 7; do
  HASTAR_RELOC_MODE=$m timeout -k 10 120 python -u tools/reloc_bench.py --n 1024 --reps 3 > $O/reloc_mode$m.json 2> $O/reloc_mode$m.err || { tail -20 $O/reloc_mode$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/reloc_mode$m.json')); print('mode $m', round(d['wall_ms_median'],2), round(d['alg_TBps_wall'],2))"
done
