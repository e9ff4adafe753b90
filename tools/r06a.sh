# round-6 GPU iteration a: housekeeping + lean CPU baseline + in-place relocation: GPU suite, smoke,
# relocation throughput (rocprofv3), 20-tick cfg5 line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k relocation > $O/pytest_reloc.txt 2>&1 || { tail -40 $O/pytest_reloc.txt; exit 1; }
tail -3 $O/pytest_reloc.txt
timeout -k 10 120 python -u tools/reloc_bench.py --n 2048 --reps 5 > $O/reloc_bench.json 2> $O/reloc_bench.err || { tail -20 $O/reloc_bench.err; exit 1; }
cat $O/reloc_bench.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/reloc_prof -o reloc -- python3 -u tools/reloc_bench.py --n 2048 --reps 5 > $O/reloc_bench_prof.json 2> $O/reloc_prof.err || { tail -20 $O/reloc_prof.err; exit 1; }
find $O/reloc_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/reloc_kernel_stats.csv
head -5 $O/reloc_kernel_stats.csv
bash tools/gpu_iter.sh r06a test smoke || exit 1
timeout -k 10 900 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); c=d['cpu_baseline']; print('cfg5', d['steps'], round(d['tick_ms'],1), sorted([round(s['ms']) for s in d['slowest_search_per_tick']])[-3:], 'cpu', round(c['tick_ms_one_core_per_pair'],1), d['parity_sample']['bit_exact'], d['parity_sample']['searches'], d['relaxed_mode']['tick_ms'])"
