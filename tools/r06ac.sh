# round-6 GPU iteration ac: the backward grid-distance field (csrc/hastar_field.hip): its GPU
# tests, a timing of one GPU and 4 stand-in ranks on cfg3 / cfg4 maps, and its kernel statistics
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_field.py > $O/pytest_field.txt 2>&1 || { tail -40 $O/pytest_field.txt; exit 1; }
grep -E "passed|failed|passes|rounds" $O/pytest_field.txt | tail -12
timeout -k 10 300 python -u tools/field_bench.py > $O/field_bench.jsonl 2> $O/field_bench.err || { tail -20 $O/field_bench.err; exit 1; }
cat $O/field_bench.jsonl
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o field -- python3 tools/field_bench.py --reps 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/field_kernel_stats.csv
head -8 $O/field_kernel_stats.csv
