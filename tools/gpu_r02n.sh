# 8 search waves per CU (16 B LDS per inner-A* node, g/prev in HBM): GPU parity suite,
# single-query stamps, the bench at the library's arena size and at 196608 pops per arena.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 300 python -u tools/profile_search.py --grid 1024 --seeds 2396 1 2 3 --replan > $O/stamps.jsonl 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cut -c1-200 $O/stamps.jsonl
timeout -k 10 900 python -u bench.py --max-pops 196608 > $O/bench_mp196608.json 2> $O/bench_mp196608.err || { tail -30 $O/bench_mp196608.err; exit 1; }
cut -c1-300 $O/bench_mp196608.json
timeout -k 10 900 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
