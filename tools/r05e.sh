# round-5 GPU iteration e: the full GPU suite, smoke, the driver's bench line, cfg5, single-query stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench_drv.json 2> $O/bench_drv.err || { tail -30 $O/bench_drv.err; exit 1; }
cut -c1-300 $O/bench_drv.json
timeout -k 10 600 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
cut -c1-300 $O/bench_cfg5.json
HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 300 python -u tools/profile_search.py --seeds 2396 1 3 > $O/stamps.jsonl 2>&1 || { tail -20 $O/stamps.jsonl; exit 1; }
cut -c1-200 $O/stamps.jsonl
