# round-5 GPU iteration b: libm fingerprint, profiler capabilities, targeted parity, stamps, short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1; echo "list rc=$?"
timeout -k 10 300 tools/bin/libm64_fingerprint 2e8 0 16 > $O/libm64_ocml.jsonl 2> $O/libm64.err && cut -c1-260 $O/libm64_ocml.jsonl &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -k "head_arenas or split_launch or cfg3_parity_batch or survey_reference" tests/test_gpu_f64.py -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 && tail -3 $O/pytest.txt &&
HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so timeout -k 10 300 python -u tools/profile_search.py --seeds 2396 1 3 > $O/stamps.jsonl 2>&1 && cut -c1-200 $O/stamps.jsonl &&
timeout -k 10 600 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --latency-queries 3 --relaxed-batch 0 > $O/bench.json 2> $O/bench.err && cut -c1-300 $O/bench.json
