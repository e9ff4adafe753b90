set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1 && echo listed &&
timeout -k 10 300 tools/bin/libm64_fingerprint 2e8 0 16 > $O/libm64_ocml.jsonl 2> $O/libm64.err && cat $O/libm64_ocml.jsonl | cut -c1-300 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -k "head_arenas or split_launch" tests/test_gpu_f64.py -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; tail -5 $O/pytest.txt
