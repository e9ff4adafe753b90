# round-5 GPU iteration j: unit kernels on the double libm ports, cfg5 line with the 16-thread CPU tick
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cxx_units.py tests/test_gpu_f64.py tests/test_local_planner.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_units.txt 2>&1 || { tail -40 $O/pytest_units.txt; exit 1; }
tail -3 $O/pytest_units.txt
timeout -k 10 600 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -30 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print(d['tick_ms'], d['cpu_baseline'], d['parity_sample']['bit_exact'])"
