set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rlx
timeout -k 10 600 python -u -m pytest tests/test_gpu_relaxed.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/rlx/pytest.log 2>&1 || { grep -E "relaxed .* ms vs exact|passed|failed|Error" gpurun_out/rlx/pytest.log | tail -20; exit 1; }
grep -E "relaxed .* ms vs exact|passed|failed" gpurun_out/rlx/pytest.log | tail -20
timeout -k 10 300 python -u tools/relaxed_sweep.py --groups syn512,cfg3,cfg5 --out gpurun_out/rlx/sweep.json > gpurun_out/rlx/sweep.log 2>&1 || { tail -30 gpurun_out/rlx/sweep.log; exit 1; }
cut -c1-300 gpurun_out/rlx/sweep.log
timeout -k 10 600 python -u bench.py --workload cfg5 --steps 3 --warmup 1 > gpurun_out/rlx/cfg5.json 2> gpurun_out/rlx/cfg5.err || { tail -30 gpurun_out/rlx/cfg5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/rlx/cfg5.json'));print(d['tick_ms'], d['relaxed_mode'])"
