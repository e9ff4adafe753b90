set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rlx
timeout -k 10 600 python -u -m pytest tests/test_gpu_relaxed.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/rlx/pytest.log 2>&1 || { grep -E "relaxed .* ms vs exact|passed|failed|Error" gpurun_out/rlx/pytest.log | tail -20; exit 1; }
grep -E "relaxed .* ms vs exact|passed|failed" gpurun_out/rlx/pytest.log | tail -20
timeout -k 10 300 python -u tools/relaxed_sweep.py --groups syn512,cfg3,cfg5 --out gpurun_out/rlx/sweep.json > gpurun_out/rlx/sweep.log 2>&1 || { tail -30 gpurun_out/rlx/sweep.log; exit 1; }
python - <<'PY'
import json
for r in json.load(open("gpurun_out/rlx/sweep.json")):
    print(r["group"], r["delta"], r["h_weight"], r["h_stop"], r["ms"], r["ok"], r["cost_ratio_mean"], [round(x[0], 2) for x in r["split_ms"]], [round(x[1], 2) for x in r["split_ms"]])
PY
