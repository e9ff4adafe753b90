set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-rlx}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_relaxed.py -x -v -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "relaxed .* ms vs exact|passed|failed|Error" $O/pytest.log | tail -20; exit 1; }
grep -E "relaxed .* ms vs exact|passed|failed" $O/pytest.log | tail -20
timeout -k 10 300 python -u tools/relaxed_sweep.py --groups syn512,cfg3,cfg5 --out $O/sweep.json > $O/sweep.log 2>&1 || { tail -30 $O/sweep.log; exit 1; }
python - "$O/sweep.json" <<'PY'
import json, sys
for r in json.load(open(sys.argv[1])):
    print(r["group"], r["delta"], r["h_weight"], r["h_stop"], r.get("h_coarse"), r["ms"], r["ok"], r["cost_ratio_mean"], [round(x[0], 2) for x in r["split_ms"]], [round(x[1], 2) for x in r["split_ms"]])
PY
