# End-of-round check of the committed tree: GPU suite, smoke, default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/final_r02
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
