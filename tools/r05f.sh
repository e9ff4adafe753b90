# round-5 GPU iteration f: device libm ports (acos included) and f64 bit parity; latency-kernel
# register variants on cfg5; HBM counter calibration
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 300 tools/bin/libm64_fingerprint 2e8 1 16 > $O/libm64_gm64.jsonl 2> $O/libm64.err && cut -c1-150 $O/libm64_gm64.jsonl || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py -q --timeout 300 --timeout-method thread > $O/pytest_f64.txt 2>&1; tail -3 $O/pytest_f64.txt
for L in lib lib_w2 lib; do
  HASTAR_LIB=path_planning_pkg_amd/$L/libhastar_amd.so timeout -k 10 300 python -u bench.py --workload cfg5 --steps 5 --no-cpu-baseline --no-relaxed > $O/cfg5_$L.json 2> $O/cfg5_$L.err || { tail -20 $O/cfg5_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg5_$L.json')); print('$L', round(d['tick_ms'],1), [(s['pair'], round(s['ms'])) for s in d['slowest_search_per_tick']], d['parity_sample']['bit_exact'])"
done
bash tools/prof_fetch_calib.sh r05f
