# round-6 GPU iteration ab: the latency kernel's inner ring mirrors its entries' f values (one
# LDS round trip per rank-query level instead of two); lib = that build, lib_base = the build before.
# The latency kernel's parity tests first, then plan latency and 5-tick cfg5 alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ab; mkdir -p $O
P=path_planning_pkg_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py \
  tests/test_gpu_scale.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for L in lib_base lib lib_base lib; do
  HASTAR_LIB=$P/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --relaxed-batch 0 > $O/lat_$L.json 2> $O/lat_$L.err || { tail -20 $O/lat_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lat_$L.json')); print('$L latency', [round(x,1) for x in d['plan_latency_ms']['gpu']], round(d['longest_query']['gpu_ms_alone'],1), 'cfg3', round(d['value']/1e6,3))"
done
for L in lib_base lib; do
  HASTAR_LIB=$P/$L/libhastar_amd.so timeout -k 10 400 python -u bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-relaxed > $O/cfg5_$L.json 2> $O/cfg5_$L.err || { tail -20 $O/cfg5_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg5_$L.json')); print('$L cfg5 tick', round(d['tick_ms'],1), d['parity_sample']['bit_exact'])"
done
