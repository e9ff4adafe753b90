# round-6 GPU iteration ah: the field kernel with 64 x 64 tiles (lib_f64t) against 32 x 32 (lib):
# its GPU tests, then tools/field_bench.py alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ah; mkdir -p $O
P=path_planning_pkg_amd
HASTAR_LIB=$P/lib_f64t/libhastar_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_field.py > $O/pytest_f64t.txt 2>&1 || { tail -30 $O/pytest_f64t.txt; exit 1; }
tail -1 $O/pytest_f64t.txt
for L in lib lib_f64t lib lib_f64t; do
  HASTAR_LIB=$P/$L/libhastar_amd.so timeout -k 10 300 python -u tools/field_bench.py --reps 5 > $O/fb_$L.jsonl 2> $O/fb_$L.err || { tail -20 $O/fb_$L.err; exit 1; }
  python3 -c "
import json
for l in open('$O/fb_$L.jsonl'):
    d=json.loads(l); print('$L', d['grid'], round(d['one_gpu_ms'],2), d['passes'], round(d['standin_ms'],2), d['rounds'], d['standin_equals_one_gpu'])"
done
