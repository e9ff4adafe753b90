"""Analysis: how often does the inner A*'s open-tree SHAPE decide a find/insert?

Builds the oracle with -DORC_SHAPE_STATS into /tmp and replays synthetic cfg3 seeds.
Per inner search: how many meet at least one shape-dependent event (a tree-free run would
have to restart them with the tree) and the pops they take before the first event.
Counts per find(): probes, probes with a node of the same cell in the open tree,
"unsafe" finds (a same-cell node with f < probe f: the lower_bound predicate is then
non-monotone and the result depends on the tree shape), unsafe inserts (same-cell node
with f > new f), max open size, pops with open size > 256 / > 1024, and violations of
the strict f order of the in-order sequence (expected 0).
"""
import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
so = "/tmp/orc_stats.so"
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DORC_SHAPE_STATS", "-shared", "-o", so,
                str(ROOT / "oracle" / "hastar_oracle.cpp"), "-lm"], check=True)
import oracle.pyoracle as po  # noqa: E402
po.LIB = Path(so)
from tests.scenarios import drive, synthetic  # noqa: E402

seeds = [int(a) for a in sys.argv[1:]] or list(range(1, 9))
from tests.scenarios import synthetic_ref  # noqa: E402
L = C.CDLL(so)
for s in seeds:
    cfg, proto = synthetic_ref(1024, 72, 200, s)
    o = po.OraclePlanner(cfg)
    drive(o, proto)
    st = (C.c_longlong * 16)()
    L.orc_shape_stats(st)
    r = o.find_path(proto["vel"], proto["start"])
    L.orc_shape_stats(st)
    names = ["probes", "same_cell_present", "unsafe_find", "unsafe_insert", "max_open", "pops_open_gt256",
             "pops_open_gt1024", "order_violations", "searches", "searches_shape_dependent", "pops_all",
             "pops_in_shape_dependent_searches", "pops_before_first_event", "hbm_pops_cap703",
             "hbm_pops_cap767", "hbm_pops_cap1023"]
    print(json.dumps(dict(seed=s, apops=r["stats"]["astar_pops"], **{n: st[q] for q, n in enumerate(names)})))
    o.close()
