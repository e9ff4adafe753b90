"""Analysis: branch frequencies of the inner A*'s per-neighbour loop (AStar.cpp:148-183) on cfg3
queries, from the oracle built with -DORC_BRANCH_STATS: valid neighbours, closed ones, find hits,
replacements, inserts, neighbours whose cell has an open node (the kernel's cell hint), pops, and
pops of an already-closed cell.  Guides the kernels' block-placement hints.

  python tools/branch_stats.py [query ids ...]
"""
import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
so = "/tmp/orc_branch.so"
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DORC_BRANCH_STATS", "-shared", "-o", so,
                str(ROOT / "oracle" / "hastar_oracle.cpp"), "-lm"], check=True)
import oracle.pyoracle as po  # noqa: E402
po.LIB = Path(so)
from tests.scenarios import drive, synthetic_ref  # noqa: E402

L = C.CDLL(so)
names = ["neighbours", "closed", "find_hit", "replace", "insert", "cell_has_open_node", "pops", "pop_of_closed_cell"]
st = (C.c_longlong * 8)()
for q in [int(a) for a in sys.argv[1:]] or [0, 1, 2, 3, 17, 101]:
    cfg, proto = synthetic_ref(1024, 72, 200, q + 1)
    o = po.OraclePlanner(cfg)
    drive(o, proto)
    o.find_path(proto["vel"], proto["start"])
    o.close()
    L.orc_branch_stats(st)
    d = {n: int(st[i]) for i, n in enumerate(names)}
    nc = max(d["neighbours"] - d["closed"], 1)
    d.update(p_closed=round(d["closed"] / max(d["neighbours"], 1), 3), p_hit_given_open=round(d["find_hit"] / nc, 3),
             p_insert_given_open=round(d["insert"] / nc, 3), p_cell_open_given_open=round(d["cell_has_open_node"] / nc, 3),
             p_replace_given_hit=round(d["replace"] / max(d["find_hit"], 1), 4),
             p_pop_closed=round(d["pop_of_closed_cell"] / max(d["pops"], 1), 4))
    print(json.dumps({"query": q, **d}), flush=True)
