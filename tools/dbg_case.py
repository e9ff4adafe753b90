"""Debug one parity case on the GPU with both search kernels (HASTAR_WIDE=1/0) against the
oracle: prints each side's stats.  Usage: python tools/dbg_case.py rowshard2048 | cfg3:<q>"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import pyoracle  # noqa: E402
from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, synthetic, synthetic_ref  # noqa: E402

what = sys.argv[1]
if what == "rowshard2048":
    cfg, proto = synthetic(2048, 36, 10, 7)
    proto["lines"] = np.array([[-60.0, -20.0, -20.0, 10.0], [-90.0, 30.0, -40.0, -30.0]], np.float32)
elif what.startswith("cfg3:"):
    cfg, proto = synthetic_ref(1024, 72, 200, int(what.split(":")[1]) + 1)
else:
    raise SystemExit("unknown case")
o = pyoracle.OraclePlanner(cfg)
drive(o, proto)
ro = o.find_path(proto["vel"], proto["start"])
keys = ("pops", "successors", "astar_pops", "astar_searches", "shots", "closed_size", "pop_digest", "astar_migrations")
print("oracle", ro["ok"], ro["cost"], {k: ro["stats"].get(k) for k in keys}, flush=True)
for wide, dbg in (("1", "0"), ("1", "1"), ("0", "0")):
    os.environ["HASTAR_WIDE"] = wide
    os.environ["HASTAR_WIDE_DBG"] = dbg
    g = gpu.HybridAStar(cfg)
    drive(g, proto)
    rg = g.find_path(proto["vel"], proto["start"])
    print("gpu wide=" + wide + " dbg=" + dbg, rg["ok"], rg["cost"], {k: rg["stats"].get(k) for k in keys}, flush=True)
    g.close()
