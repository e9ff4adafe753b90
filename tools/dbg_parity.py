"""Parity probe for debugging one library build: harness + small synthetic cases vs the oracle.
  HASTAR_LIB=<lib.so> python tools/dbg_parity.py"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle.pyoracle import OraclePlanner  # noqa: E402
from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, harness, synthetic  # noqa: E402

cases = [("harness", harness()[:2])] + [(f"syn256 s{s}", synthetic(256, 36, 10, s)) for s in (1, 2)] + \
        [("syn512 s1", synthetic(512, 72, 50, 1))]
for name, (cfg, proto) in cases:
    g, o = gpu.HybridAStar(cfg), OraclePlanner(cfg)
    for p in (g, o):
        drive(p, proto)
    rg, ro = g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"])
    bad = [k for k in ("pops", "successors", "astar_pops", "astar_searches", "shots", "closed_size", "pop_digest",
                       "closed_digest") if rg["stats"][k] != ro["stats"][k]]
    cb = np.float32(rg["cost"]).view(np.uint32) == np.float32(ro["cost"]).view(np.uint32)
    print(os.environ.get("HASTAR_LIB", "default"), name, "OK" if not bad and cb else f"MISMATCH {bad} cost_eq={cb}",
          {k: (rg["stats"][k], ro["stats"][k]) for k in ("pops", "successors", "astar_pops")}, flush=True)
