"""Relaxed-mode settings sweep on the GPU (hastar_find_path_relaxed_batch vs the exact mode).

  python tools/relaxed_sweep.py [--groups syn256,syn512,cfg3,cfg5] [--out file.json]

For each case group: the exact batch once (costs, ms), then the relaxed batch per setting
(delta, h_weight): batch ms, successes, cost ratio vs exact (mean / max), expansions, rounds.
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, replan_pairs, synthetic  # noqa: E402

# (delta, h_weight, h_stop, h_coarse)
SETTINGS = [(0.25, 1.2, 1.5, 2), (0.25, 1.2, 1.3, 2), (0.25, 1.2, 1.2, 2), (0.25, 1.35, 1.5, 2), (0.25, 1.35, 1.3, 2), (0.35, 1.2, 1.5, 2)]


def groups(names):
    out = {}
    if "syn256" in names:
        out["syn256"] = [synthetic(256, 36, 40, s) for s in (1, 2, 3, 4)]
    if "syn512" in names:
        out["syn512"] = [synthetic(512, 72, 50, s) for s in (1, 2)]
    if "cfg3" in names:
        out["cfg3"] = [synthetic(1024, 72, 200, seed=q + 1) for q in (0, 1, 2, 3, 10226)]
    if "cfg5" in names:
        out["cfg5"] = [tuple(replan_pairs(1024, 72, 200, 1, seed=1000 + q)[0][:2]) for q in range(8)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", default="syn256,syn512,cfg3,cfg5")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    gpu.load_library()
    rows = []
    for name, cases in groups(a.groups.split(",")).items():
        ps = []
        for cfg, proto in cases:
            p = gpu.HybridAStar(cfg)
            drive(p, proto)
            ps.append(p)
        vels = [p["vel"] for _, p in cases]
        starts = [p["start"] for _, p in cases]
        ex, ms_ex = gpu.find_path_batch(ps, vels, starts, cap=16384)
        print(json.dumps({"group": name, "mode": "exact", "ms": round(ms_ex, 2),
                          "ok": sum(r["ok"] for r in ex), "pops": [r["stats"]["pops"] for r in ex]}), flush=True)
        for d, w, hs, hc in SETTINGS:
            t0 = time.perf_counter()
            rel, ms = gpu.find_path_batch(ps, vels, starts, cap=16384, relaxed=dict(delta=d, h_weight=w, h_stop=hs, h_coarse=hc))
            wall = (time.perf_counter() - t0) * 1e3
            ratios = [r["cost"] / e["cost"] for r, e in zip(rel, ex) if r["ok"] and e["ok"]]
            row = {"group": name, "delta": d, "h_weight": w, "h_stop": hs, "h_coarse": hc, "ms": round(ms, 2), "wall_ms": round(wall, 2),
                   "ok": sum(r["ok"] for r in rel), "exact_ok": sum(e["ok"] for e in ex),
                   "status": sorted({r["stats"]["status"] for r in rel}),
                   "cost_ratio_mean": round(float(np.mean(ratios)), 4) if ratios else None,
                   "cost_ratio_max": round(float(np.max(ratios)), 4) if ratios else None,
                   "expansions": [r["stats"]["pops"] for r in rel],
                   "rounds": [r["stats"]["pop_digest"] for r in rel],
                   "dijkstra_cells": [r["stats"]["astar_pops"] for r in rel],
                   # per query: (clear + Dijkstra ms, search ms, Dijkstra buckets)
                   "split_ms": [(c[0] * 1e-5, c[1] * 1e-5, c[2]) for c in (p.cycles() for p in ps)]}
            rows.append(row)
            print(json.dumps(row), flush=True)
        for p in ps:
            p.close() if hasattr(p, "close") else None
    if a.out:
        Path(a.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
