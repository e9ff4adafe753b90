"""Single-query phase breakdown of the search kernel (diagnostic build with -DHASTAR_STAMPS).

  HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so python tools/profile_search.py --grid 1024 --seeds 1 3
Prints pops, A* pops, kernel ms, and the share of s_memtime cycles per phase
(0 pop+closed insert, 1 successors+APF+Dubins, 2 open/closed bookkeeping excl. A*,
3 holonomic A*, 4 Dubins shot, 5 reconstruct+stats, 6 whole loop).
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, synthetic, synthetic_ref  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=1024)
ap.add_argument("--bins", type=int, default=72)
ap.add_argument("--obstacles", type=int, default=200)
ap.add_argument("--seeds", type=int, nargs="+", default=[1])
ap.add_argument("--generator", choices=["pcg64", "mt19937"], default="mt19937")
ap.add_argument("--replan", action="store_true", help="profile the bench step: find_path, reset, find_path")
ap.add_argument("--cfg5-pairs", type=int, nargs="*", default=None,
                help="profile cfg5 replan loops instead (pair ids, bench.py --workload cfg5): every tick's search, "
                     "summed over --ticks ticks (the latency kernel)")
ap.add_argument("--ticks", type=int, default=6)
ap.add_argument("--skip-ticks", type=int, default=0, help="cfg5: run but do not sum the first ticks (cold memo)")
args = ap.parse_args()
names = ["pop", "expand", "open_bookkeeping", "astar", "shot", "reconstruct", "loop", "astar_hbm_mode"]
def cfg5_runs(pair):
    """one cfg5 pair's replan loop (no reset between ticks); yields per tick (planner, stats, ms)"""
    from tests.scenarios import replan_pairs, replan_tick_inputs
    cfg, proto, v = replan_pairs(args.grid, args.bins, args.obstacles, 1, seed=1000 + pair)[0]
    p = gpu.HybridAStar(cfg)
    drive(p, proto)
    for t in range(args.ticks):
        start, _ = replan_tick_inputs(proto, v, t)
        res, ms = gpu.find_path_batch([p], [proto["vel"]], [start])
        yield p, res[0]["stats"], ms
        _, boxes = replan_tick_inputs(proto, v, t + 1)
        p.decay()
        p.update_boxes(boxes, [proto["box_conf"]] * len(boxes), proto["apf_r"])


def runs():
    if args.cfg5_pairs is not None:
        for pair in args.cfg5_pairs:
            tot, stt, mss = None, None, 0.0
            for t, (p, st, ms) in enumerate(cfg5_runs(pair)):
                if t < args.skip_ticks:
                    continue
                cyc = p.cycles()
                tot = list(cyc) if tot is None else [a + b for a, b in zip(tot, cyc)]
                stt = dict(st) if stt is None else {k: stt[k] + st[k] if isinstance(st[k], int) and k not in
                                                    ("pop_digest", "closed_digest", "status") else st[k] for k in st}
                mss += ms
            yield f"cfg5 pair {pair} ticks {args.skip_ticks}..{args.ticks - 1}", p, tot, stt, mss
        return
    for s in args.seeds:
        gen = synthetic_ref if args.generator == "mt19937" else synthetic
        cfg, proto = gen(args.grid, args.bins, args.obstacles, s)
        p = gpu.HybridAStar(cfg)
        drive(p, proto)
        if args.replan:
            gpu.find_path_batch([p], [proto["vel"]], [proto["start"]])
            p.reset()
        res, ms = gpu.find_path_batch([p], [proto["vel"]], [proto["start"]])
        yield s, p, p.cycles(), res[0]["stats"], ms


for s, p, cyc, st, ms in runs():
    loop = max(cyc[6], 1)
    share = {names[i]: round(cyc[i] / loop, 4) for i in range(6)}
    share["open_bookkeeping"] = round((cyc[2] - cyc[3]) / loop, 4)
    share["astar_hbm_mode"] = round(cyc[7] / loop, 4)
    modes = p.astar_modes()
    print(json.dumps(dict(seed=s, kernel_ms=ms, pops=st["pops"], astar_pops=st["astar_pops"],
                          astar_searches=st["astar_searches"], successors=st["successors"],
                          loop_cycles=cyc[6], cycles_per_pop=cyc[6] / max(st["pops"], 1), share=share, **modes,
                          cyc_per_apop_lds=(cyc[3] - cyc[7]) / max(st["astar_pops"] - modes["astar_pops_hbm"], 1),
                          cyc_per_apop_hbm=cyc[7] / max(modes["astar_pops_hbm"], 1),
                          lds_astar_per_apop={n: round(cyc[8 + i] / max(st["astar_pops"] - modes["astar_pops_hbm"], 1))
                                              for i, n in enumerate(["pop_probe", "find", "insert", "unlink_hit",
                                                                     "memoise"])},
                          lds_astar_parts_per_apop={n: round(cyc[i] / max(st["astar_pops"] - modes["astar_pops_hbm"], 1))
                                                    for i, n in ((24, "pop_unlink"), (25, "insert_link"),
                                                                 (30, "ring_insert"), (31, "expansion_stores"),
                                                                 (32, "neighbour_loop"), (33, "lane_precompute"),
                                                                 (34, "replace_path"))},
                          astar_setup_per_search=round(cyc[35] / max(st["astar_searches"], 1)),
                          prep={"taken": cyc[36], "computed_here": cyc[37]},
                          pop_prefetch={"hit": cyc[38], "miss": cyc[39]},
                          outer_per_pop={n: round(cyc[13 + i] / max(st["pops"], 1))
                                         for i, n in enumerate(["find3", "insert3", "unlink3", "succ_gen", "apf",
                                                                "dubins", "insert_walk", "insert_link",
                                                                "probe_wait"])},
                          outer_tree={"fills_per_pop": cyc[22] / max(st["pops"], 1),
                                      "walk_steps_per_pop": cyc[23] / max(st["pops"], 1),
                                      "cycles_per_fill": cyc[26] / max(cyc[22], 1),
                                      "prior_ops_wait_per_fill": cyc[27] / max(cyc[22], 1),
                                      "path_walk_per_pop": cyc[28] / max(st["pops"], 1),
                                      "path_walk_ins_per_pop": cyc[29] / max(st["pops"], 1)})))
