"""Debug probe: the replan-loop test's calls one by one (prints as it goes).
usage: dbg_relaxed.py REUSE"""
import ctypes as C, faulthandler, os, sys, threading, time
sys.path.insert(0, '.')
os.environ["HASTAR_RELAXED_PROGRESS"] = "1"
faulthandler.dump_traceback_later(60, exit=True)
from path_planning_pkg_amd import planner as gpu
from tests.scenarios import drive, replan_pairs, replan_tick, replan_tick_inputs
L = gpu.load_library()
L.hastar_debug_relaxed_progress.restype = C.POINTER(C.c_uint)


def watch():
    while True:
        time.sleep(8)
        p = L.hastar_debug_relaxed_progress()
        if p:
            print("progress", [[p[w * 4 + k] for k in range(4)] for w in range(8)], flush=True)


threading.Thread(target=watch, daemon=True).start()
reuse = int(sys.argv[1])
pairs = [replan_pairs(1024, 72, 200, 1, seed=1000 + q)[0] for q in range(4)]
gs = []
for cfg, proto, _ in pairs:
    g = gpu.HybridAStar(cfg)
    drive(g, proto)
    gs.append(g)
print("driven", flush=True)
for tick in range(3):
    starts = [replan_tick_inputs(proto, v, tick)[0] for _, proto, v in pairs]
    for k in range(4):
        t = time.time()
        r = gpu.find_path_batch([gs[k]], [pairs[k][1]["vel"]], [starts[k]], cap=16384,
                                relaxed=dict(reuse_heuristic=reuse))[0][0]
        print(tick, k, r["ok"], r["cost"], {q: r["stats"][q] for q in ("status", "pops", "shots", "pop_digest")},
              "%.2f s" % (time.time() - t), list(gs[k].cycles()[:8]), flush=True)
    for (cfg, proto, v), g in zip(pairs, gs):
        replan_tick(g, proto, v, tick)
