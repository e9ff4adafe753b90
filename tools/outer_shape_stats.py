"""Analysis: how often does the OUTER open set's tree SHAPE decide a find / insert
(HybridAStar.cpp:159-193)?  The oracle built with -DORC_OUTER_STATS replays synthetic cfg3
seeds and cfg5 replan loops; per search it counts the open-set finds, those with a node of the
same key present, "unsafe" finds (a same-key node with f < the probe g: the lower_bound walk
is then shape-dependent), inserts, unsafe inserts (a same-key node with f > the new f), cases
with several same-key nodes, pops, the pops before a search's first such event, the largest
open set and the finds whose probe lies beyond the leftmost node.  A deferred outer tree
(built only at such events) pays a replay at each event.

  python tools/outer_shape_stats.py [cfg3 seeds ...] [--cfg5 pair ...]
"""
import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
so = "/tmp/orc_outer.so"
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DORC_OUTER_STATS", "-shared", "-o", so,
                str(ROOT / "oracle" / "hastar_oracle.cpp"), "-lm"], check=True)
import oracle.pyoracle as po  # noqa: E402
po.LIB = Path(so)
from tests.scenarios import drive, replan_pairs, replan_tick, replan_tick_inputs, synthetic_ref  # noqa: E402

L = C.CDLL(so)
names = ["finds", "same_key_present", "unsafe_find", "inserts", "unsafe_insert", "several_same_key", "pops",
         "pops_before_first_event", "max_open", "finds_beyond_leftmost", "searches", "searches_with_event"]
argv = sys.argv[1:]
cfg5 = []
if "--cfg5" in argv:
    i = argv.index("--cfg5")
    cfg5 = [int(a) for a in argv[i + 1:]]
    argv = argv[:i]
seeds = [int(a) for a in argv]
st = (C.c_longlong * 16)()


def dump(tag):
    L.orc_outer_stats(st)
    d = {n: int(st[i]) for i, n in enumerate(names)}
    ev = d["unsafe_find"] + d["unsafe_insert"] + d["several_same_key"]
    d["events_per_1k_pops"] = round(1000 * ev / max(d["pops"], 1), 3)
    print(json.dumps({"case": tag, **d}), flush=True)


for s in seeds:
    cfg, proto = synthetic_ref(1024, 72, 200, s)
    o = po.OraclePlanner(cfg)
    drive(o, proto)
    L.orc_outer_stats(st)
    o.find_path(proto["vel"], proto["start"])
    dump(f"cfg3 seed {s}")
for q in cfg5:
    cfg, proto, v = replan_pairs(1024, 72, 200, 1, seed=1000 + q)[0]
    o = po.OraclePlanner(cfg)
    drive(o, proto)
    L.orc_outer_stats(st)
    for t in range(8):
        o.find_path(proto["vel"], replan_tick_inputs(proto, v, t)[0])
        replan_tick(o, proto, v, t)
    dump(f"cfg5 pair {q} ticks 0-7")
