"""Pop census of a synthetic workload with the CPU oracle (test infrastructure; CPU only).

For query ids [start, start + count) of bench.py's generator (seed = id + 1) it records the
oracle's pops / astar_pops / success / wall time, with an optional pop limit so that
pathological queries end.  Used to size the device arenas and to find the queries that
outgrow them (tests/test_gpu_parity.py picks its long cases from this census).

    python tools/pop_census.py --grid 2048 --count 6144 --procs 6 --max-pops 2000000 > census.jsonl
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import Pool
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

ARGS = None


def one(q):
    from oracle import pyoracle
    from tests.scenarios import drive, synthetic, synthetic_ref
    pyoracle.set_max_pops(ARGS.max_pops)
    gen = synthetic_ref if ARGS.generator == "mt19937" else synthetic
    cfg, proto = gen(ARGS.grid, ARGS.bins, ARGS.obstacles, seed=q + 1)
    o = pyoracle.OraclePlanner(cfg)
    drive(o, proto)
    t0 = time.perf_counter()
    r = o.find_path(proto["vel"], proto["start"])
    wall = time.perf_counter() - t0
    o.close()
    st = r["stats"]
    return dict(q=q, pops=st["pops"], astar_pops=st["astar_pops"], successors=st["successors"], ok=r["ok"],
                status=st["status"], closed=st["closed_size"], wall_s=round(wall, 4))


def init(a):
    global ARGS
    ARGS = a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--bins", type=int, default=72)
    ap.add_argument("--obstacles", type=int, default=200)
    ap.add_argument("--start", type=int, default=0)
    ap.add_argument("--count", type=int, default=64)
    ap.add_argument("--max-pops", type=int, default=0)
    ap.add_argument("--procs", type=int, default=max(1, (os.cpu_count() or 2) - 2))
    ap.add_argument("--generator", choices=("mt19937", "pcg64"), default="mt19937")
    a = ap.parse_args()
    with Pool(a.procs, initializer=init, initargs=(a,)) as pool:
        for rec in pool.imap_unordered(one, range(a.start, a.start + a.count), chunksize=4):
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
