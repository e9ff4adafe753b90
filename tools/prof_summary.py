"""Summarise rocprofv3 CSV output of a bench run into profiles/.

  python tools/prof_summary.py trace  <rocprof dir> <out.json> [--warmup W --steps K]
      kernel-trace: per-kernel stats, and the search-kernel dispatches of the timed
      steps (dispatches W .. W+K-1 of hastar_search_kernel) with their mean duration —
      the number bench.py's roofline.kernel_ms must agree with.
  python tools/prof_summary.py pmc <fetch dir> <write dir> <out.json> --batch B --grid N [--dispatch I]
      HBM traffic of one search-kernel dispatch from separate FETCH_SIZE / WRITE_SIZE
      passes (MI355X_MICROARCH.md §HBM: values in KiB; gfx950 FETCH_SIZE counts half the
      bytes of wide reads, so it is doubled).
"""
import argparse
import csv
import json
from pathlib import Path

KERNEL = "hastar_search_kernel"


def rows(d, suffix):
    out = []
    for f in sorted(Path(d).rglob(f"*{suffix}")):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def trace(args):
    kt = rows(args.dir, "kernel_trace.csv")
    disp = [r for r in kt if KERNEL in r["Kernel_Name"]]
    disp.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in disp]
    timed = durs[args.warmup: args.warmup + args.steps]
    stats = rows(args.dir, "kernel_stats.csv")
    out = {"kernel": KERNEL, "dispatches_ms": durs, "timed_dispatches_ms": timed,
           "timed_mean_ms": sum(timed) / len(timed) if timed else None,
           "kernel_stats": [{k: r[k] for k in r} for r in stats]}
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps({"timed_mean_ms": out["timed_mean_ms"], "n_dispatches": len(durs)}))


def pmc(args):
    def per_dispatch(d, name):
        vals = {}
        for r in rows(d, "counter_collection.csv"):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name:
                key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(vals))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
        return [vals[k] for k in sorted(vals)]
    fetch = per_dispatch(args.fetch, "FETCH_SIZE")
    write = per_dispatch(args.write, "WRITE_SIZE")
    i = args.dispatch
    f_kib, w_kib = fetch[i], write[i]
    out = {"kernel": KERNEL, "batch": args.batch, "grid": args.grid, "dispatch_index": i,
           "fetch_size_kib": f_kib, "write_size_kib": w_kib,
           "hbm_bytes_per_launch": (2 * f_kib + w_kib) * 1024.0,
           "note": "traffic = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 B per MI355X_MICROARCH.md §HBM; the search "
                   "kernel's loads are mostly narrow scattered accesses, for which the guide's gfx950 FETCH_SIZE "
                   "calibration is unverified",
           "fetch_all_dispatches_kib": fetch, "write_all_dispatches_kib": write}
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps({k: out[k] for k in ("fetch_size_kib", "write_size_kib", "hbm_bytes_per_launch")}))


ap = argparse.ArgumentParser()
sub = ap.add_subparsers(dest="cmd", required=True)
t = sub.add_parser("trace")
t.add_argument("dir")
t.add_argument("out")
t.add_argument("--warmup", type=int, default=1)
t.add_argument("--steps", type=int, default=3)
p = sub.add_parser("pmc")
p.add_argument("fetch")
p.add_argument("write")
p.add_argument("out")
p.add_argument("--batch", type=int, required=True)
p.add_argument("--grid", type=int, default=1024)
p.add_argument("--dispatch", type=int, default=-1)
a = ap.parse_args()
trace(a) if a.cmd == "trace" else pmc(a)
