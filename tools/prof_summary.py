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
    # hastar_reserve's empty warm-up launch (every wave exits at its first queue read) is not a step
    steps = [d for d in durs if d >= 1.0]
    timed = steps[args.warmup: args.warmup + args.steps]
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
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from path_planning_pkg_amd.buildinfo import search_kernel_hash
    out = {"kernel": KERNEL, "batch": args.batch, "grid": args.grid, "dispatch_index": i,
           "kernel_src_sha": search_kernel_hash(), "fetch_size_kib": f_kib, "write_size_kib": w_kib,
           "fetch_all_dispatches_kib": fetch, "write_all_dispatches_kib": write}
    if args.rdreq:
        # the L2's read requests to the fabric by size: their bytes are the calibrated read traffic
        # (tools/fetch_calib.hip, profiles/r05_fetch_calib.json: on gfx950 every L2 miss of a
        # narrow scattered load, like a wide streaming one, is one 128-B request, and FETCH_SIZE
        # tallies it at 64 B, so FETCH_SIZE reads exactly half of these bytes)
        n = {k: per_dispatch(args.rdreq, k)[i] for k in ("TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_64B_sum",
                                                         "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_sum")}
        rd = 128.0 * n["TCC_EA0_RDREQ_128B_sum"] + 64.0 * n["TCC_EA0_RDREQ_64B_sum"] + 32.0 * n["TCC_EA0_RDREQ_32B_sum"]
        out["rdreq"] = n
        out["read_bytes_calibrated"] = rd
        out["fetch_size_factor"] = rd / (f_kib * 1024.0)
        out["hbm_bytes_per_launch"] = rd + w_kib * 1024.0
        out["note"] = ("traffic = read bytes from the L2's fabric read requests by size (128 B x RDREQ_128B + 64 B x "
                       "RDREQ_64B + 32 B x RDREQ_32B; fetch_size_factor = those bytes / FETCH_SIZE, 2.00 on this "
                       "kernel as on the calibration patterns of tools/fetch_calib.hip) + WRITE_SIZE x 1024 B; "
                       "Infinity-Cache hits are counted (MI355X_MICROARCH.md §HBM)")
    else:
        out["hbm_bytes_per_launch"] = (2 * f_kib + w_kib) * 1024.0
        out["fetch_size_factor"] = 2.0
        out["note"] = ("traffic = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 B: the factor 2 is calibrated for this "
                       "kernel's narrow scattered loads by tools/fetch_calib.hip (profiles/r05_fetch_calib.json)")
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps({k: out[k] for k in ("fetch_size_kib", "write_size_kib", "hbm_bytes_per_launch", "fetch_size_factor")}))


def counters(args):
    """Every counter of the given rocprofv3 --pmc pass directories, summed over the search
    kernel's dispatch `--dispatch` (per-XCD / per-instance rows are added up)."""
    kern = args.kernel
    out = {"kernel": kern, "batch": args.batch, "grid": args.grid, "dispatch_index": args.dispatch, "counters": {}}
    for d in args.dirs:
        per = {}
        for r in rows(d, "counter_collection.csv"):
            if kern not in r["Kernel_Name"]:
                continue
            key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            per.setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
            per[r["Counter_Name"]][key] += float(r["Counter_Value"])
        for name, vals in per.items():
            ks = sorted(vals)
            out["counters"][name] = vals[ks[args.dispatch]]
    c = out["counters"]
    der = {}
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in c:
                der[k.lower() + "_frac_of_wave_cycles"] = c[k] / c["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
        der["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if c.get("SQC_ICACHE_HITS") is not None and c.get("SQC_ICACHE_MISSES") is not None:
        tot = c["SQC_ICACHE_HITS"] + c["SQC_ICACHE_MISSES"]
        if tot > 0:
            der["icache_hit_rate"] = c["SQC_ICACHE_HITS"] / tot
    if c.get("SQ_WAVES") and c.get("SQ_WAVE_CYCLES"):
        der["mean_wave_lifetime_cycles"] = 4.0 * c["SQ_WAVE_CYCLES"] / c["SQ_WAVES"]  # quad-cycles -> cycles
    insts = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                                        "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"))
    if insts:
        der["insts_counted"] = insts
    out["derived"] = der
    out["note"] = ("SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md); "
                   "WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES")
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(der))


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
p.add_argument("--rdreq", default=None, help="pass directory with TCC_EA0_RDREQ_{128B,64B,32B,}_sum")
p.add_argument("--batch", type=int, required=True)
p.add_argument("--grid", type=int, default=1024)
p.add_argument("--dispatch", type=int, default=-1)
c = sub.add_parser("counters")
c.add_argument("out")
c.add_argument("dirs", nargs="+")
c.add_argument("--batch", type=int, required=True)
c.add_argument("--grid", type=int, default=1024)
c.add_argument("--dispatch", type=int, default=1)
c.add_argument("--kernel", default=KERNEL, help="kernel name substring (default the batch kernel)")
a = ap.parse_args()
{"trace": trace, "pmc": pmc, "counters": counters}[a.cmd](a)
