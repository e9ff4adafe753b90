"""Per-kernel counter table from rocprofv3 --pmc CSV output directories.

  python tools/pmc_table.py <out.json> <dir>... [--kernel-regex R]
Sums every counter per (kernel name, dispatch) over the directories' counter_collection.csv files
and writes {kernel: {dispatch_id: {counter: value}}}; prints one line per dispatch."""
import argparse
import csv
import json
import re
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("dirs", nargs="+")
ap.add_argument("--kernel-regex", default=".")
a = ap.parse_args()
tab = {}
for d in a.dirs:
    for f in sorted(Path(d).rglob("*counter_collection.csv")):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"]
                if not re.search(a.kernel_regex, k):
                    continue
                did = r.get("Dispatch_Id") or r.get("Correlation_Id") or "0"
                e = tab.setdefault(k, {}).setdefault(f"{Path(d).name}:{did}", {})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
Path(a.out).write_text(json.dumps(tab, indent=1))
for k, ds in tab.items():
    for did, cs in ds.items():
        print(k[:40], did, {c: round(v) for c, v in sorted(cs.items())})
