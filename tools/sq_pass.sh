#!/bin/bash
# usage: tools/sq_pass.sh <tag> <batch> <counters...>   (run on the GPU box; writes gpurun_out/sq_<tag>.txt)
tag=$1; batch=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf /tmp/sq_$tag
timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d /tmp/sq_$tag -o sq -- python3 tools/sq_probe.py --batch $batch > gpurun_out/sq_${tag}_run.txt 2>&1 || exit $?
python3 - "$tag" > gpurun_out/sq_$tag.txt <<'PY'
import csv, glob, sys
tag = sys.argv[1]
for f in glob.glob(f"/tmp/sq_{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "search" in r["Kernel_Name"]:
            print(r["Dispatch_Id"], r["Counter_Name"], r["Counter_Value"])
PY
