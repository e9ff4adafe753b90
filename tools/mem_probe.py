"""HBM cost of one planner: free device memory before/after creating n planners (cfg3 shape).
  python tools/mem_probe.py 256"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
torch.cuda.init()
f0, tot = torch.cuda.mem_get_info(0)
ps = []
for q in range(n):
    cfg, proto = synthetic(1024, 72, 200, q + 1)
    p = gpu.HybridAStar(cfg)
    if q == 0:
        f1, _ = torch.cuda.mem_get_info(0)
    drive(p, proto)
    ps.append(p)
torch.cuda.synchronize()
f2, _ = torch.cuda.mem_get_info(0)
print({"total_gib": tot / 2**30, "free0_gib": f0 / 2**30, "first_planner_mib": (f0 - f1) / 2**20,
       "per_planner_mib": (f0 - f2) / n / 2**20, "n": n})
