import sys, numpy as np
sys.path.insert(0, '.')
from path_planning_pkg_amd import planner as gpu
from tests.scenarios import synthetic_ref, drive
cases = [synthetic_ref(256, 36, 10, s) for s in (1, 2, 3, 4)]
gs = []
for cfg, proto in cases:
    g = gpu.HybridAStar(cfg); drive(g, proto); gs.append(g)
br = gpu.find_path_batch_arrays(gs, [p["vel"] for _, p in cases], [p["start"] for _, p in cases])
for g in gs:
    c = g.cycles(); t = g.timing()
    print(c[36:40], t, int(br.stats["parks"][0]))
