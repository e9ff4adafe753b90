"""MI355X-native Hybrid A* local planner (drop-in for planning::HybridAStar<float>).

The planner runs as HIP kernels on gfx950 behind the C ABI in include/hastar.h
(libhastar_amd.so, built in-tree by __graft_entry__.build()).
"""
from .capi import HastarParams, HastarStats, PlannerConfig, steering_from_degrees  # noqa: F401
from .planner import HybridAStar, HastarError, VelocityGenerator, find_path_batch, load_library  # noqa: F401
