"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every
symbol include/hastar.h, hastar_f64.h, hastar_units.h and hastar_test.h declare, and refuses to run without a
GPU (no CPU fallback).  Also the libstdc++ red-black-tree replica used by the search
kernel vs std::set (tools/rbtree_check.cpp)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    names = []
    for hdr in ("hastar.h", "hastar_f64.h", "hastar_test.h", "hastar_units.h"):
        text = (ROOT / "include" / hdr).read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"\b(hastar(?:64)?_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_declared_symbols():
    from path_planning_pkg_amd.planner import LIB_PATH
    assert LIB_PATH.exists(), "build first (__graft_entry__.build())"
    lib = C.CDLL(str(LIB_PATH))
    syms = declared_symbols()
    assert "hastar_create_f32" in syms and "hastar_find_path_batch" in syms and "hastar64_find_path" in syms
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from path_planning_pkg_amd import HastarError, HybridAStar
    from tests.scenarios import harness
    cfg, _, _ = harness()
    with pytest.raises(HastarError) as e:
        HybridAStar(cfg)
    assert e.value.rc == -5
    from path_planning_pkg_amd.planner64 import HybridAStar64
    with pytest.raises(HastarError) as e:
        HybridAStar64(cfg)
    assert e.value.rc == -5


def test_rbtree_replica_matches_std_set(tmp_path):
    exe = tmp_path / "rbtree_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(ROOT / "path_planning_pkg_amd" / "csrc"),
                    str(ROOT / "tools" / "rbtree_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "100", "20000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK")


def test_deferred_tree_replay_builds_the_same_tree(tmp_path):
    """The deferred inner tree (hastar_kernels.hip, Pend / pend_replay): logged inserts (with
    their in-order neighbours) and erases, replayed at random points with the kernel's parent
    rule, give the tree the immediate operations give, link for link and colour for colour;
    freed indices are reused while their erase is still in the log (tools/rbtree_defer_check.cpp)."""
    exe = tmp_path / "rbtree_defer_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(ROOT / "path_planning_pkg_amd" / "csrc"),
                    str(ROOT / "tools" / "rbtree_defer_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "100", "20000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK")


def test_relaxed_entry_point_rejects_bad_arguments():
    """hastar_find_path_relaxed_batch validates its arguments before touching a device, and
    hastar_relaxed_opts has the C layout the ctypes mirror declares (nine 4-byte fields: round 6
    appended reverse_cost and gear_cost); so does the direction-returning entry point."""
    from path_planning_pkg_amd.capi import HastarRelaxedOpts
    from path_planning_pkg_amd.planner import load_library
    L = load_library()
    assert C.sizeof(HastarRelaxedOpts) == 36
    assert HastarRelaxedOpts.reverse_cost.offset == 28 and HastarRelaxedOpts.gear_cost.offset == 32
    f = (C.c_float * 3)()
    i = (C.c_int * 1)()
    rc = L.hastar_find_path_relaxed_batch(None, 0, f, f, f, f, 1, i, f, i, None, None)
    assert rc == -22  # HASTAR_EINVAL
    rc = L.hastar_find_path_relaxed_batch_dir(None, 0, f, f, f, f, None, 1, i, f, i, None, None)
    assert rc == -22


def test_route_score_cold_order_key():
    """hastar_test_route_score (the cold-order key of a planner with no history, host only)
    equals sum (1 + t) / (1 + d)^3 over the boxes, d = box-to-segment distance, t = the box centre's
    position along the route (0 at the start, 1 at the goal), on hand cases and on
    tests/scenarios.py:route_score (the bench's rank deal uses the same score)."""
    import numpy as np
    from path_planning_pkg_amd.planner import load_library
    from tests.scenarios import route_score
    L = load_library()
    L.hastar_test_route_score.restype = C.c_double
    fp = C.POINTER(C.c_float)

    def lib_score(boxes, s, g):
        b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 4)
        st, gl = np.asarray(s, np.float32), np.asarray(g, np.float32)
        return L.hastar_test_route_score(b.ctypes.data_as(fp), len(b), st.ctypes.data_as(fp), gl.ctypes.data_as(fp))

    # a box crossing the route half-way counts 1.5; one 3 m beside it 1.5/64; one 1 m beyond the
    # goal 2/8
    assert lib_score([[-5, 0, 2, 2]], [-10, 0], [0, 0]) == pytest.approx(1.5)
    assert lib_score([[-5, 4, 2, 2]], [-10, 0], [0, 0]) == pytest.approx(1.5 / 64)
    assert lib_score([[2, 0, 2, 2]], [-10, 0], [0, 0]) == pytest.approx(2 / 8)
    # a diagonal route passing a box corner at distance sqrt(2)/2, the centre a quarter along it
    assert lib_score([[1.5, -0.5, 1, 1]], [0, 0], [2, 2]) == pytest.approx(1.25 / (1 + 2 ** -0.5) ** 3)
    rng = np.random.default_rng(3)
    for _ in range(20):
        b = np.concatenate([rng.uniform(-60, 20, (30, 2)), rng.uniform(1, 6, (30, 2))], 1).astype(np.float32)
        s = rng.uniform(-60, 0, 2).astype(np.float32)
        g = rng.uniform(-10, 10, 2).astype(np.float32)
        assert lib_score(b, s, g) == pytest.approx(float(route_score(b[None], s, g)[0]), rel=1e-9)
