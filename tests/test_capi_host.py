"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every
symbol include/hastar.h, include/hastar_units.h and include/hastar_test.h declare, and refuses to run without a
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
    for hdr in ("hastar.h", "hastar_test.h", "hastar_units.h"):
        text = (ROOT / "include" / hdr).read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"\b(hastar_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_declared_symbols():
    from path_planning_pkg_amd.planner import LIB_PATH
    assert LIB_PATH.exists(), "build first (__graft_entry__.build())"
    lib = C.CDLL(str(LIB_PATH))
    syms = declared_symbols()
    assert "hastar_create_f32" in syms and "hastar_find_path_batch" in syms
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


def test_rbtree_replica_matches_std_set(tmp_path):
    exe = tmp_path / "rbtree_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(ROOT / "path_planning_pkg_amd" / "csrc"),
                    str(ROOT / "tools" / "rbtree_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "100", "20000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK")


def test_relaxed_entry_point_rejects_bad_arguments():
    """hastar_find_path_relaxed_batch validates its arguments before touching a device, and
    hastar_relaxed_opts has the C layout the ctypes mirror declares (seven 4-byte fields)."""
    from path_planning_pkg_amd.capi import HastarRelaxedOpts
    from path_planning_pkg_amd.planner import load_library
    L = load_library()
    assert C.sizeof(HastarRelaxedOpts) == 28
    f = (C.c_float * 3)()
    i = (C.c_int * 1)()
    rc = L.hastar_find_path_relaxed_batch(None, 0, f, f, f, f, 1, i, f, i, None, None)
    assert rc == -22  # HASTAR_EINVAL
