"""The drop-in C++ class (include/path_planning_pkg/HybridAStar.h) over the C ABI.

CPU: the header compiles and links against libhastar_amd.so.  GPU: the reference
harness scenario run through the class reproduces the oracle's result bit-for-bit and
the reference's golden path (utils/hybrid_astar/plot.py:46-51).
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "path_planning_pkg_amd" / "lib"


def _build(tmp_path):
    exe = tmp_path / "harness"
    cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off",
           f"-I{ROOT / 'include' / 'path_planning_pkg'}", str(ROOT / "tests" / "cxx" / "harness_main.cpp"),
           f"-L{LIB}", "-lhastar_amd", f"-Wl,-rpath,{LIB}", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_dropin_header_compiles_and_links(tmp_path):
    if not (LIB / "libhastar_amd.so").exists():
        pytest.skip("library not built")
    assert _build(tmp_path).exists()


@pytest.mark.gpu
def test_dropin_harness_matches_oracle_and_golden(tmp_path, oracle_lib):
    from tests.scenarios import drive, harness
    out = subprocess.run([str(_build(tmp_path))], check=True, capture_output=True, text=True, timeout=120).stdout
    lines = out.strip().splitlines()
    ok, cost_bits, n, rows = lines[0].split()
    assert int(rows) == 60
    pts = np.array([[int(v, 16) for v in ln.split()] for ln in lines[1:]], np.uint32)
    assert len(pts) == int(n)
    cfg, proto, g = harness()
    o = oracle_lib.OraclePlanner(cfg)
    drive(o, proto)
    r = o.find_path(proto["vel"], proto["start"])
    assert bool(int(ok)) == r["ok"]
    assert int(cost_bits, 16) == int(np.float32(r["cost"]).view(np.uint32))
    assert np.array_equal(pts[:, :3], np.asarray(r["path"], np.float32).view(np.uint32))
    assert np.array_equal(pts[:, 3], np.asarray(r["curvature"], np.float32).view(np.uint32))
    # the reference's printed path (start -> goal, 43 poses)
    mine = [[float("%g" % v) for v in row] for row in pts[::-1, :3].view(np.float32).astype(np.float64)]
    assert mine == g["path_start_to_goal"]


@pytest.mark.gpu
def test_dropin_harness_relaxed_mode(tmp_path):
    """The unchanged harness with $HASTAR_RELAXED=1: the class routes find_path to the relaxed
    (non-parity) mode; the result is a path from the goal end back to the harness start."""
    import os
    env = dict(os.environ, HASTAR_RELAXED="1")
    out = subprocess.run([str(_build(tmp_path))], check=True, capture_output=True, text=True, timeout=120,
                         env=env).stdout
    lines = out.strip().splitlines()
    ok, cost_bits, n, rows = lines[0].split()
    assert int(ok) == 1 and int(n) >= 2
    pts = np.array([[int(v, 16) for v in ln.split()] for ln in lines[1:]], np.uint32)[:, :3].view(np.float32)
    assert np.allclose(pts[-1, :2], [18.0, 18.0], atol=1e-3)  # the harness start (test_hybrid_astar.cpp)
    assert np.hypot(pts[0, 0] - 26.0, pts[0, 1] - 36.0) < 1.0  # ... and the goal end first


VG_MAIN = r"""
#include <cstdio>
#include "VelocityGenerator.h"
int main() {
  planning::VelocityGenerator<float> vg(12.f, 4.f, 2.5f, 1.5f, 3.f);
  std::vector<planning::Vector3D<float>> path{{2.f, 0.f, 0.f}, {1.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
  std::vector<float> curv{0.f, 0.1f, 0.f}, vel;
  bool ok = vg.generate_velocity_profile(1.f, 9.f, path, curv, vel, false, true);
  std::printf("%d", ok ? 1 : 0);
  for (float v : vel) std::printf(" %08x", *reinterpret_cast<unsigned*>(&v));
  std::printf("\n");
  return 0;
}
"""


def _build_vg(tmp_path):
    src, exe = tmp_path / "vg_main.cpp", tmp_path / "vg_main"
    src.write_text(VG_MAIN)
    cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off",
           f"-I{ROOT / 'include' / 'path_planning_pkg'}", str(src), f"-L{LIB}", "-lhastar_amd",
           f"-Wl,-rpath,{LIB}", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_velocity_generator_header_compiles_and_links(tmp_path):
    if not (LIB / "libhastar_amd.so").exists():
        pytest.skip("library not built")
    assert _build_vg(tmp_path).exists()


@pytest.mark.gpu
def test_velocity_generator_dropin_matches_oracle(tmp_path):
    from oracle import pyoracle
    out = subprocess.run([str(_build_vg(tmp_path))], check=True, capture_output=True, text=True,
                         timeout=120).stdout.split()
    xyh = np.array([[2, 0, 0], [1, 0, 0], [0, 0, 0]], np.float32)
    ok, v = pyoracle.velocity_profile((12, 4, 2.5, 1.5, 3), 1.0, 9.0, xyh, np.array([0, 0.1, 0], np.float32),
                                      False, True)
    assert int(out[0]) == int(ok)
    assert [int(t, 16) for t in out[1:]] == v.view(np.uint32).tolist()
