"""glibc 2.35 float libm ports (path_planning_pkg_amd/csrc/glibc_mathf.h) vs the live glibc.

The device search kernel calls these ports; the reference calls glibc.  This test builds
tools/mathf_exhaustive.cpp on the host and sweeps every float in the ranges the planner
reaches (sinf/cosf on [-8, 8], acosf on [-1, 1], atanf on [-64, 64]) plus 2^24 sampled
atan2f/hypotf pairs; tests/golden/mathf_sweep_all.txt is the committed full 2^32 sweep.
Needs a host whose sinf/cosf IFUNC picks the FMA variant (both this container and the GPU
box: x86-64 with FMA+AVX2).
"""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _has_fma():
    try:
        flags = Path("/proc/cpuinfo").read_text()
    except OSError:
        return False
    return " fma " in flags and " avx2 " in flags


@pytest.mark.skipif(not _has_fma(), reason="glibc picks the non-FMA sinf/cosf variant on this host")
def test_ports_match_glibc(tmp_path):
    exe = tmp_path / "mathf_exhaustive"
    subprocess.run(["g++", "-O2", "-mfma", "-ffp-contract=off", "-fopenmp", "-I",
                    str(ROOT / "path_planning_pkg_amd" / "csrc"), str(ROOT / "tools" / "mathf_exhaustive.cpp"),
                    "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe), "fast", str(1 << 24)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "TOTAL mismatches=0" in out.stdout


def test_full_sweep_record_is_clean():
    rec = (ROOT / "tests" / "golden" / "mathf_sweep_all.txt").read_text()
    assert "TOTAL mismatches=0" in rec
    for fn in ("sinf", "cosf", "acosf", "atanf"):
        assert f"{fn}     inputs=4294967296 mismatches=0" in rec or f"{fn}    inputs=4294967296 mismatches=0" in rec
