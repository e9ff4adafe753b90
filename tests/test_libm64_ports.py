"""The double planner's libm (path_planning_pkg_amd/csrc/hastar_libm64.h) against this host's
glibc 2.35, on the host (CPU test; tools/libm64_fingerprint.hip runs the same comparison on the
device, `-m gpu` in test_gpu_f64.py).

sin, cos, atan2, acos and hypot are ports of glibc's routines (the FMA variants the x86-64 libm
dispatches to) and must match bit for bit.
Arguments: the planner's ranges (headings and arc sums, centre and obstacle offsets in metres,
2 r / dist) plus edge cases."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "path_planning_pkg_amd" / "csrc"

SRC = r"""
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <cmath>
#include <cfloat>
#include "hastar_libm64.h"
static inline uint64_t mix64(uint64_t z) { z += 0x9e3779b97f4a7c15ull; z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull; return z ^ (z >> 31); }
static inline double unit(uint64_t b) { return (double)(b >> 11) * 0x1.0p-53; }
static double H(int f, double a, double b) { return f == 0 ? std::sin(a) : f == 1 ? std::cos(a) : f == 2 ? std::atan2(a, b)
  : f == 3 ? std::acos(a) : std::hypot(a, b); }
static double G(int f, double a, double b) { return f == 0 ? gm64::sin(a) : f == 1 ? gm64::cos(a) : f == 2 ? gm64::atan2(a, b)
  : f == 3 ? gm64::acos(a) : gm64::hypot(a, b); }
int main(int argc, char** argv) {
  const long n = atol(argv[1]);
  const double edge[] = {0.0, -0.0, 1e-300, -1e-300, 0x1p-1030, 1.0, -1.0, 0.5, 3.141592653589793, -3.141592653589793,
                         1.5707963267948966, 2.426265, 0.855469, 0.126, 1e5, 1e300, -1e300, INFINITY, -INFINITY, NAN};
  for (int f = 0; f < 5; ++f) {
    long mm = 0;
    for (double a : edge) for (double b : edge) {
      const double r = H(f, a, b), g = G(f, a, b);
      if (memcmp(&r, &g, 8) && !(std::isnan(r) && std::isnan(g))) ++mm;
    }
    for (long i = 0; i < n; ++i) {
      const double u = unit(mix64(2 * i + 7919 * f)), v = unit(mix64(2 * i + 1 + 7919 * f));
      double a, b = 0;
      if (f < 2) a = (i & 1) ? (u * 2 - 1) * 3.141592653589793 : (u * 2 - 1) * 10.0;
      else if (f == 3) a = (i & 1) ? u : u * 2 - 1;
      else { const double s = (i & 3) == 0 ? 3.0 : 300.0; a = (u * 2 - 1) * s; b = (v * 2 - 1) * s; }
      const double r = H(f, a, b), g = G(f, a, b);
      if (memcmp(&r, &g, 8)) ++mm;
    }
    printf("%d %ld\n", f, mm);
  }
}
"""


def _host_is_glibc235_x86_fma():
    """The ports (and the tables read from libm.so.6) are glibc 2.35's x86-64 FMA variants: on
    another glibc, a non-x86 host or a CPU without FMA the host libm runs other code, and a
    comparison with it would measure that difference, not the ports."""
    import ctypes
    import platform
    if platform.machine() not in ("x86_64", "AMD64"):
        return False, f"host is {platform.machine()}, not x86-64"
    try:
        libc = ctypes.CDLL("libc.so.6")
        libc.gnu_get_libc_version.restype = ctypes.c_char_p
        ver = libc.gnu_get_libc_version().decode()
    except (OSError, AttributeError):
        return False, "not glibc"
    if ver != "2.35":
        return False, f"glibc {ver}, the ports are of 2.35"
    try:
        flags = Path("/proc/cpuinfo").read_text()
    except OSError:
        return False, "no /proc/cpuinfo"
    if " fma" not in flags:
        return False, "CPU without FMA (glibc dispatches to its non-FMA variants)"
    return True, ""


@pytest.fixture(scope="module")
def ports(tmp_path_factory):
    ok, why = _host_is_glibc235_x86_fma()
    if not ok:
        pytest.skip(why)
    d = tmp_path_factory.mktemp("libm64")
    (d / "t.cpp").write_text(SRC)
    exe = d / "t"
    # -ffp-contract=off: only the explicit fma() calls fuse, as in the device build
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", f"-I{CSRC}", str(d / "t.cpp"), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe), "400000"], check=True, capture_output=True, text=True).stdout.split("\n")
    return {int(a): int(b) for a, b in (line.split() for line in out if line.strip())}


@pytest.mark.parametrize("fn,name", [(0, "sin"), (1, "cos"), (2, "atan2"), (3, "acos"), (4, "hypot")])
def test_glibc_ports_bit_exact(ports, fn, name):
    assert ports[fn] == 0, f"{name}: {ports[fn]} mismatches with the host glibc"
