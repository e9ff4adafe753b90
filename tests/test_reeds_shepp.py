"""The Reeds-Shepp restatement (oracle/reeds_shepp.py), the checker of the relaxed mode's
reversing model (csrc/hastar_rs.h).  The reference has no reversing model, so nothing pins
these against reference code ("parity unpinned"); the checks are the ones the geometry gives:

  * every candidate of every family, under every symmetry, integrates segment by segment to
    the goal (a wrong formula, sign or symmetry lands elsewhere);
  * all 18 words occur over random goals;
  * the shortest length is a metric: symmetric in its two poses, obeys the triangle inequality,
    and is never longer than the forward-only Dubins path between the same poses;
  * known values: a straight reverse of d costs d, a straight forward of d costs d.
"""
import math
import random

import pytest

from oracle import reeds_shepp as rs


def _dubins_forward(x, y, phi):
    """Shortest forward-only Dubins length (radius 1) by its CSC and CCC words (Shkel & Lumelsky),
    an upper bound the Reeds-Shepp length may not exceed."""
    d = math.hypot(x, y)
    th = math.atan2(y, x)
    a, b = rs.mod2pi(-th) % (2 * math.pi), rs.mod2pi(phi - th) % (2 * math.pi)
    sa, sb, ca, cb, cab = math.sin(a), math.sin(b), math.cos(a), math.cos(b), math.cos(a - b)
    best = math.inf
    m = lambda v: v % (2 * math.pi)  # noqa: E731
    p2 = 2 + d * d - 2 * cab + 2 * d * (sa - sb)  # LSL
    if p2 >= 0:
        t = math.atan2(cb - ca, d + sa - sb)
        best = min(best, m(-a + t) + math.sqrt(p2) + m(b - t))
    p2 = 2 + d * d - 2 * cab + 2 * d * (sb - sa)  # RSR
    if p2 >= 0:
        t = math.atan2(ca - cb, d - sa + sb)
        best = min(best, m(a - t) + math.sqrt(p2) + m(-b + t))
    p2 = -2 + d * d + 2 * cab + 2 * d * (sa + sb)  # LSR
    if p2 >= 0:
        p = math.sqrt(p2)
        t = math.atan2(-ca - cb, d + sa + sb) - math.atan2(-2, p)
        best = min(best, m(-a + t) + p + m(-b + t))
    p2 = -2 + d * d + 2 * cab - 2 * d * (sa + sb)  # RSL
    if p2 >= 0:
        p = math.sqrt(p2)
        t = math.atan2(ca + cb, d - sa - sb) - math.atan2(2, p)
        best = min(best, m(a - t) + p + m(b - t))
    v = (6 - d * d + 2 * cab + 2 * d * (sa - sb)) / 8  # RLR
    if abs(v) <= 1:
        p = m(2 * math.pi - math.acos(v))
        t = m(a - math.atan2(ca - cb, d - sa + sb) + p / 2)
        best = min(best, t + p + m(a - b - t + p))
    v = (6 - d * d + 2 * cab + 2 * d * (-sa + sb)) / 8  # LRL
    if abs(v) <= 1:
        p = m(2 * math.pi - math.acos(v))
        t = m(-a - math.atan2(ca - cb, d + sa - sb) + p / 2)
        best = min(best, t + p + m(m(b) - a - t + p))
    return best


def test_every_candidate_reaches_the_goal():
    rng = random.Random(1)
    words = set()
    n = 0
    for _ in range(6000):
        x, y, phi = rng.uniform(-8, 8), rng.uniform(-8, 8), rng.uniform(-math.pi, math.pi)
        cands = rs.candidates(x, y, phi)
        assert cands, (x, y, phi)
        for w, segs in cands:
            ex, ey, eh = rs.integrate(w, segs)
            assert max(abs(ex - x), abs(ey - y), abs(rs.mod2pi(eh - phi))) < 1e-7, (w, segs, x, y, phi)
            words.add(w)
            n += 1
    assert words == set(range(18)), sorted(set(range(18)) - words)
    assert n > 30000


def test_metric_properties_and_known_values():
    rng = random.Random(2)
    P = lambda: (rng.uniform(-6, 6), rng.uniform(-6, 6), rng.uniform(-math.pi, math.pi))  # noqa: E731
    for _ in range(2000):
        a, b, c = P(), P(), P()
        dab, dba = rs.length(a, b, 1.0), rs.length(b, a, 1.0)
        assert abs(dab - dba) < 1e-9
        assert rs.length(a, c, 1.0) <= dab + rs.length(b, c, 1.0) + 1e-9
    for d in (0.5, 3.0, 17.0):
        assert rs.length((0, 0, 0), (-d, 0, 0), 1.0) == pytest.approx(d, abs=1e-12)
        assert rs.length((0, 0, 0), (d, 0, 0), 2.5) == pytest.approx(d, abs=1e-12)


def test_never_longer_than_forward_dubins():
    rng = random.Random(3)
    for _ in range(3000):
        x, y, phi = rng.uniform(-10, 10), rng.uniform(-10, 10), rng.uniform(-math.pi, math.pi)
        L = rs.shortest(x, y, phi)[0]
        assert L <= _dubins_forward(x, y, phi) + 1e-9


def test_sampling_is_continuous_and_ends_at_the_goal():
    rng = random.Random(4)
    for _ in range(200):
        s = (rng.uniform(-20, 20), rng.uniform(-20, 20), rng.uniform(-math.pi, math.pi))
        g = (rng.uniform(-20, 20), rng.uniform(-20, 20), rng.uniform(-math.pi, math.pi))
        L, pts = rs.sample(s, g, 4.0, 0.5)
        assert pts[0][:3] == s
        assert math.hypot(pts[-1][0] - g[0], pts[-1][1] - g[1]) < 1e-7
        assert abs(rs.mod2pi(pts[-1][2] - g[2])) < 1e-7
        assert max(math.hypot(b[0] - a[0], b[1] - a[1]) for a, b in zip(pts, pts[1:])) <= 0.5 + 1e-9
        assert L == pytest.approx(rs.length(s, g, 4.0))
