"""Reeds-Shepp shortest paths, CPU restatement (TEST INFRASTRUCTURE: the checker of the relaxed
mode's device Reeds-Shepp code, path_planning_pkg_amd/csrc/hastar_rs.h; nothing in the product
path imports it).

The reference has no reversing motion model (lib/VehicleModel.cpp:97-101 expands forward arcs
only; include/path_planning_pkg/Dubins.h:13-19 is forward CSC Dubins), so there is no reference
code or fixture to pin this against: **parity unpinned**.  BASELINE.json configs[2] asks for
"Reeds-Shepp reversals enabled"; the relaxed (non-parity) mode offers them as an option.

The algorithm is the published one: J. A. Reeds and L. A. Shepp, "Optimal paths for a car that
goes both forwards and backwards", Pacific J. Math. 145(2), 1990 — formulas 8.1-8.11 for the
families CSC, CCC, CCCC, CCSC and CCSCC, each tried under the time-flip, reflection and
backwards symmetries (48 words), in the formulation popularised by OMPL's
ReedsSheppStateSpace (including its corrections of the paper's typos in 8.3/8.4 and 8.11).
Everything is in units of the turning radius: start at the origin heading 0, goal (x, y, phi).

The self-checks here are the ones that need no reference: every candidate word returned by any
family must integrate (segment by segment) to the goal, and the shortest word is no longer than
the forward-only Dubins path between the same poses.
"""
import math

PI = math.pi
ZERO = 1e-9
L_, S_, R_, N_ = 1, 0, -1, 2  # segment kinds: left, straight, right, none

# the 18 words (segment kinds), OMPL's reedsSheppPathType table order
WORDS = [
    (L_, R_, L_, N_, N_), (R_, L_, R_, N_, N_),
    (L_, R_, L_, R_, N_), (R_, L_, R_, L_, N_),
    (L_, R_, S_, L_, N_), (R_, L_, S_, R_, N_),
    (L_, S_, R_, L_, N_), (R_, S_, L_, R_, N_),
    (L_, R_, S_, R_, N_), (R_, L_, S_, L_, N_),
    (R_, S_, R_, L_, N_), (L_, S_, L_, R_, N_),
    (L_, S_, R_, N_, N_), (R_, S_, L_, N_, N_),
    (L_, S_, L_, N_, N_), (R_, S_, R_, N_, N_),
    (L_, R_, S_, L_, R_), (R_, L_, S_, R_, L_),
]


def mod2pi(x):
    v = math.fmod(x, 2 * PI)
    if v < -PI:
        v += 2 * PI
    elif v > PI:
        v -= 2 * PI
    return v


def polar(x, y):
    return math.hypot(x, y), math.atan2(y, x)


def tau_omega(u, v, xi, eta, phi):
    delta = mod2pi(u - v)
    A = math.sin(u) - math.sin(delta)
    B = math.cos(u) - math.cos(delta) - 1.0
    t1 = math.atan2(eta * A - xi * B, xi * A + eta * B)
    t2 = 2.0 * (math.cos(delta) - math.cos(v) - math.cos(u)) + 3.0
    tau = mod2pi(t1 + PI) if t2 < 0 else mod2pi(t1)
    omega = mod2pi(tau - u + v - phi)
    return tau, omega


# ---- the base formulas (each returns (t, u, v) or None) ------------------------------------
def LpSpLp(x, y, phi):  # 8.1
    u, t = polar(x - math.sin(phi), y - 1.0 + math.cos(phi))
    if t >= -ZERO:
        v = mod2pi(phi - t)
        if v >= -ZERO:
            return t, u, v
    return None


def LpSpRp(x, y, phi):  # 8.2
    u1, t1 = polar(x + math.sin(phi), y - 1.0 - math.cos(phi))
    u1 = u1 * u1
    if u1 >= 4.0:
        u = math.sqrt(u1 - 4.0)
        theta = math.atan2(2.0, u)
        t = mod2pi(t1 + theta)
        v = mod2pi(t - phi)
        if t >= -ZERO and v >= -ZERO:
            return t, u, v
    return None


def LpRmL(x, y, phi):  # 8.3 / 8.4
    xi, eta = x - math.sin(phi), y - 1.0 + math.cos(phi)
    u1, theta = polar(xi, eta)
    if u1 <= 4.0:
        u = -2.0 * math.asin(0.25 * u1)
        t = mod2pi(theta + 0.5 * u + PI)
        v = mod2pi(phi - t + u)
        if t >= -ZERO and u <= ZERO:
            return t, u, v
    return None


def LpRupLumRm(x, y, phi):  # 8.7
    xi, eta = x + math.sin(phi), y - 1.0 - math.cos(phi)
    rho = 0.25 * (2.0 + math.hypot(xi, eta))
    if rho <= 1.0:
        u = math.acos(rho)
        t, v = tau_omega(u, -u, xi, eta, phi)
        if t >= -ZERO and v <= ZERO:
            return t, u, v
    return None


def LpRumLumRp(x, y, phi):  # 8.8
    xi, eta = x + math.sin(phi), y - 1.0 - math.cos(phi)
    rho = (20.0 - xi * xi - eta * eta) / 16.0
    if 0.0 <= rho <= 1.0:
        u = -math.acos(rho)
        if u >= -0.5 * PI:
            t, v = tau_omega(u, u, xi, eta, phi)
            if t >= -ZERO and v >= -ZERO:
                return t, u, v
    return None


def LpRmSmLm(x, y, phi):  # 8.9
    xi, eta = x - math.sin(phi), y - 1.0 + math.cos(phi)
    rho, theta = polar(xi, eta)
    if rho >= 2.0:
        r = math.sqrt(rho * rho - 4.0)
        u = 2.0 - r
        t = mod2pi(theta + math.atan2(r, -2.0))
        v = mod2pi(phi - 0.5 * PI - t)
        if t >= -ZERO and u <= ZERO and v <= ZERO:
            return t, u, v
    return None


def LpRmSmRm(x, y, phi):  # 8.10
    xi, eta = x + math.sin(phi), y - 1.0 - math.cos(phi)
    rho, theta = polar(-eta, xi)
    if rho >= 2.0:
        t = theta
        u = 2.0 - rho
        v = mod2pi(t + 0.5 * PI - phi)
        if t >= -ZERO and u <= ZERO and v <= ZERO:
            return t, u, v
    return None


def LpRmSLmRp(x, y, phi):  # 8.11
    xi, eta = x + math.sin(phi), y - 1.0 - math.cos(phi)
    rho, theta = polar(xi, eta)
    if rho >= 2.0:
        u = 4.0 - math.sqrt(rho * rho - 4.0)
        if u <= ZERO:
            t = mod2pi(math.atan2((4.0 - u) * xi - 2.0 * eta, -2.0 * xi + (u - 4.0) * eta))
            v = mod2pi(t - phi)
            if t >= -ZERO and v >= -ZERO:
                return t, u, v
    return None


# ---- the 48 candidates: (word index, segment lengths) ---------------------------------------
def candidates(x, y, phi):
    """Every candidate of every family under the four symmetries (and the backwards ones), in
    the order the shortest-path search tries them."""
    out = []
    hp = 0.5 * PI
    xb = x * math.cos(phi) + y * math.sin(phi)
    yb = x * math.sin(phi) - y * math.cos(phi)
    # CSC
    for f, wa, wb in ((LpSpLp, 14, 15), (LpSpRp, 12, 13)):
        r = f(x, y, phi)
        if r: out.append((wa, (r[0], r[1], r[2])))
        r = f(-x, y, -phi)
        if r: out.append((wa, (-r[0], -r[1], -r[2])))
        r = f(x, -y, -phi)
        if r: out.append((wb, (r[0], r[1], r[2])))
        r = f(-x, -y, phi)
        if r: out.append((wb, (-r[0], -r[1], -r[2])))
    # CCC
    for xx, yy, back in ((x, y, False), (xb, yb, True)):
        for sx, sy, sp, w, sg in ((1, 1, 1, 0, 1), (-1, 1, -1, 0, -1), (1, -1, -1, 1, 1), (-1, -1, 1, 1, -1)):
            r = LpRmL(sx * xx, sy * yy, sp * phi)
            if r:
                t, u, v = r
                segs = (v, u, t) if back else (t, u, v)
                out.append((w, tuple(sg * s for s in segs)))
    # CCCC
    for sx, sy, sp, w, sg in ((1, 1, 1, 2, 1), (-1, 1, -1, 2, -1), (1, -1, -1, 3, 1), (-1, -1, 1, 3, -1)):
        r = LpRupLumRm(sx * x, sy * y, sp * phi)
        if r:
            t, u, v = r
            out.append((w, (sg * t, sg * u, -sg * u, sg * v)))
    for sx, sy, sp, w, sg in ((1, 1, 1, 2, 1), (-1, 1, -1, 2, -1), (1, -1, -1, 3, 1), (-1, -1, 1, 3, -1)):
        r = LpRumLumRp(sx * x, sy * y, sp * phi)
        if r:
            t, u, v = r
            out.append((w, (sg * t, sg * u, sg * u, sg * v)))
    # CCSC
    for f, wf, wr in ((LpRmSmLm, 4, 5), (LpRmSmRm, 8, 9)):
        for sx, sy, sp, refl, sg in ((1, 1, 1, False, 1), (-1, 1, -1, False, -1), (1, -1, -1, True, 1), (-1, -1, 1, True, -1)):
            r = f(sx * x, sy * y, sp * phi)
            if r:
                t, u, v = r
                out.append((wr if refl else wf, (sg * t, -sg * hp, sg * u, sg * v)))
    for f, wf, wr in ((LpRmSmLm, 6, 7), (LpRmSmRm, 10, 11)):
        for sx, sy, sp, refl, sg in ((1, 1, 1, False, 1), (-1, 1, -1, False, -1), (1, -1, -1, True, 1), (-1, -1, 1, True, -1)):
            r = f(sx * xb, sy * yb, sp * phi)
            if r:
                t, u, v = r
                out.append((wr if refl else wf, (sg * v, sg * u, -sg * hp, sg * t)))
    # CCSCC
    for sx, sy, sp, w, sg in ((1, 1, 1, 16, 1), (-1, 1, -1, 16, -1), (1, -1, -1, 17, 1), (-1, -1, 1, 17, -1)):
        r = LpRmSLmRp(sx * x, sy * y, sp * phi)
        if r:
            t, u, v = r
            out.append((w, (sg * t, -sg * hp, sg * u, -sg * hp, sg * v)))
    return out


def shortest(x, y, phi):
    """(length, word, segment lengths) of the shortest path in radius units, or None."""
    best = None
    for w, segs in candidates(x, y, phi):
        L = sum(abs(s) for s in segs)
        if best is None or L < best[0]:
            best = (L, w, segs)
    return best


def integrate(word, segs, x=0.0, y=0.0, h=0.0):
    """The end pose of a word's segments from (x, y, h), radius 1."""
    for kind, s in zip(WORDS[word], segs):
        if kind == L_:
            x, y, h = x + math.sin(h + s) - math.sin(h), y - math.cos(h + s) + math.cos(h), h + s
        elif kind == R_:
            x, y, h = x - math.sin(h - s) + math.sin(h), y + math.cos(h - s) - math.cos(h), h - s
        elif kind == S_:
            x, y = x + s * math.cos(h), y + s * math.sin(h)
    return x, y, h


def to_local(start, goal, r):
    """(x, y, phi) of `goal` in `start`'s frame, in units of the radius r."""
    dx, dy = goal[0] - start[0], goal[1] - start[1]
    c, s = math.cos(start[2]), math.sin(start[2])
    return (c * dx + s * dy) / r, (-s * dx + c * dy) / r, goal[2] - start[2]


def length(start, goal, r):
    """Shortest Reeds-Shepp length between two poses for turning radius r (metres)."""
    b = shortest(*to_local(start, goal, r))
    return b[0] * r


def sample(start, goal, r, step):
    """Poses every `step` metres along the shortest path (and its end), with each pose's
    direction of travel (+1 forward, -1 reverse): the shape the device's shot samples."""
    L, w, segs = shortest(*to_local(start, goal, r))
    x, y, h = start
    pts = [(x, y, h, 1 if segs[0] >= 0 else -1)]
    for kind, s in zip(WORDS[w], segs):
        if kind == N_ or s == 0.0:
            continue
        d = 1 if s >= 0 else -1
        n = max(1, int(math.ceil(abs(s) * r / step)))
        for k in range(1, n + 1):
            a = s * k / n
            if kind == L_:
                px, py, ph = x + r * (math.sin(h + a) - math.sin(h)), y + r * (-math.cos(h + a) + math.cos(h)), h + a
            elif kind == R_:
                px, py, ph = x + r * (-math.sin(h - a) + math.sin(h)), y + r * (math.cos(h - a) - math.cos(h)), h - a
            else:
                px, py, ph = x + r * a * math.cos(h), y + r * a * math.sin(h), h
            pts.append((px, py, ph, d))
        x, y, h = pts[-1][:3]
    return L * r, pts
