"""VelocityGenerator<float>: GPU kernel vs the CPU oracle.

The reference holds no golden vectors for VelocityGenerator.cpp, so the oracle's
restatement (oracle/hastar_oracle.cpp::orc_velocity_profile) is cross-checked here against
a second, independent numpy restatement of VelocityGenerator.cpp:19-84; the GPU path is
then compared with the oracle bit for bit (NaN compared as NaN: negative curvature or a
lateral acceleration above the limit makes the reference's sqrt return NaN, and the NaN
payload is not part of the contract).
"""
import numpy as np
import pytest

from oracle import pyoracle
from tests.scenarios import drive, harness

PARAMS = (12.0, 4.0, 2.5, 1.5, 3.0)  # max_velocity, coast_velocity, max_lat_acc, max_long_acc, max_long_dec


def numpy_profile(params, vel_init, vmax_curr, xyh, curv, coast, stop):
    """VelocityGenerator.cpp:19-84 with numpy scalars (T = float32; `1.0 - x` is float64)."""
    f = np.float32
    vmax_p, vcoast, a_lat, a_acc, a_dec = (f(p) for p in params)
    a_lat2 = f(a_lat * a_lat)
    X = np.asarray(xyh, np.float32).reshape(-1, 3)
    K = np.asarray(curv, np.float32)
    n = len(X)
    vel_init, vmax_curr = f(vel_init), f(vmax_curr)
    smin = lambda a, b: b if b < a else a  # noqa: E731  std::min / std::max, NaN-faithful
    smax = lambda a, b: b if a < b else a  # noqa: E731
    vm = vcoast if coast else vmax_p
    vm = smin(vm, vmax_curr)
    vm2 = f(vm * vm)
    vsq = np.zeros(n, np.float32)
    vel = np.zeros(n, np.float32)
    vsq[0] = vel_init * vel_init
    cur = vsq[0]

    def step(a, b):
        return np.hypot(f(X[a, 0] - X[b, 0]), f(X[a, 1] - X[b, 1]))

    def rem(acc, v2, k):
        lat = f(v2 * k)
        return f(np.float64(acc) * np.sqrt(np.float64(1.0) - np.float64(f(f(lat * lat) / a_lat2))))

    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        for i in range(n - 1):
            pi = n - i - 1
            a = f(cur - f(f(f(2) * rem(a_dec, vsq[i], K[pi])) * step(pi - 1, pi)))
            cur = smax(a, vm2)
            if K[pi - 1] != 0:
                q = f(a_lat / K[pi - 1])
                vsq[i + 1] = smin(q, cur)
            else:
                vsq[i + 1] = cur
        if stop:
            vsq[n - 1] = 0
        for i in range(n - 1):
            pi = n - i - 1
            a = f(vsq[i] + f(f(f(2) * rem(a_acc, vsq[i], K[pi])) * step(pi - 1, pi)))
            vsq[i + 1] = smin(a, vsq[i + 1])
        for i in range(n - 1, 0, -1):
            pi = n - i - 1
            a = f(vsq[i] + f(f(f(2) * rem(a_dec, vsq[i], K[pi])) * step(pi + 1, pi)))
            vsq[i - 1] = smin(a, vsq[i - 1])
            vel[i - 1] = np.sqrt(vsq[i - 1])
        vel[n - 1] = np.sqrt(vsq[n - 1])
    return bool(vel_init < f(vel[0] + f(0.25))), vel


def bits(a):
    a = np.ascontiguousarray(a, np.float32)
    b = a.view(np.uint32).copy()
    b[np.isnan(a)] = 0x7FC00000
    return b


def random_cases(seed, count, signed=False):
    rng = np.random.default_rng(seed)
    cases = []
    for c in range(count):
        n = int(rng.choice([1, 2, 3, 17, 64, 300]))
        h = np.cumsum(rng.uniform(-0.2, 0.2, n)).astype(np.float32)
        xy = np.cumsum(np.stack([np.cos(h), np.sin(h)], 1) * rng.uniform(0.05, 0.6), 0).astype(np.float32)
        xyh = np.concatenate([xy, h[:, None]], 1).astype(np.float32)
        k = rng.uniform(-0.3 if signed else 0.0, 0.3, n).astype(np.float32)
        k[rng.random(n) < 0.3] = 0.0
        cases.append(dict(xyh=xyh, curv=k, v0=float(rng.uniform(0, 8)), vmax=float(rng.uniform(1, 15)),
                          coast=bool(rng.random() < 0.5), stop=bool(rng.random() < 0.5)))
    return cases


def test_oracle_matches_numpy_restatement():
    for case in random_cases(7, 60, signed=True):
        ok_o, vo = pyoracle.velocity_profile(PARAMS, case["v0"], case["vmax"], case["xyh"], case["curv"],
                                             case["coast"], case["stop"])
        ok_n, vn = numpy_profile(PARAMS, case["v0"], case["vmax"], case["xyh"], case["curv"], case["coast"],
                                 case["stop"])
        assert ok_o == ok_n
        assert (bits(vo) == bits(vn)).all(), (vo, vn)


def test_oracle_hand_case():
    """Straight 3-point path, no curvature: v² grows by 2·a·s per metre forward and the
    stop-at-goal braking gives v² = 2·d·s backward (VelocityGenerator.cpp:54-76)."""
    xyh = np.array([[2, 0, 0], [1, 0, 0], [0, 0, 0]], np.float32)  # goal -> start
    ok, v = pyoracle.velocity_profile((10, 4, 2, 1, 2), 0.0, 10.0, xyh, np.zeros(3, np.float32), False, True)
    assert ok
    np.testing.assert_allclose(v, [0.0, np.sqrt(2.0), 0.0], rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_velocity_profile_gpu_parity():
    from path_planning_pkg_amd import VelocityGenerator
    vg = VelocityGenerator(*PARAMS)
    cases = random_cases(11, 200, signed=True)
    # plus the reference harness's own path (find_path output, goal -> start)
    from path_planning_pkg_amd import HybridAStar
    cfg, proto, _ = harness()
    g = HybridAStar(cfg)
    drive(g, proto)
    r = g.find_path(proto["vel"], proto["start"])
    for coast in (False, True):
        for stop in (False, True):
            cases.append(dict(xyh=r["path"], curv=r["curvature"], v0=float(proto["vel"]), vmax=9.0, coast=coast,
                              stop=stop))
    ok_g, vel_g = vg.generate_velocity_profiles([c["v0"] for c in cases], [c["vmax"] for c in cases],
                                                [c["xyh"] for c in cases], [c["curv"] for c in cases],
                                                [c["coast"] for c in cases], [c["stop"] for c in cases])
    for i, c in enumerate(cases):
        ok_o, vo = pyoracle.velocity_profile(PARAMS, c["v0"], c["vmax"], c["xyh"], c["curv"], c["coast"], c["stop"])
        assert bool(ok_g[i]) == ok_o, i
        assert (bits(vel_g[i]) == bits(vo)).all(), (i, vel_g[i], vo)
    # single-path entry point == batch
    ok1, v1 = vg.generate_velocity_profile(cases[-1]["v0"], 9.0, r["path"], r["curvature"], True, True)
    assert ok1 == bool(ok_g[-1]) and (bits(v1) == bits(vel_g[-1])).all()


@pytest.mark.gpu
def test_velocity_profile_rejects_empty_path():
    from path_planning_pkg_amd import HastarError, VelocityGenerator
    vg = VelocityGenerator(*PARAMS)
    with pytest.raises(HastarError):
        vg.generate_velocity_profiles([1.0], [5.0], [np.zeros((0, 3), np.float32)], [np.zeros(0, np.float32)],
                                      [False])
