"""CPU checks of the synthetic workload generator (tests/scenarios.py)."""
import numpy as np

from tests.scenarios import _synthetic_boxes, _synthetic_boxes_loop, replan_tick_inputs, replan_pairs, synthetic


def test_vectorised_boxes_equal_the_loop():
    """The vectorised draw (bench setup) gives exactly the one-at-a-time generator's boxes."""
    for N, K in ((256, 10), (512, 50), (1024, 200), (2048, 200)):
        for seed in (1, 2, 3, 10227, 3299):
            a = np.array(_synthetic_boxes_loop(N * 0.5, K, np.random.default_rng(seed), 8.0))
            b = np.array(_synthetic_boxes(N * 0.5, K, np.random.default_rng(seed), 8.0))
            assert a.shape == b.shape == (K, 4)
            assert np.array_equal(a, b)


def test_synthetic_case_shape():
    cfg, proto = synthetic(1024, 72, 200, seed=4)
    assert cfg.grid_size == 1024 and proto["boxes"].shape == (200, 4)
    W = 512.0
    b = proto["boxes"]
    assert (b[:, 2:] >= 1).all() and (b[:, 2:] <= 6).all()
    assert (b[:, 0] >= -0.8 * W).all() and (b[:, 0] <= 0.2 * W).all()


def test_replan_ticks_move_boxes_and_start():
    (cfg, proto, vel), = replan_pairs(256, 36, 12, 1, seed=5)
    s0, b0 = replan_tick_inputs(proto, vel, 0)
    s2, b2 = replan_tick_inputs(proto, vel, 2)
    assert np.allclose(b2[:, :2] - b0[:, :2], vel * 0.1, atol=1e-4)
    assert s2 != s0
