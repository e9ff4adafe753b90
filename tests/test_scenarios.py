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


def test_vectorised_mt19937_generator_matches_per_seed_draws():
    """synthetic_ref_boxes_many (one std::mt19937 stream per seed, vectorised over the seeds)
    draws the same boxes as the per-seed generator; predicted_cost reads those boxes."""
    import numpy as np
    from tests.scenarios import (_mt19937_words, predicted_cost, route_score, synthetic_ref_boxes,
                                 synthetic_ref_boxes_many)
    w = _mt19937_words([5, 4357], 1500)
    for i, s in enumerate((5, 4357)):
        ref = np.random.RandomState(s).randint(0, 2 ** 32, size=1500, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(w[i], ref)
    seeds = [1, 2, 3, 2396, 19303]
    boxes, stx = synthetic_ref_boxes_many(1024, 200, seeds)
    for i, s in enumerate(seeds):
        b, st = synthetic_ref_boxes(1024, 200, s)
        assert np.array_equal(boxes[i], b) and st == stx
    p = predicted_cost(1024, 200, np.array(seeds) - 1)
    assert np.allclose(p, route_score(boxes, [stx, 0.0], [0.0, 0.0]))
