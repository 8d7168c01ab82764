"""Config-3 host logic (CPU): query generation and the rank sharding of bench.py."""
import numpy as np


def test_config3_queries_are_free_and_deterministic():
    from pathplanning_amd import scenes

    raw = scenes.field512()
    s1, g1, sd1 = scenes.config3_queries(raw, 0, 40)
    s2, g2, sd2 = scenes.config3_queries(raw, 20, 20)
    assert np.array_equal(s1[20:], s2) and np.array_equal(g1[20:], g2)
    assert sd1.tolist() == list(range(42, 82))
    circ = np.asarray(raw["circles"])
    for pose in np.concatenate([s1, g1]):
        d2 = (circ[:, 0] - pose[0]) ** 2 + (circ[:, 1] - pose[1]) ** 2
        assert (d2 > (circ[:, 2] + 0.5 + 1.0) ** 2).all()
        assert 0.5 <= pose[0] <= 511.5 and 0.5 <= pose[1] <= 511.5 and -np.pi <= pose[2] < np.pi


def test_shard_ranges_cover_queries_once():
    import bench

    for total in (8192, 1000, 7):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                a, b = bench.shard(total, world, r)
                seen.extend(range(a, b))
            assert seen == list(range(total))


def test_config5_field_and_queries():
    """BASELINE config 5's field (10240 discs on 2048^2) and its query recipe: deterministic,
    starts clear of every inflated disc, shards concatenate to the whole batch"""
    import bench
    from pathplanning_amd import scenes

    raw = scenes.config5_field()
    circ = np.asarray(raw["circles"])
    assert circ.shape == (10240, 3) and raw["bounds"] == (0.0, 0.0, 2048.0, 2048.0)
    assert (circ[:, 2] >= 1.0).all() and (circ[:, 2] < 4.0).all()
    whole, _, seeds = scenes.config3_queries(raw, 0, 24)
    parts = []
    for r in range(4):
        a, b = bench.shard(24, 4, r)
        s, _, sd = scenes.config3_queries(raw, a, b - a)
        assert sd.tolist() == seeds[a:b].tolist()
        parts.append(s)
    assert np.array_equal(np.concatenate(parts), whole)
    for pose in whole:
        d2 = (circ[:, 0] - pose[0]) ** 2 + (circ[:, 1] - pose[1]) ** 2
        assert (d2 > (circ[:, 2] + 0.5 + 1.0) ** 2).all()
