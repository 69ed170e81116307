"""The oracle's PSS-MLT chain shards (ora_mlt_render_shard, the checker of the
C5 chain-subset parity test): the shards of an n-chain render are its chains
c = r + j * K, so their films and counters sum to the full render, and each
chain's fingerprint and final state do not depend on the shard it ran in."""
import numpy as np

import oracle


def test_shards_sum_to_full_render(cornell_obj):
    nx, ny, chains, steps = 40, 30, 60, 48
    sc = oracle.OracleScene("cornell_box_obj", cornell_obj, nx / ny)
    full, b, cnt = sc.mlt_render(nx, ny, chains, steps, seed=5, n_init=500, nthreads=4)
    one, b1, cnt1, fp1, u1 = sc.mlt_render_shard(nx, ny, chains, steps, 0, 1, seed=5, n_init=500, nthreads=3)
    assert b1 == b and cnt1.rays == cnt.rays
    assert np.allclose(one, full, rtol=0, atol=1e-13)
    K = 4
    tot = np.zeros_like(full)
    rays = samples = 0
    for r in range(K):
        f, br, c, fp, u = sc.mlt_render_shard(nx, ny, chains, steps, r, K, seed=5, n_init=500, nthreads=2)
        assert br == b and len(fp) == len(range(r, chains, K))
        assert np.array_equal(fp, fp1[r::K]) and np.array_equal(u, u1[r::K])
        tot += f
        rays += c.rays
        samples += c.samples
    assert rays == cnt.rays and samples == chains * steps
    assert np.allclose(tot, full, rtol=0, atol=1e-13)
    assert (fp1[:, 0] <= steps).all() and fp1[:, 0].sum() > 0
    assert ((u1 >= 0) & (u1 <= 1)).all()


def test_shard_beyond_chain_count_is_empty(cornell_obj):
    sc = oracle.OracleScene("cornell_box_obj", cornell_obj, 1.0)
    f, b, c, fp, u = sc.mlt_render_shard(16, 16, 3, 8, 5, 8, seed=1, n_init=100)
    assert len(fp) == 0 and c.rays == 0 and not f.any()
