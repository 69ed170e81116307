"""Golden images: converged oracle renders committed as fixtures
(tests/golden/make_golden_images.py, seed 1000).  The oracle on an
independent seed must agree with them within Monte-Carlo noise (tolerances
set from measured spreads: block max 1.6 %, image mean 0.1 % at 1024 spp),
and the golden Cornell mean must match the survey's run of the reference
itself, (0.1341, 0.0890, 0.0276) at 64x64x16 spp."""
import numpy as np

import golden_images as G
import oracle


def test_golden_cornell_matches_reference_run():
    m = G.cornell64().reshape(-1, 3).mean(0)
    ref = np.array([0.1341, 0.0890, 0.0276])
    assert np.all(np.abs(m - ref) / ref < 0.02), m


def test_oracle_independent_seed_converges_to_golden(cornell_obj):
    g = G.cornell64()
    o, _ = oracle.OracleScene("cornell_box_obj", cornell_obj, 1.0).render(64, 64, 1024, seed=7)
    o = o.reshape(64, 64, 3)
    rel = G.block_rel(o, G.blocks(g, 8), 8)
    assert rel.max() < 0.05 and np.median(rel) < 0.01
    assert np.all(np.abs(o.mean((0, 1)) - g.mean((0, 1))) / g.mean((0, 1)) < 0.01)


def test_cornell256_blocks_consistent_with_64():
    """The 256x256 fixture's image mean equals the 64x64 fixture's (same camera,
    aspect 1) within noise."""
    b, _ = G.cornell256_blocks()
    m256 = b.reshape(-1, 3).mean(0)
    m64 = G.cornell64().reshape(-1, 3).mean(0)
    assert np.all(np.abs(m256 - m64) / m64 < 0.01)
