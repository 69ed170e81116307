"""Statistical checks of the counter RNG stream (one
mix32 round per dimension since round 4).  The kernels and the oracle share
the stream, so parity tests cannot see a weak stream; these can.  The spec is
restated vectorised in numpy, checked against the oracle's ora_rng_uniform
value for value, then tested for bias and correlation over millions of draws:
per-dimension mean and variance, lag-1 correlation across dimensions, between
neighbouring pixels and between neighbouring samples, and a 16x16 chi-square
over successive dimension pairs (the pairs a 2-D sample uses)."""
import numpy as np
import pytest

import oracle

M32 = np.uint64(0xFFFFFFFF)


def mix32(x):
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def uniform(seed, pixel, sample, dim):
    """key (k0, k1) per (seed, pixel, sample), one mix32 round per dimension."""
    pixel, sample, dim = (np.asarray(v, np.uint64) for v in (pixel, sample, dim))
    a = mix32(np.uint64(seed) ^ np.uint64(0x2545F491))
    k0 = mix32((mix32(a ^ pixel) + sample * np.uint64(0x9E3779B9)) & M32)
    k1 = mix32(mix32((a + pixel * np.uint64(0x632BE5AB)) & M32)
               ^ ((sample * np.uint64(0x85157AF5) + np.uint64(0x5851F42D)) & M32))
    x = (mix32(((k0 ^ ((dim * np.uint64(0x85EBCA77) + np.uint64(0xC2B2AE3D)) & M32)) + k1) & M32))
    return (x >> np.uint64(8)).astype(np.float64) * 2.0 ** -24


def test_numpy_restatement_matches_oracle():
    rng = np.random.default_rng(5)
    for _ in range(200):
        seed, p, s, d = (int(v) for v in rng.integers(0, 2 ** 32, 4))
        d %= 2048
        assert uniform(seed, p, s, d) == oracle.rng_uniform(seed, p, s, d)


@pytest.fixture(scope="module")
def draws():
    """u[pixel, sample, dim] for 4096 pixels x 64 samples x 16 dims (4.2 M draws)."""
    p = np.arange(4096, dtype=np.uint64)[:, None, None]
    s = np.arange(64, dtype=np.uint64)[None, :, None]
    d = np.arange(16, dtype=np.uint64)[None, None, :]
    return uniform(0, p, s, d)


def corr(a, b):
    a = a - a.mean()
    b = b - b.mean()
    return float((a * b).mean() / np.sqrt((a * a).mean() * (b * b).mean()))


def test_moments_per_dimension(draws):
    n = draws.shape[0] * draws.shape[1]
    for d in range(draws.shape[2]):
        u = draws[:, :, d]
        assert abs(u.mean() - 0.5) < 5 * np.sqrt(1 / 12 / n)
        assert abs(u.var() - 1 / 12) < 5 * np.sqrt(1 / 180 / n)   # var of (u - 1/2)^2 = 1/80 - 1/144


def test_lag1_correlations(draws):
    lim = 5 / np.sqrt(draws.size / draws.shape[2])
    for d in range(draws.shape[2] - 1):                 # successive dimensions of one sample
        assert abs(corr(draws[:, :, d], draws[:, :, d + 1])) < lim
    assert abs(corr(draws[:-1], draws[1:])) < 5 / np.sqrt(draws[1:].size)           # neighbouring pixels
    assert abs(corr(draws[:, :-1], draws[:, 1:])) < 5 / np.sqrt(draws[:, 1:].size)   # neighbouring samples


def test_pair_uniformity_chi2(draws):
    """(dim 2k, dim 2k+1) pairs in 16 x 16 cells: chi-square with 255 degrees of
    freedom, mean 255 and standard deviation 22.6."""
    for k in range(draws.shape[2] // 2):
        x = np.minimum((draws[:, :, 2 * k] * 16).astype(int), 15).ravel()
        y = np.minimum((draws[:, :, 2 * k + 1] * 16).astype(int), 15).ravel()
        h = np.bincount(x * 16 + y, minlength=256).astype(np.float64)
        e = x.size / 256.0
        chi2 = float(((h - e) ** 2 / e).sum())
        assert chi2 < 255 + 5 * 22.6, (k, chi2)
