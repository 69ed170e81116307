"""PSS-MLT on the GPU (one lane per Markov chain) against the oracle's
restatement of pssmlt.cpp on the same chain streams.  Short chains are
path-exact (an accept decision flips only if u lands within fp32 rounding of
the acceptance ratio), so the splat films agree to fp32 accumulation noise;
long runs are checked statistically against the path tracer."""
import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = frt.Context(0)
    yield c
    c.close()


def rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


@pytest.mark.parametrize("kind,objfix", [("cornell_box_obj", "cornell_obj"), ("veach_mis", "veach_obj")])
def test_short_chains_match_oracle(ctx, kind, objfix, request):
    obj = request.getfixturevalue(objfix)
    nx, ny, mpp, chains = 64, 48, 4, 3072          # 4 mutations/pixel -> 4 steps per chain
    hs = frt.HostScene(kind, obj, nx / ny)
    ctx.upload(hs)
    film = np.zeros((ny, nx, 3), np.float32)
    film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, mpp, chains, seed=7, bootstrap=2000), film)
    steps = mpp * nx * ny // chains
    ref, b, cnt = oracle.OracleScene(kind, obj, nx / ny).mlt_render(nx, ny, chains, steps, seed=7, n_init=2000)
    e = rmse(film, ref)
    print(kind, "mlt rmse", e, "mean", film.reshape(-1, 3).mean(0), ref.reshape(-1, 3).mean(0), "b", b)
    assert st.samples == chains * steps == cnt.samples
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    scale = max(1.0, float(np.abs(ref).max()))
    assert e <= 1e-3 * scale
    # the chains' trajectory fingerprints and final states (frt_mlt_chain_state)
    u, fp = ctx.mlt_chain_state(0, chains)
    _, _, _, fp_o, u_o = oracle.OracleScene(kind, obj, nx / ny).mlt_render_shard(nx, ny, chains, steps, 0, 1, seed=7,
                                                                                 n_init=2000)
    same = np.all(fp == fp_o, axis=1)
    print(kind, "path-exact chains", int(same.sum()), "of", chains, "accepts", int(fp[:, 0].sum()), int(fp_o[:, 0].sum()))
    assert same.mean() >= 0.99
    assert np.abs(u[same] - u_o[same]).max() <= 1e-5


@pytest.mark.parametrize("flags", [frt.FRT_FLAG_NO_LDS_SCENE, frt.FRT_FLAG_NO_LDS_SCENE | frt.FRT_FLAG_BVH2])
def test_short_chains_hbm_scene(ctx, cornell_obj, tmp_path, flags):
    """The HBM-resident chain kernels (4-wide and binary BVH) on a tessellated
    Cornell box against the oracle's chains."""
    dst = str(tmp_path / "tess.obj")
    frt.write_tessellated_obj(cornell_obj, 12, dst)
    nx, ny, mpp, chains = 48, 32, 4, 1536
    ctx.upload(frt.HostScene("cornell_box_obj", dst, nx / ny))
    film = np.zeros((ny, nx, 3), np.float32)
    film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, mpp, chains, seed=9, bootstrap=2000, flags=flags), film)
    steps = mpp * nx * ny // chains
    ref, b, cnt = oracle.OracleScene("cornell_box_obj", dst, nx / ny).mlt_render(nx, ny, chains, steps, seed=9,
                                                                                 n_init=2000)
    assert st.scene_in_lds == 0
    assert st.samples == chains * steps == cnt.samples
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert rmse(film, ref) <= 1e-3 * max(1.0, float(np.abs(ref).max()))


@pytest.mark.parametrize("objfix", ["sphere_obj", "glass_obj"])
def test_short_chains_specular(ctx, objfix, request):
    """pssmlt::Li's specular branch (pssmlt.cpp:232-249) vs the oracle's chains:
    phong spheres (Sphere) and a dielectric sphere (Glass)."""
    obj = request.getfixturevalue(objfix)
    nx, ny, mpp, chains = 48, 48, 4, 2304
    ctx.upload(frt.HostScene("cornell_box_obj", obj, 1.0))
    film = np.zeros((ny, nx, 3), np.float32)
    film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, mpp, chains, seed=4, bootstrap=2000), film)
    steps = mpp * nx * ny // chains
    ref, b, cnt = oracle.OracleScene("cornell_box_obj", obj, 1.0).mlt_render(nx, ny, chains, steps, seed=4,
                                                                            n_init=2000)
    assert st.samples == chains * steps == cnt.samples
    assert abs(st.rays - cnt.rays) / cnt.rays < 5e-3
    assert rmse(film, ref) <= 2e-3 * max(1.0, float(np.abs(ref).max()))


def test_sharded_chains_sum_to_single(ctx, cornell_obj):
    nx, ny = 32, 32
    ctx.upload(frt.HostScene("cornell_box_obj", cornell_obj, 1.0))
    one = np.zeros((ny, nx, 3), np.float32)
    ctx.render(frt.RenderParams.pssmlt(nx, ny, 8, 1024, seed=2, bootstrap=1000), one)
    two = np.zeros((ny, nx, 3), np.float32)
    for r in range(2):
        ctx.render(frt.RenderParams.pssmlt(nx, ny, 8, 1024, seed=2, bootstrap=1000, shard_index=r, shard_count=2), two)
    assert np.allclose(one, two, rtol=1e-4, atol=1e-5)


def test_splat_film_reproducible(ctx, cornell_obj):
    """Splats land in a fixed-point film with 64-bit integer atomics, so the
    film does not depend on the order the chains' atomics arrive in: two runs
    give the same bytes (float atomics did not)."""
    nx, ny = 96, 64
    ctx.upload(frt.HostScene("cornell_box_obj", cornell_obj, nx / ny))
    films = []
    for _ in range(3):
        f = np.zeros((ny, nx, 3), np.float32)
        f, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, 16, 4096, seed=9, bootstrap=1000), f)
        films.append(f)
    assert np.isfinite(films[0]).all() and films[0].max() > 0
    assert np.array_equal(films[0], films[1]) and np.array_equal(films[0], films[2])


def test_converges_to_path_tracer(ctx, cornell_obj):
    """Same image as the path tracer (depth <= 10) once the chains are long:
    the reference starts chains from uniform states with no burn-in, so short
    chains are biased low (start-up bias; 64 steps/chain ~ -20 %, 4096 ~ 0 %).
    2048 chains x 4096 mutations here; the C5 bench config runs ~4050."""
    nx, ny = 64, 64
    ctx.upload(frt.HostScene("cornell_box_obj", cornell_obj, 1.0))
    film = np.zeros((ny, nx, 3), np.float32)
    film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, 2048, 2048, seed=1), film)
    ref, _ = ctx.render(frt.RenderParams.make(nx, ny, 2048, seed=1, max_depth=10))
    fb = film.reshape(8, 8, 8, 8, 3).mean(axis=(1, 3))
    rb = ref.reshape(8, 8, 8, 8, 3).mean(axis=(1, 3))
    rel = np.abs(fb - rb) / (rb + 1e-2)
    print("mlt vs path block rel: median", np.median(rel), "max", rel.max(), "means", film.mean((0, 1)), ref.mean((0, 1)))
    assert np.median(rel) < 0.05
    assert abs(film.mean() - ref.mean()) / ref.mean() < 0.03


def test_block_means_match_oracle_path(ctx, cornell_obj):
    """C5's RMSE gate at a reduced size (bench.py mlt_block_rmse, the same
    comparison the bench line reports at 1080p): the GPU's PSS-MLT film in
    8x8-block means against the oracle's fp64 path::Li at pssmlt's depth cap
    (max_depth 10), 256 spp in two independent halves.  128x96 at 1024
    mutations/pixel over 1536 chains = 8192 mutations a chain.  Each film is
    first corrected for the noise of PSS-MLT's normaliser b (10^4 bootstrap
    paths, pssmlt.cpp:303-312) with the oracle's b from 10^7 paths.  One
    run's mean still carries the chains' own noise and start-up transient
    (a single seed at 512 mutations/pixel read +2.6 % with b's noise out,
    profiles/r04/r04j), so the mean is taken over four
    independent runs (seeds 3..6).  Tolerance: median per-block relative error
    <= 0.05 in every run, mean over the blocks and runs within 2 %."""
    import bench
    nx, ny = 128, 96
    ctx.upload(frt.HostScene("cornell_box_obj", cornell_obj, nx / ny))
    errs = []
    for seed in (3, 4, 5, 6):
        film = np.zeros((ny, nx, 3), np.float32)
        film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, 1024, 1536, seed=seed), film)
        r = bench.mlt_block_rmse("cornell_box_obj", cornell_obj, nx, ny, film.reshape(-1), 16, 0.0, spp=256,
                                 seed=seed)
        print("seed", seed, "pssmlt vs oracle path blocks:", r)
        assert r["blocks"] == (nx // 8) * (ny // 8)
        assert r["rel_block_err_median"] <= r["tolerance"]["rel_block_err_median"]
        errs.append(r["mean_rel_err_b_corrected"])
    print("mean_rel_err_b_corrected per seed", errs, "mean", float(np.mean(errs)))
    assert abs(float(np.mean(errs))) <= r["tolerance"]["mean_rel_err_b_corrected"]


def test_chain_state_needs_a_pssmlt_render(ctx, cornell_obj):
    ctx.upload(frt.HostScene("cornell_box_obj", cornell_obj, 1.0))
    ctx.render(frt.RenderParams.make(16, 16, 1, seed=1))
    with pytest.raises(frt.FrtError):
        ctx.mlt_chain_state(0, 1)
    f = np.zeros((16, 16, 3), np.float32)
    ctx.render(frt.RenderParams.pssmlt(16, 16, 4, 64, seed=1, bootstrap=100, shard_index=1, shard_count=2), f)
    u, fp = ctx.mlt_chain_state(0, 32)                     # shard (1, 2) holds 32 chains
    assert u.shape == (32, 92) and ((u >= 0) & (u <= 1)).all()
    with pytest.raises(frt.FrtError):
        ctx.mlt_chain_state(0, 33)


def test_c5_chain_shard_matches_oracle(ctx, cornell_obj):
    """C5 at its own config: CornellBox-Original 1920x1080,
    512 mutations per pixel over 2^18 chains = 4050 mutations a chain.  The GPU
    renders shard (0, 256) -- the 1024 chains c = 0 mod 256, each for the full
    4050 mutations -- and the oracle's fp64 restatement of pssmlt.cpp runs the
    same chains on the same streams (ora_mlt_render_shard).  A chain is
    path-exact when its trajectory fingerprint (accepted proposals, sum of the
    accepted steps' indices) equals the oracle's; fp32 rounding can flip one
    accept or hit decision, after which the two copies walk apart until both
    accept the same large step (`diverged_chains`; 133 of 16,384 = 0.8 % in the
    bench's shard of 16, profiles/r05/r05a).  Gates: samples equal, ray counts
    within 2e-3, >= 97 % of the chains path-exact, their final states within
    1e-4, shard-film means within 1e-3 and 8x8-block means within 1 % (relative
    L2), and the full-frame RMSE estimate sqrt(K) x shard RMSE <= 1e-3 (the
    north star's gate).  It also prints the start-up bias of both against the
    GPU path tracer at pssmlt's depth cap: the GPU's chains and the oracle's
    carry the same bias."""
    import bench
    nx, ny, mpp, n_chains, K = 1920, 1080, 512, 1 << 18, 256
    ctx.upload(frt.HostScene("cornell_box_obj", cornell_obj, nx / ny))
    r = bench.mlt_shard_parity(ctx, "cornell_box_obj", cornell_obj, nx, ny, mpp, n_chains, K, 0, 16)
    r.pop("gpu_film")
    pt, _ = ctx.render(frt.RenderParams.make(nx, ny, 32, seed=11, max_depth=10))
    ptm = float(pt.mean())
    print("C5 shard parity:", r)
    print("start-up bias vs path tracer (depth 10, 32 spp, mean %.6f): gpu %+.4f oracle %+.4f"
          % (ptm, K * np.mean(r["mean_gpu"]) / ptm - 1.0, K * np.mean(r["mean_oracle"]) / ptm - 1.0))
    assert r["samples_gpu"] == r["samples_oracle"] == r["chains"] * r["steps_per_chain"]
    assert r["steps_per_chain"] == 4050 and r["chains"] == 1024
    assert r["rays_rel_diff"] < 2e-3
    assert r["path_exact_chains"] >= 0.97 * r["chains"]
    assert r["state_maxdiff_path_exact"] <= 1e-4
    assert abs(r["mean_rel_diff"]) <= 1e-3
    assert r["block8_rel_l2"] <= 0.01
    assert r["full_frame_rmse_est"] <= 1e-3
