"""GPU parity of the reference's other integrators, run by the same persistent
megakernel (KIND template, csrc/frt_render.hip) through the C-ABI:
ambient occlusion (ao::Li, first_ray/ao.cpp:4-27) and shading normals
(normals_renderer::Li, first_ray/debug_renderer.h:8-17), against the fp64
oracle on the same counter-RNG streams.

Tolerance: per-pixel max |diff| <= 1e-3 except where fp32 rounding sends a
sample to another primitive (at most 1% of pixels); the others agree to
1e-5 RMSE.  Camera-ray and sample counts are exact.  A constant non-black
environment is set (the reference scenes' is black, so AO would be all 0)."""
import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle

pytestmark = pytest.mark.gpu

AO, NORMALS = frt.FRT_INTEGRATOR_AO, frt.FRT_INTEGRATOR_NORMALS
ENV = (1.0, 0.75, 0.5)


@pytest.fixture(scope="module")
def ctx():
    c = frt.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def tess_obj(cornell_obj, tmp_path_factory):
    """CornellBox tessellated k=24 (~20k triangles): HBM-resident, 4-wide BVH plan."""
    dst = str(tmp_path_factory.mktemp("tess") / "t24.obj")
    frt.write_tessellated_obj(cornell_obj, 24, dst)
    return dst


def render_pair(ctx, kind, obj, nx, ny, spp, integrator, env=ENV, seed=2, flags=0):
    hs = frt.HostScene(kind, obj, nx / ny)
    hs.set_env(env)
    ctx.upload(hs)
    film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=seed, integrator=integrator, flags=flags))
    osc = oracle.OracleScene(kind, obj, nx / ny)
    osc.set_env(env)
    ref, cnt = osc.render(nx, ny, spp, seed=seed, integrator=integrator)
    return film.reshape(-1, 3).astype(np.float64), st, ref, cnt


def check_close(film, ref, max_frac=0.01):
    d = np.abs(film - ref).max(axis=1)
    bad = d > 1e-3
    assert bad.sum() <= max(1, max_frac * len(d)), (int(bad.sum()), len(d))
    assert float(np.sqrt(np.mean((film[~bad] - ref[~bad]) ** 2))) < 1e-5
    return int(bad.sum())


CASES = [("cornell_box_obj", "cornell_obj", 0),                            # LDS-resident binary BVH
         ("cornell_box_obj", "cornell_obj", frt.FRT_FLAG_NO_LDS_SCENE),    # HBM, 4-wide quantized BVH
         ("cornell_box_obj", "cornell_obj", frt.FRT_FLAG_NO_LDS_SCENE | frt.FRT_FLAG_BVH2),
         ("veach_mis", "veach_obj", 0),                                    # list world (spheres)
         ("cornell_box_obj", "sphere_obj", 0),                             # modified_phong
         ("cornell_box_obj", "glass_obj", 0),                              # dielectric
         ("cornell_box_obj", "tess_obj", 0)]                               # ~20k triangles in HBM


@pytest.mark.parametrize("kind,objfix,flags", CASES)
def test_ao_matches_oracle(ctx, kind, objfix, flags, request):
    obj = request.getfixturevalue(objfix)
    nx, ny, spp = 96, 64, 16
    film, st, ref, cnt = render_pair(ctx, kind, obj, nx, ny, spp, AO, flags=flags)
    flips = check_close(film, ref)
    assert st.samples == st.camera_rays == cnt.camera_rays == nx * ny * spp
    assert abs(int(st.shadow_rays) - int(cnt.shadow_rays)) <= spp * max(flips, 1)
    assert st.extension_rays == 0
    assert (film >= 0).all() and (film <= np.array(ENV) + 1e-6).all()


@pytest.mark.parametrize("kind,objfix,flags", CASES)
def test_normals_match_oracle(ctx, kind, objfix, flags, request):
    obj = request.getfixturevalue(objfix)
    nx, ny, spp = 96, 64, 4
    film, st, ref, cnt = render_pair(ctx, kind, obj, nx, ny, spp, NORMALS, env=(0.25, 0.5, 0.75), flags=flags)
    check_close(film, ref)
    assert st.camera_rays == cnt.camera_rays == nx * ny * spp and st.shadow_rays == 0


def test_ao_launch_plan(ctx, cornell_obj, tess_obj):
    """AO runs the default plans: LDS-resident binary BVH for CornellBox, the
    4-wide HBM BVH for the tessellated scene."""
    for obj, lds in ((cornell_obj, 1), (tess_obj, 0)):
        hs = frt.HostScene("cornell_box_obj", obj, 1.0)
        ctx.upload(hs)
        _, st = ctx.render(frt.RenderParams.make(64, 64, 2, integrator=AO))
        assert st.scene_in_lds == lds
        assert st.waves_cap == (5 if lds else 6)


def test_ao_deterministic_and_shard_invariant(ctx, cornell_obj):
    """Bit-identical run to run and when the frame is split into shards."""
    hs = frt.HostScene("cornell_box_obj", cornell_obj, 1.0)
    hs.set_env(ENV)
    ctx.upload(hs)
    p = frt.RenderParams.make(80, 72, 8, seed=9, integrator=AO)
    a, _ = ctx.render(p)
    b, _ = ctx.render(p)
    assert np.array_equal(a, b)
    c = np.zeros_like(a)
    for k in range(3):
        ctx.render(frt.RenderParams.make(80, 72, 8, seed=9, integrator=AO, shard_index=k, shard_count=3), c)
    assert np.array_equal(a, c)


@pytest.mark.parametrize("nx,ny,spp", [(7, 5, 1), (33, 17, 3)])
def test_ao_ragged_frames(ctx, cornell_obj, nx, ny, spp):
    film, st, ref, cnt = render_pair(ctx, "cornell_box_obj", cornell_obj, nx, ny, spp, AO)
    check_close(film, ref, max_frac=0.05)
    assert st.samples == nx * ny * spp
