"""metal and rough_conductor (GGX / Beckmann visible-normal sampling) on the
GPU against the fp64 oracle, in scenes built with the incremental builder
(tests/scene_specs.py): path::Li, pssmlt::Li and ao::Li.  Tolerance as in
test_gpu_parity.py: image RMSE <= 1e-3 on linear radiance."""
import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle
import scene_specs as SS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = frt.Context(0)
    yield c
    c.close()


def rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64).reshape(-1, 3) - np.asarray(b, np.float64).reshape(-1, 3)) ** 2)))


@pytest.mark.parametrize("sphere_dist,cube_dist,world,flags", [
    ("ggx", "beckmann", "bvh", 0),                               # LDS-resident binary BVH
    ("beckmann", "ggx", "bvh", frt.FRT_FLAG_NO_LDS_SCENE),       # HBM 4-wide BVH
    ("ggx", "beckmann", "list", 0)])                             # hitable_list world
def test_path_conductors(ctx, sphere_dist, cube_dist, world, flags):
    spec = SS.cornell_conductors(sphere_dist, cube_dist, world)
    nx, ny, spp = 96, 72, 32
    ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
    film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=11, flags=flags))
    ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=11)
    e = rmse(film, ref)
    print(sphere_dist, cube_dist, world, flags, "rmse", e, "rays", st.rays, cnt.rays)
    assert st.samples == cnt.samples and st.camera_rays == cnt.camera_rays
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert np.isfinite(film).all()
    assert e <= 1e-3


def test_register_caps_agree(ctx, monkeypatch):
    """The material kernels give the same film under every register cap and
    plan (FRT_MATS_WAVES 0 / 3 / 4 / 5 / 6; LDS binary, HBM 4-wide, HBM binary).
    A source restructuring of the specular dispatch once compiled to kernels
    that were right uncapped and wrong (RMSE 0.04-0.18) under some caps, with
    unchanged ray counts; this pins every cap against the oracle."""
    spec = SS.cornell_conductors("beckmann", "ggx", "bvh")
    nx, ny, spp = 64, 48, 16
    ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
    ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=12)
    films = []
    for flags in (0, frt.FRT_FLAG_NO_LDS_SCENE, frt.FRT_FLAG_NO_LDS_SCENE | frt.FRT_FLAG_BVH2):
        for w in ("0", "3", "4", "5", "6"):
            monkeypatch.setenv("FRT_MATS_WAVES", w)
            film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=12, flags=flags))
            assert st.waves_cap == int(w)
            e = rmse(film, ref)
            assert e <= 1e-3, (flags, w, e)
            films.append(film)
    for f in films[1:]:                                   # the same hits and sums: bit-identical
        assert np.array_equal(f, films[0])


def test_pssmlt_conductors(ctx):
    """pssmlt::Li's specular branch with metal + rough conductors: short chains vs the oracle's."""
    spec = SS.cornell_conductors()
    nx, ny, mpp, chains = 48, 48, 4, 2304
    ctx.upload(frt.HostScene.from_spec(spec, 1.0))
    film = np.zeros((ny, nx, 3), np.float32)
    film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, mpp, chains, seed=4, bootstrap=2000), film)
    steps = mpp * nx * ny // chains
    ref, b, cnt = oracle.OracleScene.from_spec(spec, 1.0).mlt_render(nx, ny, chains, steps, seed=4, n_init=2000)
    assert st.samples == chains * steps == cnt.samples
    assert abs(st.rays - cnt.rays) / cnt.rays < 5e-3
    assert rmse(film, ref) <= 2e-3 * max(1.0, float(np.abs(ref).max()))


def test_ao_rough_conductor(ctx):
    """ao::Li samples the rough conductor's visible normals (pdf.h:465-482)."""
    spec = SS.cornell_conductors(metal=False)
    spec["env"] = (1.0, 1.0, 1.0)
    nx = ny = 64
    ctx.upload(frt.HostScene.from_spec(spec, 1.0))
    film, st = ctx.render(frt.RenderParams.make(nx, ny, 16, seed=2, integrator=frt.FRT_INTEGRATOR_AO))
    ref, cnt = oracle.OracleScene.from_spec(spec, 1.0).render(nx, ny, 16, seed=2, integrator=2)
    assert st.shadow_rays == cnt.shadow_rays
    assert rmse(film, ref) <= 1e-3


def test_ao_metal_rejected(ctx):
    ctx.upload(frt.HostScene.from_spec(SS.cornell_conductors(), 1.0))
    with pytest.raises(frt.FrtError, match="metal"):
        ctx.render(frt.RenderParams.make(8, 8, 1, integrator=frt.FRT_INTEGRATOR_AO))
