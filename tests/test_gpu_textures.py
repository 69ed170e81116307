"""checker_texture (texture.h:30-49) on the GPU against the fp64 oracle: a
vt-mapped OBJ quad (lambertian), a rough conductor sphere with veach_ajar's
floor checker and a dielectric with a checkered specular reflectance
(tests/scene_specs.py cornell_textured), in path::Li and pssmlt::Li.
Tolerance as in test_gpu_parity.py: image RMSE <= 1e-3 on linear radiance."""
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


@pytest.mark.parametrize("world,flags", [
    ("bvh", 0),                               # LDS-resident binary BVH
    ("bvh", frt.FRT_FLAG_NO_LDS_SCENE),       # HBM 4-wide BVH
    ("list", 0)])                             # hitable_list world
def test_path_textures(ctx, world, flags):
    spec = SS.cornell_textured(world)
    nx, ny, spp = 96, 72, 32
    ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
    film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=11, flags=flags))
    ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=11)
    e = rmse(film, ref)
    print(world, flags, "rmse", e, "rays", st.rays, cnt.rays)
    assert st.samples == cnt.samples and st.camera_rays == cnt.camera_rays
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert np.isfinite(film).all()
    assert e <= 1e-3


def test_texture_edge_flips(ctx):
    """The GPU picks checker cells in fp32 (tu * u_scale * 2 and the sphere's
    atan2 / asin), the oracle in fp64: near a cell edge the other colour can be
    chosen, a flip worth ~|c1 - c0| / spp on its pixel -- systematic along the
    edges, so measured apart from the image RMSE: the pixels carrying a flip
    (max |diff| > 1e-3) are counted and the rest must agree to 2e-4.  128 spp
    on the veach_ajar-scale checker (20 x 80) sphere and the floor quad."""
    spec = SS.cornell_textured()
    nx, ny, spp = 128, 96, 128
    ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
    film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=23))
    ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=23)
    d = np.abs(film.reshape(-1, 3).astype(np.float64) - ref).max(axis=1)
    bad = d > 1e-3
    rest = rmse(film.reshape(-1, 3)[~bad], ref[~bad])
    print(f"texture edge flips: {int(bad.sum())} of {nx * ny} px ({100.0 * bad.mean():.2f} %), "
          f"rmse(all) {rmse(film, ref):.3e}, rmse(rest) {rest:.3e}")
    assert bad.mean() <= 0.02
    assert rest <= 2e-4
    assert rmse(film, ref) <= 1e-3


@pytest.mark.parametrize("make", [SS.cornell_textured, SS.cornell_image_textured])
def test_pssmlt_textures(ctx, make):
    """pssmlt::Li with checker and image textures: short chains vs the oracle's."""
    spec = make()
    nx, ny, mpp, chains = 48, 48, 4, 2304
    ctx.upload(frt.HostScene.from_spec(spec, 1.0))
    film = np.zeros((ny, nx, 3), np.float32)
    film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, mpp, chains, seed=4, bootstrap=2000), film)
    steps = mpp * nx * ny // chains
    ref, b, cnt = oracle.OracleScene.from_spec(spec, 1.0).mlt_render(nx, ny, chains, steps, seed=4, n_init=2000)
    assert st.samples == chains * steps == cnt.samples
    assert abs(st.rays - cnt.rays) / cnt.rays < 5e-3
    assert rmse(film, ref) <= 2e-3 * max(1.0, float(np.abs(ref).max()))


def test_checker_light_rejected(ctx):
    spec = {"objects": [{"obj": SS.CORNELL_OBJ, "geo": True},
                        {"sphere": (0, 1, 0), "radius": 0.1, "where": "both",
                         "material": SS.checker({"type": "diffuse_light", "emit": (4, 4, 4)}, (1, 1, 1), (2, 2))}],
            "camera": SS.CORNELL_CAM}
    with pytest.raises(frt.FrtError, match="checker"):
        ctx.upload(frt.HostScene.from_spec(spec, 1.0))


@pytest.mark.parametrize("world,flags", [
    ("bvh", 0),                               # LDS-resident binary BVH (texels in HBM)
    ("bvh", frt.FRT_FLAG_NO_LDS_SCENE),       # HBM 4-wide BVH
    ("list", 0)])                             # hitable_list world
def test_path_image_textures(ctx, world, flags):
    """image_texture (texture.h:51-95): 8-bit sRGB and HDR images (tests/scene_specs.py
    cornell_image_textured) against the oracle; a texel edge can round to the neighbour
    in fp32, as the checker's cell edges can, so the gate is the image RMSE."""
    spec = SS.cornell_image_textured(world)
    nx, ny, spp = 96, 72, 32
    ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
    film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=11, flags=flags))
    ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=11)
    e = rmse(film, ref)
    print(world, flags, "rmse", e, "rays", st.rays, cnt.rays)
    assert st.samples == cnt.samples and st.camera_rays == cnt.camera_rays
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert np.isfinite(film).all()
    assert e <= 1e-3
