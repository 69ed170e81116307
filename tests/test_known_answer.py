"""Known-answer scenes, built with the scene builder:

* empty scene (every ray misses): the film is the environment colour exactly,
  one camera ray per sample;
* white furnace: a convex lambertian object under a constant environment and
  no lights.  Every camera ray that hits it scatters once (cosine lobe,
  f cos / pdf = albedo) and escapes, so a hit pixel is albedo * env and a miss
  is env -- exact, with no Monte-Carlo noise.  Albedo 1 makes the object
  vanish.

Checked for the oracle, the device path code run on the host, and (gpu) the
kernels, on a sphere (list world and one-primitive BVH) and on the cube OBJ
(BVH)."""
import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle
import scene_specs as SS

ENV = (1.0, 0.8, 0.6)
ALBEDO = (0.5, 0.7, 0.25)
CAM = {"lookfrom": (0.0, 0.0, 4.0), "lookat": (0.0, 0.0, 0.0), "vup": (0.0, 1.0, 0.0), "vfov": 40.0,
       "aperture": 0.0, "focus": 4.0}


def furnace_spec(kind, world, albedo=ALBEDO):
    lam = {"type": "lambertian", "albedo": albedo}
    obj = ({"sphere": (0.0, 0.0, 0.0), "radius": 0.8, "material": lam} if kind == "sphere" else
           {"obj": SS.CUBE_OBJ, "to_world": SS.to_world(0.6, 30.0, (0.0, 0.0, 0.0)), "bsdf": lam, "geo": True})
    return {"objects": [obj], "camera": CAM, "world": world, "env": ENV}


def empty_spec(world):
    # one small sphere behind the camera: no camera ray can reach it
    return {"objects": [{"sphere": (0.0, 0.0, 50.0), "radius": 0.1,
                         "material": {"type": "lambertian", "albedo": (1, 1, 1)}}],
            "camera": CAM, "world": world, "env": ENV}


def classify(img, albedo):
    """Every pixel is env (miss) or albedo*env (hit); returns the hit fraction."""
    img = np.asarray(img, np.float64).reshape(-1, 3)
    env, hit = np.array(ENV), np.array(albedo) * np.array(ENV)
    is_env = np.abs(img - env).max(1) < 1e-5
    is_hit = np.abs(img - hit).max(1) < 1e-5
    # pixels on the silhouette average hits and misses: their value lies on the segment
    t = (img - env) / (hit - env + 1e-30)
    mixed = ~(is_env | is_hit)
    on_seg = np.abs(t[mixed] - t[mixed][:, :1]).max(1) < 1e-4 if mixed.any() else np.array([], bool)
    assert on_seg.all()
    assert mixed.mean() < 0.1
    return is_hit.mean()


CASES = [("sphere", "list"), ("sphere", "bvh"), ("cube", "bvh")]


@pytest.mark.parametrize("kind,world", CASES)
def test_furnace_oracle_and_host_replay(kind, world):
    nx = ny = 32
    spec = furnace_spec(kind, world)
    ref, cnt = oracle.OracleScene.from_spec(spec, 1.0).render(nx, ny, 4, seed=1)
    frac = classify(ref, ALBEDO)
    assert 0.1 < frac < 0.9
    hs = frt.HostScene.from_spec(spec, 1.0)
    g, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 4, seed=1), np.arange(nx * ny, dtype=np.int32))
    assert abs(classify(g, ALBEDO) - frac) < 1e-9
    assert st.shadow_rays == 0 == cnt.shadow_rays                       # no lights: no NEE (pick_sample -> -1)
    assert st.rays == cnt.rays


@pytest.mark.parametrize("kind,world", CASES)
def test_white_furnace_is_invisible(kind, world):
    nx = ny = 24
    spec = furnace_spec(kind, world, albedo=(1.0, 1.0, 1.0))
    ref, _ = oracle.OracleScene.from_spec(spec, 1.0).render(nx, ny, 2, seed=3)
    assert np.abs(ref - np.array(ENV)).max() < 1e-12
    g, _ = frt.selftest_path_host(frt.HostScene.from_spec(spec, 1.0), frt.RenderParams.make(nx, ny, 2, seed=3),
                                  np.arange(nx * ny, dtype=np.int32))
    assert np.abs(g.reshape(-1, 3) - np.array(ENV)).max() < 1e-5


@pytest.mark.parametrize("world", ["list", "bvh"])
def test_empty_scene_is_env(world):
    nx, ny, spp = 20, 12, 3
    spec = empty_spec(world)
    ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=0)
    assert np.abs(ref - np.array(ENV)).max() < 1e-14                  # mean of ns equal samples
    assert cnt.rays == cnt.camera_rays == nx * ny * spp
    g, st = frt.selftest_path_host(frt.HostScene.from_spec(spec, nx / ny), frt.RenderParams.make(nx, ny, spp),
                                   np.arange(nx * ny, dtype=np.int32))
    assert np.abs(g.reshape(-1, 3) - np.array(ENV)).max() < 1e-6
    assert st.rays == nx * ny * spp


@pytest.mark.gpu
@pytest.mark.parametrize("kind,world", CASES)
def test_furnace_gpu(kind, world):
    ctx = frt.Context(0)
    try:
        nx, ny = 64, 48
        spec = furnace_spec(kind, world)
        ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
        film, st = ctx.render(frt.RenderParams.make(nx, ny, 8, seed=4))
        ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, 8, seed=4)
        assert abs(classify(film, ALBEDO) - classify(ref, ALBEDO)) < 2.0 / (nx * ny)
        assert st.shadow_rays == 0 and st.rays == cnt.rays
        white = furnace_spec(kind, world, albedo=(1.0, 1.0, 1.0))
        ctx.upload(frt.HostScene.from_spec(white, nx / ny))
        film, _ = ctx.render(frt.RenderParams.make(nx, ny, 4, seed=4))
        assert np.abs(film.reshape(-1, 3) - np.array(ENV)).max() < 1e-5
        ctx.upload(frt.HostScene.from_spec(empty_spec(world), nx / ny))
        film, st = ctx.render(frt.RenderParams.make(nx, ny, 4))
        assert np.abs(film.reshape(-1, 3) - np.array(ENV)).max() < 1e-6
        assert st.rays == st.camera_rays == nx * ny * 4
    finally:
        ctx.close()
