"""The reference's other integrators on the same traversal: ambient occlusion
(ao::Li, first_ray/ao.cpp:4-27) and shading normals (normals_renderer::Li,
first_ray/debug_renderer.h:8-17).  The fp64 oracle restates both; the device
code (csrc/frt_path.hpp ao_shade / normals_shade) runs on the host through the
self-test hook on the same counter-RNG streams.

Tolerance: per-pixel max |diff| <= 1e-3 on all but the pixels where fp32
rounding sends one sample to another primitive (a silhouette or box edge);
those are at most 1% of the pixels, and the rest agree to 1e-5 RMSE.  Sample
and ray counts are exact up to those flips.  The reference scenes have a black
environment (which makes every AO sample 0), so the tests set a constant one."""
import math

import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle

AO, NORMALS = frt.FRT_INTEGRATOR_AO, frt.FRT_INTEGRATOR_NORMALS


def pair(kind, obj, nx, ny, spp, integrator, env, seed=1, pixels=None):
    pix = np.arange(nx * ny, dtype=np.int32) if pixels is None else pixels
    hs = frt.HostScene(kind, obj, nx / ny)
    hs.set_env(env)
    out, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, spp, seed=seed, integrator=integrator), pix)
    osc = oracle.OracleScene(kind, obj, nx / ny)
    osc.set_env(env)
    ref, cnt = osc.render(nx, ny, spp, seed=seed, pixels=pix, integrator=integrator)
    return out.astype(np.float64), st, ref, cnt


def check_close(out, ref, max_frac=0.01):
    d = np.abs(out - ref).max(axis=1)
    bad = d > 1e-3
    assert bad.sum() <= max(1, max_frac * len(d)), (int(bad.sum()), len(d))
    good = ~bad
    assert float(np.sqrt(np.mean((out[good] - ref[good]) ** 2))) < 1e-5
    return int(bad.sum())


def test_ao_tmax_is_half_the_world_box_height(cornell_obj, veach_obj):
    """ao.cpp:19-21: t_max = bbox.size.y() * 0.50f; CornellBox-Original spans
    y in [0, 1.99].  A list world has no box: hitable_list::bounding_box
    returns before assigning it (hitable_list.cpp:27-29) and the default aabb
    is NaN (geometry.h:345-348)."""
    osc = oracle.OracleScene("cornell_box_obj", cornell_obj, 1.0)
    hs = frt.HostScene("cornell_box_obj", cornell_obj, 1.0).arrays()
    root_box = hs["node_box"][hs["root"]]
    assert osc.ao_tmax() == pytest.approx(0.995, abs=1e-6)
    assert osc.ao_tmax() == (root_box[4] - root_box[1]) * 0.5
    assert math.isnan(oracle.OracleScene("veach_mis", veach_obj, 1.0).ao_tmax())


@pytest.mark.parametrize("kind,objfix", [("cornell_box_obj", "cornell_obj"), ("veach_mis", "veach_obj"),
                                         ("cornell_box_obj", "sphere_obj"), ("cornell_box_obj", "glass_obj")])
def test_ao_device_code_matches_oracle(kind, objfix, request):
    obj = request.getfixturevalue(objfix)
    env = (1.0, 0.75, 0.5)
    out, st, ref, cnt = pair(kind, obj, 48, 32, 8, AO, env)
    flips = check_close(out, ref)
    assert st.camera_rays == cnt.camera_rays == 48 * 32 * 8
    assert abs(int(st.shadow_rays) - int(cnt.shadow_rays)) <= 8 * max(flips, 1)
    assert st.extension_rays == cnt.extension_rays == 0
    # each sample is 0 or the environment
    assert (out >= -1e-7).all() and (out <= np.array(env) + 1e-6).all()


@pytest.mark.parametrize("kind,objfix", [("cornell_box_obj", "cornell_obj"), ("veach_mis", "veach_obj"),
                                         ("cornell_box_obj", "glass_obj")])
def test_normals_device_code_matches_oracle(kind, objfix, request):
    obj = request.getfixturevalue(objfix)
    out, st, ref, cnt = pair(kind, obj, 48, 32, 2, NORMALS, (0.25, 0.5, 0.75))
    check_close(out, ref)
    assert st.camera_rays == cnt.camera_rays and st.shadow_rays == 0 == cnt.shadow_rays


def test_normals_are_unit_or_env(cornell_obj):
    """1 spp: a pixel is the hit's unit shading normal or the environment."""
    env = (7.0, 7.0, 7.0)
    out, st, ref, cnt = pair("cornell_box_obj", cornell_obj, 40, 40, 1, NORMALS, env)
    miss = np.all(ref == np.array(env), axis=1)
    assert miss.any() and (~miss).any()
    assert np.allclose(np.linalg.norm(ref[~miss], axis=1), 1.0, atol=1e-12)


def test_ao_black_environment_is_black(cornell_obj):
    """The reference scenes' environment is black: AO returns 0 everywhere."""
    out, st, ref, cnt = pair("cornell_box_obj", cornell_obj, 24, 24, 4, AO, (0.0, 0.0, 0.0))
    assert not out.any() and not ref.any()
    assert cnt.shadow_rays > 0


def test_ao_list_world_only_spheres_occlude(veach_obj):
    """veach_mis is a hitable_list: AO's t_max is NaN, so triangle hits never
    count (triangle.h `t < t_max`) and sphere hits always do (sphere.h
    `t > t_max` passes NaN).  The oracle gets this by running the restated
    code with NaN; the device code by testing only the list's spheres.  The
    plank / floor AO rays rarely point at the five small sphere lights, so
    the image is nearly the environment."""
    env = (1.0, 1.0, 1.0)
    out, st, ref, cnt = pair("veach_mis", veach_obj, 64, 48, 8, AO, env, seed=5)
    check_close(out, ref)
    assert ref.mean() > 0.9 and (ref < 1.0).any()    # some AO rays do reach a sphere
    assert cnt.tri_tests > 0


def test_unknown_integrator_rejected(cornell_obj):
    """Parameter checks (frt_shard_slot_count, no GPU needed) and the oracle
    both refuse an integrator the reference does not have."""
    with pytest.raises(frt.FrtError):
        frt.shard_slots(frt.RenderParams.make(8, 8, 1, integrator=7))
    assert len(frt.shard_slots(frt.RenderParams.make(8, 8, 1, integrator=AO))) == 32 * 32
    osc = oracle.OracleScene("cornell_box_obj", cornell_obj, 1.0)
    pix, out = np.zeros(1, np.int32), np.zeros(3)
    assert oracle.lib().ora_render_integrator(osc.ptr, 7, 8, 8, 1, 0, pix.ctypes.data, 1, 1, out.ctypes.data,
                                              None) == -3
