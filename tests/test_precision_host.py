"""The fp64 instantiation of the device code (frt_path.hpp / frt_device.hpp
with R = double; DESIGN.md "Precision") on the host through
frt_selftest_path_host (FRT_FLAG_FP64), against the fp64 oracle on the same
RNG streams.  The fp64 kernels exist for C3 (veach_mi: sphere lights down to
r = 0.033), where fp32 rounding moves samples onto or off the lights; in fp64
the replay matches the oracle to the fp32 film's own rounding."""
import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle


def light_patch(hs, nx, ny, centre, half):
    """Pixels of a (2 half + 1)^2 patch around the image of `centre` (camera.h:30-35)."""
    v = hs.view()
    o, llc = np.array(v.cam_origin[:]), np.array(v.cam_lower_left[:])
    H, V = np.array(v.cam_horizontal[:]), np.array(v.cam_vertical[:])
    u, w, _ = np.linalg.solve(np.stack([H, V, o - np.asarray(centre)], 1), o - llc)
    px, py = int(u * nx), int(w * ny)
    return np.array([y * nx + x for y in range(py - half, py + half + 1) for x in range(px - half, px + half + 1)],
                    np.int32)


def test_veach_small_lights_fp64(veach_obj):
    """veach_mis at 1920x1080: the patches around the r = 0.033 and r = 0.1
    lights (their silhouettes included), 256 spp.  fp64: the oracle's ray count
    and image (max deviation = half an fp32 ulp of the 901.8 radiance)."""
    nx, ny, spp = 1920, 1080, 256
    hs = frt.HostScene("veach_mis", veach_obj, nx / ny)
    pix = np.unique(np.concatenate([light_patch(hs, nx, ny, (-3.75, 0, 0), 8),
                                    light_patch(hs, nx, ny, (-1.25, 0, 0), 18)]))
    ref, cnt = oracle.OracleScene("veach_mis", veach_obj, nx / ny).render(nx, ny, spp, seed=5, pixels=pix)
    out, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, spp, seed=5, flags=frt.FRT_FLAG_FP64), pix)
    d = np.abs(out.astype(np.float64) - ref)
    assert st.fp64 == 1
    assert st.rays == cnt.rays
    assert (d <= 6.2e-5 * np.maximum(1.0, np.abs(ref))).all(), d.max()
    assert ref.max() > 100.0                                    # the patch does see the lights


@pytest.mark.parametrize("objfix", ["cornell_obj", "sphere_obj", "glass_obj"])
def test_bvh_scenes_fp64(objfix, request):
    """The fp64 binary-tree traversal and specular shading: ray counts equal,
    image within fp32 film rounding."""
    obj = request.getfixturevalue(objfix)
    nx, ny, spp = 32, 32, 8
    hs = frt.HostScene("cornell_box_obj", obj, nx / ny)
    pix = np.arange(nx * ny, dtype=np.int32)
    ref, cnt = oracle.OracleScene("cornell_box_obj", obj, nx / ny).render(nx, ny, spp, seed=3, pixels=pix)
    out, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, spp, seed=3, flags=frt.FRT_FLAG_FP64), pix)
    assert st.rays == cnt.rays
    assert np.abs(out.astype(np.float64) - ref).max() < 1e-5
