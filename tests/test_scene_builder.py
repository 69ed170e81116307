"""The incremental scene builder (frt_scene_new ... frt_scene_finish: what
main.cpp's scene functions do with create_triangle_mesh(file, toWorld, bsdf),
spheres, the camera and create_bvh) against the oracle's builder, and the
metal / rough_conductor shading code run on the host against the oracle.
Scene arrays are bit-exact (fp64 host pipeline on both sides)."""
import ctypes

import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle
import scene_specs as SS


def both(spec, aspect=1.0):
    return frt.HostScene.from_spec(spec, aspect), oracle.OracleScene.from_spec(spec, aspect)


def host_materials(hs):
    v = hs.view()
    return np.array([[m.type, *m.albedo, *m.emit, *m.specular, m.exponent, m.ior, m.distribution, m.alpha,
                      *m.eta, *m.k, m.texture, *m.tex_odd, *m.tex_scale] for m in
                     (ctypes.cast(v.materials, ctypes.POINTER(frt.Material))[i] for i in range(v.n_materials))])


@pytest.mark.parametrize("world", ["bvh", "list"])
def test_builder_scene_matches_oracle(world):
    hs, osc = both(SS.cornell_conductors(world=world), 16 / 9)
    assert (hs.info.n_tris, hs.info.n_spheres, hs.info.n_materials, hs.info.n_lights, hs.info.world_kind) == \
        (osc.info.n_tris, osc.info.n_spheres, osc.info.n_materials, osc.info.n_lights, osc.info.world_kind)
    a = hs.arrays()
    tv, tm = osc.tris()
    assert np.array_equal(a["tri_v"], tv) and np.array_equal(a["tri_material"], tm)
    assert np.array_equal(host_materials(hs), osc.materials())
    assert np.array_equal(a["lights"], osc.lights())
    if world == "bvh":
        b, l, r = osc.bvh()
        assert np.array_equal(a["node_box"], b)
        assert np.array_equal(a["node_child"][:, 0], l) and np.array_equal(a["node_child"][:, 1], r)
    else:
        # insertion order: the Cornell triangles, the two spheres, the cube's triangles
        n = hs.info.n_tris
        assert list(a["list"]) == list(range(n - 12)) + [frt.FRT_PRIM_SPHERE | k for k in range(2)] + \
            list(range(n - 12, n))
    v = hs.view()
    cam = np.concatenate([list(v.cam_origin), list(v.cam_lower_left), list(v.cam_horizontal),
                          list(v.cam_vertical), list(v.cam_u), list(v.cam_v), [v.cam_lens_radius]])
    assert np.array_equal(cam, osc.camera())


def test_builder_transform_and_override():
    """toWorld moves the cube's vertices (point transform) and every cube
    triangle takes the one override material (triangle.cpp:36-52)."""
    spec = SS.cornell_conductors()
    hs = frt.HostScene.from_spec(spec, 1.0)
    a = hs.arrays()
    cube = a["tri_v"][-12:].reshape(-1, 3)
    M = np.array(spec["objects"][-1]["to_world"]).reshape(4, 4)
    corners = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], float)
    want = corners @ M[:3, :3].T + M[:3, 3]
    assert all(np.abs(want - c).sum(1).min() < 1e-12 for c in cube)
    mats = host_materials(hs)
    cm = set(a["tri_material"][-12:])
    assert len(cm) == 1 and mats[cm.pop()][0] == frt.MAT_TYPES["rough_conductor"]


def test_builder_reproduces_named_scene(cornell_obj):
    """The builder with CornellBox-Original alone is cornell_box_obj (main.cpp:222-252)."""
    hs = frt.HostScene.from_spec({"objects": [{"obj": cornell_obj, "geo": True}], "camera": SS.CORNELL_CAM}, 1.0)
    ref = frt.HostScene("cornell_box_obj", cornell_obj, 1.0)
    a, b = hs.arrays(), ref.arrays()
    for k in ("tri_v", "tri_material", "node_box", "node_child", "lights"):
        assert np.array_equal(a[k], b[k]), k


def test_builder_errors(cornell_obj):
    singular = dict(SS.cornell_conductors())
    singular["objects"] = [{"obj": SS.CUBE_OBJ, "to_world": [0.0] * 16}]
    with pytest.raises(frt.FrtError):
        frt.HostScene.from_spec(singular, 1.0)
    bad = {"objects": [{"sphere": (0, 0, 0), "radius": 1.0, "material": SS.rough("ggx", 0.0)}], "camera": SS.CORNELL_CAM}
    with pytest.raises(frt.FrtError):
        frt.HostScene.from_spec(bad, 1.0)
    missing = {"objects": [{"obj": "/nonexistent.obj"}], "camera": SS.CORNELL_CAM}
    with pytest.raises(frt.FrtError):
        frt.HostScene.from_spec(missing, 1.0)


@pytest.mark.parametrize("sphere_dist,cube_dist", [("ggx", "beckmann"), ("beckmann", "ggx")])
def test_conductor_shading_host_vs_oracle(sphere_dist, cube_dist):
    """The megakernel's per-lane path code (fp32, frt_path.hpp: metal + rough
    conductor specular branch, NEE with their pdfs) run on the host against the
    fp64 oracle on the same streams."""
    spec = SS.cornell_conductors(sphere_dist, cube_dist)
    hs, osc = both(spec)
    nx = ny = 48
    pix = np.arange(nx * ny, dtype=np.int32)
    g, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 8, seed=5), pix)
    ref, cnt = osc.render(nx, ny, 8, seed=5)
    g = g.reshape(-1, 3).astype(np.float64)
    assert st.samples == cnt.samples and st.camera_rays == cnt.camera_rays
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert float(np.sqrt(np.mean((g - ref) ** 2))) < 1e-3


@pytest.mark.parametrize("world", ["bvh", "list"])
def test_textured_scene_host_vs_oracle(world):
    """checker textures (texture.h:30-49) at OBJ-vt and sphere uv: the builder keeps the
    vt (mesh_loader.cpp:34-38; 0 for meshes without), and the device path code run on the
    host matches the oracle; without the textures the image differs."""
    spec = SS.cornell_textured(world)
    hs, osc = both(spec)
    assert np.array_equal(host_materials(hs), osc.materials())
    v = hs.view()
    uv = np.ctypeslib.as_array(ctypes.cast(v.tri_uv, ctypes.POINTER(ctypes.c_double)), shape=(v.n_tris * 6,))
    assert not uv[:-12].any()                                           # CornellBox-Original has no vt
    assert sorted(set(uv[-12:])) == [0.0, 1.0] and uv[-12:].sum() == 6.0  # the quad's two triangles
    nx = ny = 48
    g, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 8, seed=5), np.arange(nx * ny, dtype=np.int32))
    ref, cnt = osc.render(nx, ny, 8, seed=5)
    assert st.camera_rays == cnt.camera_rays
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert float(np.sqrt(np.mean((g.reshape(-1, 3) - ref) ** 2))) < 1e-3
    plain = dict(spec, objects=[{k: ({kk: vv for kk, vv in x.items() if kk != "checker"} if isinstance(x, dict) else x)
                                 for k, x in o.items()} for o in spec["objects"]])
    ref0, _ = oracle.OracleScene.from_spec(plain, 1.0).render(nx, ny, 8, seed=5)
    assert float(np.sqrt(np.mean((ref0 - ref) ** 2))) > 1e-2


def test_texture_rejections():
    """checker on a light's emission or on metal's albedo is not mapped: upload refuses it
    loudly; an unknown texture kind fails in the builder."""
    light = {"objects": [{"obj": SS.CORNELL_OBJ, "geo": True},
                         {"sphere": (0, 1, 0), "radius": 0.1, "where": "both",
                          "material": SS.checker({"type": "diffuse_light", "emit": (4, 4, 4)}, (1, 1, 1), (2, 2))}],
             "camera": SS.CORNELL_CAM}
    hs = frt.HostScene.from_spec(light, 1.0)
    with pytest.raises(frt.FrtError):
        frt.selftest_path_host(hs, frt.RenderParams.make(4, 4, 1), np.arange(16, dtype=np.int32))
    m = frt.Material.from_spec({"type": "lambertian", "albedo": (0.5, 0.5, 0.5)})
    m.texture = 7
    s = ctypes.c_void_p()
    L = frt.lib()
    assert L.frt_scene_new(ctypes.byref(s)) == 0
    c = (ctypes.c_double * 3)(0, 0, 0)
    assert L.frt_scene_add_sphere(s, c, ctypes.c_double(1.0), ctypes.byref(m), 1) != 0
    L.frt_scene_destroy(s)


def test_ao_rejects_metal():
    """ao::Li asks metal's constant_pdf to generate(), which throws (pdf.h:195-198)."""
    hs, osc = both(SS.cornell_conductors())
    with pytest.raises(frt.FrtError):
        frt.selftest_path_host(hs, frt.RenderParams.make(8, 8, 1, integrator=frt.FRT_INTEGRATOR_AO),
                               np.arange(64, dtype=np.int32))
    with pytest.raises(RuntimeError):
        osc.render(8, 8, 1, integrator=2)


def test_binned_sah_tree_host(cornell_obj):
    """frt_scene_build_bvh_sah: a valid tree over every world prim, and the
    device path code over it (host replay) matches the oracle's render."""
    spec = SS.cornell_conductors(world="list")
    hs = frt.HostScene.from_spec(spec, 1.0)
    n = hs.info.n_list
    hs.build_bvh_sah()
    a = hs.arrays()
    assert hs.info.world_kind == 0 and hs.info.n_nodes == n - 1
    child = a["node_child"].reshape(-1)
    assert sorted(~c for c in child if c < 0) == sorted(list(range(hs.info.n_tris)) +
                                                       [frt.FRT_PRIM_SPHERE | k for k in range(2)])
    assert sorted(c for c in child if c >= 0) == [i for i in range(n - 1) if i != a["root"]]
    boxes = a["node_box"]
    assert np.all(boxes[:, :3] <= boxes[:, 3:])
    nx = ny = 40
    g, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 4, seed=8), np.arange(nx * ny, dtype=np.int32))
    ref, cnt = oracle.OracleScene.from_spec(dict(spec, world="bvh"), 1.0).render(nx, ny, 4, seed=8)
    assert st.camera_rays == cnt.camera_rays
    assert float(np.sqrt(np.mean((g.reshape(-1, 3) - ref) ** 2))) < 1e-3


@pytest.mark.parametrize("world", ["bvh", "list"])
def test_image_textured_scene_host_vs_oracle(world):
    """image_texture (texture.h:51-95): an 8-bit sRGB image on the vt-mapped floor quad and
    on a modified_phong sphere, an HDR float image on a rough conductor sphere; the device
    path code run on the host matches the oracle, and without the images the film differs."""
    spec = SS.cornell_image_textured(world)
    hs, osc = both(spec)
    assert hs.view().n_images == 2
    nx = ny = 48
    g, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 8, seed=5), np.arange(nx * ny, dtype=np.int32))
    ref, cnt = osc.render(nx, ny, 8, seed=5)
    assert st.camera_rays == cnt.camera_rays
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert float(np.sqrt(np.mean((g.reshape(-1, 3) - ref) ** 2))) < 1e-3
    plain = dict(spec, objects=[{k: ({kk: vv for kk, vv in x.items() if kk != "image"} if isinstance(x, dict) else x)
                                 for k, x in o.items()} for o in spec["objects"]])
    ref0, _ = oracle.OracleScene.from_spec(plain, 1.0).render(nx, ny, 8, seed=5)
    assert float(np.sqrt(np.mean((ref0 - ref) ** 2))) > 1e-2


def test_image_texture_rejections():
    """An image index with no image behind it fails in the builder; an image on a light's
    emission is refused at upload; malformed images fail in frt_scene_add_image."""
    L = frt.lib()
    s = ctypes.c_void_p()
    assert L.frt_scene_new(ctypes.byref(s)) == 0
    m = frt.Material.from_spec({"type": "lambertian", "albedo": (0.5, 0.5, 0.5), "image": 0})
    c = (ctypes.c_double * 3)(0, 0, 0)
    assert L.frt_scene_add_sphere(s, c, ctypes.c_double(1.0), ctypes.byref(m), 1) != 0   # no image 0 yet
    img = np.zeros((2, 3, 3), np.uint8)
    idx = ctypes.c_int(-1)
    assert L.frt_scene_add_image(s, ctypes.byref(frt.Image(3, 2, frt.FRT_IMAGE_SRGB8, 0, img.ctypes.data)),
                                 ctypes.byref(idx)) == 0 and idx.value == 0
    assert L.frt_scene_add_sphere(s, c, ctypes.c_double(1.0), ctypes.byref(m), 1) == 0
    assert L.frt_scene_add_image(s, ctypes.byref(frt.Image(0, 2, frt.FRT_IMAGE_SRGB8, 0, img.ctypes.data)),
                                 ctypes.byref(idx)) != 0
    assert L.frt_scene_add_image(s, ctypes.byref(frt.Image(3, 2, 5, 0, img.ctypes.data)), ctypes.byref(idx)) != 0
    L.frt_scene_destroy(s)
    light = {"objects": [{"obj": SS.CORNELL_OBJ, "geo": True},
                         {"sphere": (0, 1, 0), "radius": 0.1, "where": "both",
                          "material": {"type": "diffuse_light", "emit": (4, 4, 4), "image": 0}}],
             "camera": SS.CORNELL_CAM, "images": [{"data": SS.test_image(4, 4)}]}
    hs = frt.HostScene.from_spec(light, 1.0)
    with pytest.raises(frt.FrtError):
        frt.selftest_path_host(hs, frt.RenderParams.make(4, 4, 1), np.arange(16, dtype=np.int32))
