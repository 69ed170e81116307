"""The megakernel's per-lane path code (csrc/frt_path.hpp: traversal, NEE, MIS,
bounce) compiled for the host via the frt_selftest_path_host hook, against the
fp64 oracle on the same RNG streams.  Runs on CPU, so logic errors in the
device code are caught before a GPU run.  Tolerance: RMSE <= 1e-3 (the gate);
in practice fp32-vs-fp64 rounding gives ~1e-7."""
import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle


def run(kind, obj, nx, ny, spp, seed, pixels=None, max_depth=33):
    hs = frt.HostScene(kind, obj, nx / ny)
    pix = np.arange(nx * ny, dtype=np.int32) if pixels is None else pixels
    out, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, spp, seed=seed, max_depth=max_depth), pix)
    ref, cnt = oracle.OracleScene(kind, obj, nx / ny).render(nx, ny, spp, seed=seed, pixels=pix)
    return out, st, ref, cnt


def test_cornell(cornell_obj):
    out, st, ref, cnt = run("cornell_box_obj", cornell_obj, 48, 48, 16, seed=0)
    e = float(np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2)))
    assert e < 1e-4, e
    assert st.camera_rays == cnt.camera_rays
    assert abs(st.rays - cnt.rays) <= 1e-3 * cnt.rays


def test_cornell_widescreen_sampled_pixels(cornell_obj):
    pix = np.linspace(0, 1920 * 1080 - 1, 300).astype(np.int32)
    out, st, ref, cnt = run("cornell_box_obj", cornell_obj, 1920, 1080, 32, seed=7, pixels=pix)
    assert float(np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2))) < 1e-4


def test_veach(veach_obj):
    out, st, ref, cnt = run("veach_mis", veach_obj, 48, 32, 32, seed=1)
    assert float(np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2))) < 1e-3
    assert st.rays == pytest.approx(cnt.rays, rel=1e-3)


def test_tessellated(cornell_obj, tmp_path):
    dst = str(tmp_path / "t.obj")
    frt.write_tessellated_obj(cornell_obj, 6, dst)
    out, st, ref, cnt = run("cornell_box_obj", dst, 32, 32, 8, seed=3)
    assert float(np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2))) < 1e-4


@pytest.mark.parametrize("kind,objfix", [("cornell_box_obj", "cornell_obj"), ("veach_mis", "veach_obj"),
                                         ("cornell_box_obj", "sphere_obj"), ("cornell_box_obj", "glass_obj")])
def test_pssmlt_eye_paths(kind, objfix, request):
    """PSS-MLT eye paths (frt_mlt.hpp, pssmlt.cpp:105-277) vs the oracle on the
    bootstrap primary-sample stream: film position and contribution."""
    obj = request.getfixturevalue(objfix)
    nx, ny, seed, n = 96, 64, 3, 400
    hs = frt.HostScene(kind, obj, nx / ny)
    got = frt.selftest_mlt_paths_host(hs, nx, ny, seed, n)
    osc = oracle.OracleScene(kind, obj, nx / ny)
    ref = np.zeros((n, 6))
    for i in range(n):
        pr = oracle.darr([oracle.rng_uniform(seed ^ 0xB5297A4D, i, 0, d) for d in range(92)])
        out = oracle.darr(np.zeros(6))
        oracle.lib().ora_mlt_eye_path(osc.ptr, nx, ny, pr[1], out[1])
        ref[i] = out[0]
    assert np.abs(got[:, :2] - ref[:, :2]).max() < 1e-3                      # film position (pixels)
    rel = np.abs(got[:, 2:] - ref[:, 2:]).max(axis=1) / (np.abs(ref[:, 2:]).max(axis=1) + 1e-6)
    assert (rel > 1e-3).sum() <= 1
    assert got[:, 5].mean() == pytest.approx(osc.mlt_bootstrap(nx, ny, seed, n), rel=1e-5)


@pytest.mark.parametrize("kind,objfix,tess", [("cornell_box_obj", "cornell_obj", 0),
                                              ("cornell_box_obj", "cornell_obj", 5),
                                              ("veach_mis", "veach_obj", 0)])
def test_leaf_size_invariance(kind, objfix, tess, request, tmp_path, monkeypatch):
    """Multi-triangle leaves (collapse_leaves) change node visits, never hits:
    the closest hit is the (t, DFS rank) minimum in any visit order, so leaf
    sizes 1 (the reference's one-prim leaves), 2 and 4 give bit-identical
    samples and identical ray counts."""
    obj = request.getfixturevalue(objfix)
    if tess:
        obj2 = str(tmp_path / "t.obj")
        frt.write_tessellated_obj(obj, tess, obj2)
        obj = obj2
    nx, ny = 40, 30
    hs = frt.HostScene(kind, obj, nx / ny)
    pix = np.arange(nx * ny, dtype=np.int32)
    res = {}
    for leaf in (1, 2, 4):
        monkeypatch.setenv("FRT_LEAF_SIZE", str(leaf))
        out, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 8, seed=11), pix)
        res[leaf] = (out, st.rays)
    for leaf in (2, 4):
        assert np.array_equal(res[leaf][0], res[1][0])
        assert res[leaf][1] == res[1][1]


@pytest.mark.parametrize("kind,objfix,tess", [("cornell_box_obj", "cornell_obj", 0),
                                              ("cornell_box_obj", "cornell_obj", 12),
                                              ("obj_smooth", "cornell_obj", 5)])
def test_bvh4_matches_binary(kind, objfix, tess, request, tmp_path):
    """The 4-wide quantized BVH (trace_bvh4), with an 8-entry stack so the
    private overflow entries are used, returns the binary traversal's hits bit
    for bit: identical samples and ray counts."""
    obj = request.getfixturevalue(objfix)
    if tess:
        obj2 = str(tmp_path / "t.obj")
        frt.write_tessellated_obj(obj, tess, obj2)
        obj = obj2
    nx, ny = 40, 30
    hs = frt.HostScene(kind, obj, nx / ny)
    pix = np.arange(nx * ny, dtype=np.int32)
    wide, st4 = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 8, seed=13), pix)
    bin2, st2 = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 8, seed=13, flags=frt.FRT_FLAG_BVH2), pix)
    assert np.array_equal(wide, bin2)
    assert st4.rays == st2.rays
    assert st4.stack_entries == 8 and 0 < st4.bvh_depth < st2.bvh_depth   # the wide tree was traversed


@pytest.mark.parametrize("objfix", ["sphere_obj", "mirror_obj", "glass_obj"])
def test_specular_scenes(objfix, request):
    """modified_phong (Sphere, Mirror: Ns 1024 lobes) and dielectric (Glass):
    the specular branch of path::Li (path.cpp:78-95) on the host build of the
    device code vs the oracle, same streams."""
    obj = request.getfixturevalue(objfix)
    out, st, ref, cnt = run("cornell_box_obj", obj, 40, 40, 16, seed=3)
    assert float(np.sqrt(np.mean((out.astype(np.float64).reshape(-1, 3) - ref.reshape(-1, 3)) ** 2))) < 1e-4
    assert st.rays == pytest.approx(cnt.rays, rel=1e-3)
    assert float(ref.mean()) > 0.01


def test_bvh4_tiny_far_nodes(tmp_path):
    """4-wide nodes tiny against their distance from the ray origin, where an
    axis' quantized planes round to one value (255 * a vanishes in the slab
    FMA): a real child's hit is then tn == tf and must stay a hit.  (An empty
    slot, an inverted box, passes the same test only when all three axes
    collapse and their entry distances are equal in fp32; its ref is then a
    one-primitive leaf of the scene's first primitive, which cannot change the
    answer: build_bvh4, ADVICE r2.  This scene collapses the z axis only.)  A 20 x 20 grid of
    1e-6-sized triangles around the origin (nodes of ~1e-5, the padding of a
    unit-scale scene) seen from 1e3 away (farther, the reference's own
    t_min = EPSILON * |o| would cull the hits, parallel_bvh.h:46-51).  Shading
    normals (normals_renderer::Li) of the 4-wide traversal vs the binary one
    and the oracle."""
    lines, k = [], 1
    for i in range(20):
        for j in range(20):
            x, y = (i - 10) * 2e-6, (j - 10) * 2e-6
            z = 1e-7 * ((i * 7 + j * 3) % 5)
            lines += [f"v {x!r} {y!r} {z!r}", f"v {x + 1e-6!r} {y!r} {z!r}", f"v {x!r} {y + 1e-6!r} {z + 5e-7!r}"]
            lines.append(f"f {k} {k + 1} {k + 2}")
            k += 3
    obj = tmp_path / "tiny.obj"
    obj.write_text("\n".join(lines) + "\n")
    nx, ny = 40, 40
    cam = {"lookfrom": (0.0, 0.0, 1e3), "lookat": (0.0, 0.0, 0.0), "vup": (0.0, 1.0, 0.0),
           "vfov": 2.4e-6, "aperture": 0.0, "focus": 1e3}
    spec = {"objects": [{"obj": str(obj), "geo": True,
                         "bsdf": {"type": "lambertian", "albedo": (0.5, 0.5, 0.5)}}],
            "camera": cam, "world": "bvh"}
    env = (0.25, 0.5, 0.75)
    hs = frt.HostScene.from_spec(spec, 1.0)
    hs.set_env(env)
    pix = np.arange(nx * ny, dtype=np.int32)
    p = dict(integrator=frt.FRT_INTEGRATOR_NORMALS)
    wide, st4 = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 1, seed=1, **p), pix)
    bin2, st2 = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 1, seed=1, flags=frt.FRT_FLAG_BVH2, **p), pix)
    osc = oracle.OracleScene.from_spec(spec, 1.0)
    osc.set_env(env)
    ref, _ = osc.render(nx, ny, 1, seed=1, pixels=pix, integrator=3)
    assert st4.bvh_depth < st2.bvh_depth                       # the 4-wide tree was traversed
    hit = np.abs(ref - env).max(axis=1) > 1e-6
    assert hit.mean() > 0.05
    assert np.array_equal(wide, bin2)
    # fp32 vs fp64: a few edge pixels may round to the other side
    assert (np.abs(wide.astype(np.float64) - ref).max(axis=1) > 1e-3).mean() < 0.01
