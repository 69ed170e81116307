"""Native host pipeline (libfrt.so, C++) against the C restatement (oracle/):
scene ingest, camera, lights, materials and the reference-topology BVH must be
identical (bit-exact fp64 / exact integers).  CPU only."""
import ctypes
import os
import re

import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "frt.h")).read()
    declared = set(re.findall(r"\b(frt_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(frt.EXPORTS)
    L = frt.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert L.frt_get_abi_version() == frt.ABI_VERSION == 9


def test_create_without_device_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(frt.FrtError):
        frt.Context(0)


def dfs(root, child, leaf_key):
    """Left-first DFS signature of a binary tree: nested tuples of leaf keys."""
    out = []
    st = [root]
    while st:
        x = st.pop()
        if x >= 0:
            out.append("N")
            st.append(child(x, 1))
            st.append(child(x, 0))
        else:
            out.append(leaf_key(~x))
    return out


def host_tree(a):
    ch = a["node_child"]
    return a["root"], (lambda x, s: int(ch[x][s]))


def oracle_tree(osc):
    _, left, right = osc.bvh()
    return 0, (lambda x, s: int(left[x] if s == 0 else right[x]))


@pytest.mark.parametrize("aspect", [1.0, 1920.0 / 1080.0])
def test_cornell_scene_matches_oracle(cornell_obj, aspect):
    hs = frt.HostScene("cornell_box_obj", cornell_obj, aspect)
    osc = oracle.OracleScene("cornell_box_obj", cornell_obj, aspect)
    a = hs.arrays()
    ov, om = osc.tris()
    assert hs.info.n_tris == osc.info.n_tris == 36
    assert np.array_equal(a["tri_v"], ov)                       # bit-exact vertices (float parse + triangulation)
    assert np.array_equal(a["tri_material"], om)
    assert list(a["lights"]) == list(osc.lights()) and len(a["lights"]) == 2
    # camera (camera.h:10-28) bit-exact
    v = hs.view()
    cam = np.concatenate([list(v.cam_origin), list(v.cam_lower_left), list(v.cam_horizontal),
                          list(v.cam_vertical), list(v.cam_u), list(v.cam_v), [v.cam_lens_radius]])
    assert np.array_equal(cam, osc.camera())
    # materials: the oracle's 20-double description
    mats = np.array([[m.type, *m.albedo, *m.emit, *m.specular, m.exponent, m.ior, m.distribution, m.alpha,
                      *m.eta, *m.k, m.texture, *m.tex_odd, *m.tex_scale] for m in
                     (ctypes.cast(v.materials, ctypes.POINTER(frt.Material))[i] for i in range(v.n_materials))])
    assert np.array_equal(mats, osc.materials())


def test_cornell_bvh_topology_matches_oracle(cornell_obj):
    hs = frt.HostScene("cornell_box_obj", cornell_obj, 1.0)
    osc = oracle.OracleScene("cornell_box_obj", cornell_obj, 1.0)
    a = hs.arrays()
    r1, c1 = host_tree(a)
    r2, c2 = oracle_tree(osc)
    assert dfs(r1, c1, lambda p: p) == dfs(r2, c2, lambda p: p)
    assert hs.info.n_nodes == osc.info.n_nodes == 35
    assert hs.info.bvh_depth == osc.info.bvh_depth
    # node boxes (DFS order) identical
    boxes_o, _, _ = osc.bvh()
    order = []
    st = [r1]
    while st:
        x = st.pop()
        if x >= 0:
            order.append(x)
            st.append(c1(x, 1)); st.append(c1(x, 0))
    assert np.array_equal(a["node_box"][order], boxes_o)


def test_tessellated_bvh_topology_matches_oracle(cornell_obj, tmp_path):
    # many equal sort keys: exercises glibc merge-sort tie order (bvh.h comparators)
    dst = str(tmp_path / "tess.obj")
    frt.write_tessellated_obj(cornell_obj, 4, dst)
    hs = frt.HostScene("cornell_box_obj", dst, 1.0)
    osc = oracle.OracleScene("cornell_box_obj", dst, 1.0)
    assert hs.info.n_tris == osc.info.n_tris == 17 * 2 * 16 + 2
    a = hs.arrays()
    ov, _ = osc.tris()
    assert np.array_equal(a["tri_v"], ov)
    r1, c1 = host_tree(a)
    r2, c2 = oracle_tree(osc)
    assert dfs(r1, c1, lambda p: p) == dfs(r2, c2, lambda p: p)


def test_veach_scene_matches_oracle(veach_obj):
    hs = frt.HostScene("veach_mis", veach_obj, 1920.0 / 1080.0)
    osc = oracle.OracleScene("veach_mis", veach_obj, 1920.0 / 1080.0)
    a = hs.arrays()
    ov, _ = osc.tris()
    assert hs.info.n_tris == 12 and hs.info.n_spheres == 10 and hs.info.world_kind == frt.FRT_WORLD_LIST
    assert np.array_equal(a["tri_v"], ov)
    assert len(a["list"]) == 17 and list(a["lights"]) == list(osc.lights())
    # plates alias the floor's first six vertices
    assert np.array_equal(a["tri_v"][4], a["tri_v"][0])
    # smooth normals of the axis-aligned floor/wall are exact
    n = np.ctypeslib.as_array(ctypes.cast(hs.view().tri_n, ctypes.POINTER(ctypes.c_double)), shape=(12 * 9,))
    n = n.reshape(12, 3, 3)
    assert np.allclose(np.abs(n).max(axis=2), 1.0)


def test_shards_partition_the_frame():
    for nx, ny, tile, n in [(256, 256, 32, 1), (1920, 1080, 32, 8), (100, 37, 16, 3), (7, 5, 8, 4)]:
        seen = []
        for r in range(n):
            p = frt.RenderParams.make(nx, ny, 4, tile_size=tile, shard_index=r, shard_count=n)
            s = frt.shard_slots(p)
            seen.append(s[s >= 0])
        allp = np.concatenate(seen)
        assert len(allp) == nx * ny and len(np.unique(allp)) == nx * ny


def test_pfm_writer_matches_reference_layout(tmp_path):
    film = (np.arange(2 * 3 * 3, dtype=np.float32).reshape(2, 3, 3) * 0.1 + np.float32(1 / 3))
    p1, p2 = str(tmp_path / "a.pfm"), str(tmp_path / "b.pfm")
    frt.write_pfm(p1, film)
    oracle.lib().ora_write_pfm(p2.encode(), 3, 2, oracle.darr(film.astype(np.float64).ravel())[1])
    assert open(p1, "rb").read() == open(p2, "rb").read()


@pytest.mark.parametrize("objfix", ["glossy_floor_obj", "sphere_obj", "mirror_obj", "glass_obj"])
def test_specular_scene_materials_and_topology(objfix, request):
    """Specular CornellBox variants: the host loader and the oracle loader agree
    on every material (type, Kd, Ks, Ns, Ni via mesh_loader.cpp:59-112) and on
    the BVH topology."""
    obj = request.getfixturevalue(objfix)
    hs = frt.HostScene("cornell_box_obj", obj, 1.0)
    osc = oracle.OracleScene("cornell_box_obj", obj, 1.0)
    v = hs.view()
    mats = np.array([[m.type, *m.albedo, *m.emit, *m.specular, m.exponent, m.ior, m.distribution, m.alpha,
                      *m.eta, *m.k, m.texture, *m.tex_odd, *m.tex_scale] for m in
                     (ctypes.cast(v.materials, ctypes.POINTER(frt.Material))[i] for i in range(v.n_materials))])
    assert np.array_equal(mats, osc.materials())
    types = set(mats[:, 0].astype(int))
    want = frt.FRT_MAT_DIELECTRIC if objfix == "glass_obj" else frt.FRT_MAT_MODIFIED_PHONG
    assert want in types
    assert hs.info.n_nodes == osc.info.n_nodes and hs.info.bvh_depth == osc.info.bvh_depth


def test_one_hip_and_rccl_runtime_per_process():
    """libfrt.so links librccl.so.1 / libamdhip64.so.7 by soname; with torch imported
    first (as the binding does) those sonames resolve to torch's bundled copies, so the
    process holds one HIP runtime and one RCCL (frt_render_multi's RCCL and
    torch.distributed's are the same library)."""
    import torch  # noqa: F401
    frt.lib()
    maps = open("/proc/self/maps").read().splitlines()
    libs = {l.split()[-1] for l in maps if "librccl" in l or "libamdhip64" in l}
    assert len([x for x in libs if "librccl" in x]) <= 1, libs
    assert len([x for x in libs if "libamdhip64" in x]) == 1, libs


def test_work_granule_bounded_workspace():
    """The work granule (frt_render.hip work_granule): the per-item
    sample cap grows the chunk count with spp, but the (chunk, slot) partial
    sums stay bounded by a fixed multiple of the resident lanes at any spp, and
    the bench configs get their chunk counts (round 4: 8 samples an item, at
    most 384 items per resident lane, so that an eighth of the frame still has
    ~40 items per lane -- the N-way split's balance with whole-frame chunks;
    Cornell 57 chunks of 9 samples, cornell_1m 64 of 8 at 1080p 512 spp)."""
    P, AO = frt.FRT_INTEGRATOR_PATH, frt.FRT_INTEGRATOR_AO
    slots_1080 = 60 * 34 * 32 * 32                         # 1920x1080 in 32x32 tiles
    slots_4k = 120 * 68 * 32 * 32
    lanes_lds, lanes_hbm = 256 * 5 * 256, 256 * 6 * 256    # resident lanes of the two plans
    assert frt.work_granule(P, 512, slots_1080, lanes_lds) == (9, 57)
    assert frt.work_granule(P, 512, slots_1080, lanes_hbm) == (8, 64)
    assert frt.work_granule(AO, 512, slots_1080, lanes_lds)[1] == 6
    for spp, slots, lanes in ((8192, slots_1080, lanes_lds), (50000, slots_1080, lanes_lds),
                              (12400, slots_4k, lanes_hbm), (1 << 20, slots_4k, lanes_lds)):
        spi, k = frt.work_granule(P, spp, slots, lanes)
        assert k * spi >= spp and (k - 1) * spi < spp          # the chunks cover the samples exactly once
        items = k * slots
        assert items <= max(384 * lanes, slots)                 # bounded workspace: 12 B an item
        assert items + (lanes // 64) * (64 + 64) < 2 ** 32      # fits the 32-bit work queue
    # tiny frames keep ~40 items per lane (the first rule)
    spi, k = frt.work_granule(P, 4096, 64 * 64, lanes_lds)
    assert k * 64 * 64 <= 48 * lanes_lds and spi >= 1
    # the caller's samples_per_item wins
    assert frt.work_granule(P, 100, slots_1080, lanes_lds, spi_req=7) == (7, 15)


def test_frame_size_limit():
    """Pixel indices are int32 (frt_shard_slots, the kernels' item state): a
    frame of 2^31 or more pixels is rejected as bad params, not wrapped."""
    with pytest.raises(frt.FrtError):
        frt.shard_slots(frt.RenderParams.make(46341, 46341, 1))          # 2,147,488,281 px
    assert len(frt.shard_slots(frt.RenderParams.make(64, 48, 1, tile_size=16))) == 64 * 48

