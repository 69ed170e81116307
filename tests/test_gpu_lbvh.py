"""Alternative BVHs: the GPU builders (frt_scene_build_bvh_gpu_algo, csrc/frt_lbvh.hip:
Morton keys and a device radix sort, then PLOC clustering or the Karras
hierarchy with atomic refit, or a top-down binned SAH on the device) and the
host binned SAH builder (frt_scene_build_bvh_sah).  Either tree replaces the
reference-topology tree; hits can differ from the oracle's only at exact t ties
between primitives, so renders meet the same RMSE gate and the ray counts agree
within rounding-divergence noise."""
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


def check_tree(hs, n_prims):
    a = hs.arrays()
    assert hs.info.world_kind == 0 and hs.info.n_nodes == n_prims - 1 and a["root"] == 0
    child = a["node_child"]
    leaves = sorted(~c for c in child.reshape(-1) if c < 0)
    assert len(leaves) == n_prims and len(set(leaves)) == n_prims      # every prim in exactly one leaf
    internal = sorted(c for c in child.reshape(-1) if c >= 0)
    assert internal == list(range(1, n_prims - 1))                    # every node but the root has one parent


def build(hs, ctx, how):
    return hs.build_bvh_gpu(ctx, how) if how in ("ploc", "lbvh", "gsah") else hs.build_bvh_sah()


@pytest.mark.parametrize("how", ["ploc", "lbvh", "gsah", "sah"])
@pytest.mark.parametrize("spec_name", ["cornell", "conductors"])
def test_gpu_bvh_render_matches_oracle(ctx, cornell_obj, spec_name, how):
    spec = ({"objects": [{"obj": cornell_obj, "geo": True}], "camera": SS.CORNELL_CAM} if spec_name == "cornell"
            else SS.cornell_conductors())
    spec = dict(spec, world="list")                                      # skip the host SAH build
    nx, ny, spp = 96, 72, 16
    hs = frt.HostScene.from_spec(spec, nx / ny)
    n = hs.info.n_list
    ms = build(hs, ctx, how)
    check_tree(hs, n)
    print(spec_name, how, "build", ms, "ms depth", hs.info.bvh_depth)
    ctx.upload(hs)
    film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=5))
    ref, cnt = oracle.OracleScene.from_spec(dict(spec, world="bvh"), nx / ny).render(nx, ny, spp, seed=5)
    assert st.camera_rays == cnt.camera_rays
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert rmse(film, ref) <= 1e-3


@pytest.mark.parametrize("how", ["ploc", "lbvh", "gsah", "sah"])
@pytest.mark.parametrize("flags", [0, frt.FRT_FLAG_BVH2])
def test_gpu_bvh_large_scene_matches_host_tree(ctx, cornell_obj, tmp_path, flags, how):
    """~20k triangles (HBM plan: BVH4Q from the GPU-built binary tree, or binary
    with FRT_FLAG_BVH2): same image as the host SAH tree up to exact-tie noise."""
    dst = str(tmp_path / "t24.obj")
    frt.write_tessellated_obj(cornell_obj, 24, dst)
    nx, ny, spp = 128, 96, 8
    sah = frt.HostScene("cornell_box_obj", dst, nx / ny)
    ctx.upload(sah)
    ref, st0 = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=1, flags=flags))
    hs = frt.HostScene.from_spec({"objects": [{"obj": dst, "geo": True}], "camera": SS.CORNELL_CAM, "world": "list"},
                                 nx / ny)
    ms = build(hs, ctx, how)
    check_tree(hs, sah.info.n_tris)
    ctx.upload(hs)
    film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=1, flags=flags))
    print("t24", how, "build", ms, "ms; depth", hs.info.bvh_depth, "vs reference", sah.info.bvh_depth)
    assert st.scene_in_lds == 0 and st.camera_rays == st0.camera_rays
    assert abs(st.rays - st0.rays) / st0.rays < 1e-3
    assert rmse(film, ref) <= 1e-4


def test_bench_default_tree_all_integrators(ctx, cornell_obj):
    """The bench's default scene build (binned SAH tree built on the GPU)
    against the oracle (reference topology) for every integrator: path,
    PSS-MLT short chains, AO, normals."""
    nx, ny = 64, 48
    hs = frt.HostScene.from_spec({"objects": [{"obj": cornell_obj, "geo": True}], "camera": frt.CORNELL_CAMERA,
                                  "world": "list"}, nx / ny)
    hs.build_bvh_gpu(ctx)
    hs.set_env((1.0, 1.0, 1.0))
    ctx.upload(hs)
    osc = oracle.OracleScene("cornell_box_obj", cornell_obj, nx / ny)
    osc.set_env((1.0, 1.0, 1.0))
    for integ in (frt.FRT_INTEGRATOR_PATH, frt.FRT_INTEGRATOR_AO, frt.FRT_INTEGRATOR_NORMALS):
        film, st = ctx.render(frt.RenderParams.make(nx, ny, 16, seed=6, integrator=integ))
        ref, cnt = osc.render(nx, ny, 16, seed=6, integrator=integ)
        assert st.camera_rays == cnt.camera_rays and abs(st.rays - cnt.rays) / cnt.rays < 2e-3
        assert rmse(film, ref) <= 1e-3, integ
    chains, mpp = 1536, 4
    film = np.zeros((ny, nx, 3), np.float32)
    film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, mpp, chains, seed=3, bootstrap=2000), film)
    ref, b, cnt = osc.mlt_render(nx, ny, chains, mpp * nx * ny // chains, seed=3, n_init=2000)
    assert abs(st.rays - cnt.rays) / cnt.rays < 2e-3
    assert rmse(film, ref) <= 1e-3 * max(1.0, float(np.abs(ref).max()))
