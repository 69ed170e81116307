"""GPU: ray queries (frt_trace_device, batched Scene::world->hit) against the
oracle's world_hit (parallel_bvh_node::hit parallel_bvh.h:39-64,
hitable_list::hit hitable_list.cpp:4-21) on the same rays.  fp32 vs fp64: the
hit primitive agrees except where rounding decides a silhouette or an edge
(bounded here at 0.2 % of the rays), t to fp32 rounding."""
import numpy as np
import pytest
import torch

import first_raytracer_amd as frt
import oracle

pytestmark = pytest.mark.gpu


def random_rays(n, rng, lo, hi, shadow=False):
    o = rng.uniform(lo, hi, (n, 3))
    if shadow:                                   # segment to another point, t_max = 1 - SHADOW_EPSILON
        d = rng.uniform(lo, hi, (n, 3)) - o
        tmax = np.full(n, 1.0 - 1e-3)
    else:
        d = rng.normal(size=(n, 3))
        tmax = np.full(n, 3.4e38)
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3] = o
    r[:, 3] = tmax
    r[:, 4:7] = d
    r[:, 7] = np.array([1 if shadow else 0], np.int32).view(np.float32)[0]
    return r


def trace(ctx, rays, flags=0):
    dev = torch.device("cuda", 0)
    tr = torch.tensor(rays, device=dev)
    th = torch.empty((rays.shape[0], 4), dtype=torch.float32, device=dev)
    st = ctx.trace_device(tr.data_ptr(), rays.shape[0], th.data_ptr(), flags)
    h = th.cpu().numpy()
    return h, h[:, 3].copy().view(np.int32), st


@pytest.mark.parametrize("kind,objfix,lo,hi,flags", [
    ("cornell_box_obj", "cornell_obj", (-1.0, 0.0, -1.0), (1.0, 2.0, 1.0), 0),                           # LDS plan
    ("cornell_box_obj", "cornell_obj", (-1.0, 0.0, -1.0), (1.0, 2.0, 1.0), frt.FRT_FLAG_NO_LDS_SCENE),   # HBM BVH4Q
    ("cornell_box_obj", "cornell_obj", (-1.0, 0.0, -1.0), (1.0, 2.0, 1.0),
     frt.FRT_FLAG_NO_LDS_SCENE | frt.FRT_FLAG_BVH2),                                                     # HBM binary
    ("veach_mis", "veach_obj", (-6.0, -3.0, -6.0), (6.0, 5.0, 6.0), 0)])                                # list world
@pytest.mark.parametrize("shadow", [False, True])
def test_trace_vs_oracle(kind, objfix, lo, hi, flags, shadow, request):
    obj = request.getfixturevalue(objfix)
    n = 4000
    rays = random_rays(n, np.random.default_rng(7 + shadow), lo, hi, shadow)
    ctx = frt.Context(0)
    try:
        ctx.upload(frt.HostScene(kind, obj, 1.0))
        h, prim, st = trace(ctx, rays, flags)
    finally:
        ctx.close()
    osc = oracle.OracleScene(kind, obj, 1.0)
    agree = hits = 0
    for i in range(n):
        r = rays[i].astype(np.float64)
        ok, t, p, _ = osc.world_hit(r[0:3], r[4:7], 1e-4, float(r[3]))
        if not shadow:
            if ok == (prim[i] >= 0) and (not ok or p == prim[i]):
                agree += 1
                if ok:
                    hits += 1
                    assert abs(h[i, 0] - t) <= 1e-5 * max(1.0, t), (i, h[i], t)
        else:                                    # any-hit: only occlusion is defined
            agree += ok == (prim[i] >= 0)
            hits += ok
    print(kind, flags, "shadow" if shadow else "closest", "agree", agree, "of", n, "hits", hits, "kernel ms", st.kernel_ms)
    assert agree >= 0.998 * n
    assert hits > 0.1 * n


def test_trace_empty_and_miss(cornell_obj):
    """n = 0 is a no-op; rays pointing away from the scene miss with t = t_max."""
    ctx = frt.Context(0)
    try:
        ctx.upload(frt.HostScene("cornell_box_obj", cornell_obj, 1.0))
        _, _, st = trace(ctx, np.zeros((0, 8), np.float32))
        rays = random_rays(64, np.random.default_rng(1), (10.0, 10.0, 10.0), (11.0, 11.0, 11.0))
        rays[:, 4:7] = (1.0, 1.0, 1.0)
        h, prim, _ = trace(ctx, rays)
        assert (prim == -1).all()
        assert np.array_equal(h[:, 0], rays[:, 3])
    finally:
        ctx.close()
