"""The fp64 list kernels' fp32 filter (frt_path.hpp trace_list_filtered): the
query with the filter must give the plain fp64 loop's answer (hitable_list::hit,
hitable_list.cpp:4-21 -- primitive, t, u, v bit for bit for closest hits;
occluded or not for any-hit queries) on every ray.  The rays are built to sit
on the filter's boundaries: aimed at triangle edges and vertices within
1e-16..1e-5 of them, tangent to the sphere lights within 1e-16..1e-5 of the
silhouette, shadow rays ending on the light surfaces, plus random rays.  Runs
the device code on the host (frt_internal_list_filter_check).  CPU only."""
import ctypes

import numpy as np
import pytest

import first_raytracer_amd as frt


def check(sv, rays):
    L = frt.lib()
    f = L.frt_internal_list_filter_check
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    rays = np.ascontiguousarray(rays, np.float64)
    out = np.zeros(len(rays), np.int32)
    rc = f(ctypes.byref(sv), rays.ctypes.data, len(rays), out.ctypes.data)
    assert rc == 0
    return out


def scene_prims(sv, a):
    tris = a["tri_v"].reshape(-1, 3, 3)
    sph = np.ctypeslib.as_array(ctypes.cast(sv.sphere, ctypes.POINTER(ctypes.c_double)),
                                shape=(sv.n_spheres * 4,)).reshape(-1, 4).copy()
    return tris, sph


def make_rays(o, target, tmax, anyhit):
    d = target - o
    n = len(o)
    r = np.zeros((n, 8))
    r[:, 0:3] = o
    r[:, 3] = tmax
    r[:, 4:7] = d
    r[:, 7] = anyhit
    return r


@pytest.mark.parametrize("anyhit", [0, 1])
def test_filter_matches_fp64_list(veach_obj, anyhit):
    rng = np.random.default_rng(7 + anyhit)
    hs = frt.HostScene("veach_mis", veach_obj, 1920 / 1080)
    sv = hs.view()
    tris, sph = scene_prims(sv, hs.arrays())
    lo = np.minimum(tris.min(axis=(0, 1)), (sph[:, :3] - sph[:, 3:]).min(0)) - 2.0
    hi = np.maximum(tris.max(axis=(0, 1)), (sph[:, :3] + sph[:, 3:]).max(0)) + 2.0
    n = 40000
    tmax_any = 1.0 - float(np.float32(1e-3))              # shadow rays: 1 - SHADOW_EPSILON (path.cpp:71)
    tmax = tmax_any if anyhit else float(np.finfo(np.float32).max)
    batches = []
    # 1) rays through points on triangle edges / vertices, nudged by 1e-16 .. 1e-5
    k = rng.integers(0, len(tris), n)
    w = rng.random((n, 3))
    side = rng.integers(0, 4, n)                          # 0,1,2: an edge (one barycentric 0), 3: a vertex
    w[np.arange(n), np.minimum(side, 2)] = 0.0
    w[side == 3] = np.eye(3)[rng.integers(0, 3, (side == 3).sum())]
    w /= w.sum(1, keepdims=True)
    p = np.einsum("ni,nij->nj", w, tris[k])
    eps = 10.0 ** rng.uniform(-16, -5, (n, 1)) * rng.choice([-1, 1], (n, 3))
    o = lo + rng.random((n, 3)) * (hi - lo)
    tgt = p + eps * (1.0 + np.abs(p))
    if anyhit:                                            # shadow-like: end past the surface or just before it
        tgt = o + (tgt - o) * rng.choice([0.999, 1.0005, 1.5], (n, 1))
    batches.append(make_rays(o, tgt, tmax, anyhit))
    # 2) rays tangent to the spheres (the light silhouettes), offsets 1e-16 .. 1e-5 of r
    j = rng.integers(0, len(sph), n)
    c, r = sph[j, :3], sph[j, 3:]
    o = lo + rng.random((n, 3)) * (hi - lo)
    oc = c - o
    dist = np.linalg.norm(oc, axis=1, keepdims=True)
    u = oc / dist
    perp = rng.normal(size=(n, 3))
    perp -= (perp * u).sum(1, keepdims=True) * u
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    off = r * (1.0 + 10.0 ** rng.uniform(-16, -5, (n, 1)) * rng.choice([-1, 1], (n, 1)))
    tgt = c + perp * off
    batches.append(make_rays(o, tgt, tmax, anyhit))
    # 3) shadow-style rays onto sampled light-surface points, and random rays
    surf = rng.normal(size=(n, 3))
    surf /= np.linalg.norm(surf, axis=1, keepdims=True)
    tgt = c + r * surf
    batches.append(make_rays(lo + rng.random((n, 3)) * (hi - lo), tgt, tmax, anyhit))
    o = lo + rng.random((n, 3)) * (hi - lo)
    batches.append(make_rays(o, o + rng.normal(size=(n, 3)), tmax, anyhit))
    rays = np.concatenate(batches)
    bad = check(sv, rays)
    assert bad.sum() == 0, np.nonzero(bad)[0][:10]
