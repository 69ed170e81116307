#!/usr/bin/env python3
"""Ray-query throughput (frt_trace_device: batched Scene::world->hit) on the
bench scenes, for the kinds of rays a path tracer casts: camera rays,
incoherent diffuse bounce rays (cosine lobe about the hit normal) and NEE
shadow rays toward random points of the emitters (any hit).  The rays are
built on the GPU from a first camera pass; every batch is traced `--rounds`
times for each register cap in --waves (FRT_TRACE_WAVES), interleaved, in one
process.  Prints one JSON line per (ray kind, cap): median ms, Grays/s.

    python tools/trace_bench.py [--scene cornell_1m] [--rays-per-pixel 4]
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell_1m")
    ap.add_argument("--res", default="1920x1080")
    ap.add_argument("--rays-per-pixel", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--waves", default="6,8,10")
    ap.add_argument("--flags", type=int, default=0)
    args = ap.parse_args()
    import torch
    import first_raytracer_amd as frt
    from bench import scene_spec
    dev = torch.device("cuda", 0)
    nx, ny = (int(v) for v in args.res.split("x"))
    kind, obj, name = scene_spec(args.scene, "/tmp")
    ctx = frt.Context(0)
    if kind == "cornell_box_obj":      # the bench's tree: binned SAH built on the GPU
        hs = frt.HostScene.from_spec({"objects": [{"obj": obj, "geo": True}], "camera": frt.CORNELL_CAMERA,
                                      "world": "list"}, nx / ny)
        hs.build_bvh_gpu(ctx, "gsah")
    else:
        hs = frt.HostScene(kind, obj, nx / ny)
    ctx.upload(hs)
    v = hs.view()
    A = hs.arrays()
    tv = torch.tensor(A["tri_v"], dtype=torch.float64, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    k = args.rays_per_pixel
    n = nx * ny * k
    # camera rays (camera.h:30-35, pinhole), k jittered samples per pixel
    pix = torch.arange(nx * ny, device=dev).repeat(k)
    px = (pix % nx).double() + torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    py = (pix // nx).double() + torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    o = torch.tensor(v.cam_origin[:], dtype=torch.float64, device=dev)
    llc = torch.tensor(v.cam_lower_left[:], dtype=torch.float64, device=dev)
    H = torch.tensor(v.cam_horizontal[:], dtype=torch.float64, device=dev)
    V = torch.tensor(v.cam_vertical[:], dtype=torch.float64, device=dev)
    d = llc + (px / nx)[:, None] * H + (py / ny)[:, None] * V - o

    def pack(orig, dirs, tmax, anyhit):
        r = torch.empty((orig.shape[0], 8), dtype=torch.float32, device=dev)
        r[:, 0:3] = orig.float()
        r[:, 3] = tmax
        r[:, 4:7] = dirs.float()
        r[:, 7] = torch.tensor([1 if anyhit else 0], dtype=torch.int32, device=dev).view(torch.float32)
        return r

    cam = pack(o.expand(n, 3), d, 3.4e38, False)
    hits = torch.empty((n, 4), dtype=torch.float32, device=dev)
    ctx.trace_device(cam.data_ptr(), n, hits.data_ptr(), args.flags)
    prim = hits[:, 3].view(torch.int32).long()
    ok = (prim >= 0) & (prim < (1 << 30))
    t = hits[:, 0].double()
    p = o + t[:, None] * d
    tri = tv[prim.clamp(min=0)]
    e1, e2 = tri[:, 3:6] - tri[:, 0:3], tri[:, 6:9] - tri[:, 0:3]
    nrm = torch.nn.functional.normalize(torch.cross(e1, e2, dim=1), dim=1)
    nrm = torch.where(((nrm * d).sum(1) > 0)[:, None], -nrm, nrm)
    p, nrm = p[ok], nrm[ok]
    m = p.shape[0]
    # diffuse bounce: cosine lobe about the normal (pdf.h:13-23)
    r1 = torch.rand(m, generator=g, device=dev, dtype=torch.float64)
    r2 = torch.rand(m, generator=g, device=dev, dtype=torch.float64)
    a = torch.where((nrm[:, 0].abs() > 0.9)[:, None], torch.tensor([0.0, 1.0, 0.0], device=dev, dtype=torch.float64),
                    torch.tensor([1.0, 0.0, 0.0], device=dev, dtype=torch.float64))
    vv = torch.nn.functional.normalize(torch.cross(nrm, a, dim=1), dim=1)
    uu = torch.cross(vv, nrm, dim=1)
    phi = 2 * np.pi * r2
    bd = (r1.sqrt() * phi.cos())[:, None] * uu + (r1.sqrt() * phi.sin())[:, None] * vv + (1 - r1).sqrt()[:, None] * nrm
    po = p + 1e-4 * nrm
    bounce = pack(po, bd, 3.4e38, False)
    # NEE shadow rays to random points of random emitter triangles, t_max = 1 - SHADOW_EPSILON (path.cpp:50)
    lights = torch.tensor(A["lights"], dtype=torch.long, device=dev)
    lights = lights[lights < (1 << 30)]
    li = lights[torch.randint(0, lights.numel(), (m,), generator=g, device=dev)]
    lt = tv[li]
    su = torch.rand(m, generator=g, device=dev, dtype=torch.float64).sqrt()
    b1 = torch.rand(m, generator=g, device=dev, dtype=torch.float64) * su
    b0 = 1 - su
    lp = lt[:, 0:3] + b0[:, None] * (lt[:, 3:6] - lt[:, 0:3]) + b1[:, None] * (lt[:, 6:9] - lt[:, 0:3])
    shadow = pack(po, lp - po, 1.0 - 1e-3, True)
    batches = {"camera": (cam, n), "bounce": (bounce, m), "shadow": (shadow, m)}
    waves = [w for w in args.waves.split(",")]
    res = {(b, w): [] for b in batches for w in waves}
    out = torch.empty((max(n, m), 4), dtype=torch.float32, device=dev)
    for r in range(args.rounds + 1):
        for b, (rays, cnt) in batches.items():
            for w in waves:
                os.environ["FRT_TRACE_WAVES"] = w
                st = ctx.trace_device(rays.data_ptr(), cnt, out.data_ptr(), args.flags)
                if r > 0:
                    res[(b, w)].append(st.kernel_ms)
                if r == 0 and w == waves[0]:
                    hit_frac = float((out[:cnt, 3].view(torch.int32) >= 0).float().mean())
                    print(json.dumps({"batch": b, "rays": cnt, "hit_frac": round(hit_frac, 4)}), file=sys.stderr)
    for b, (rays, cnt) in batches.items():
        for w in waves:
            ms = statistics.median(res[(b, w)])
            print(json.dumps({"scene": args.scene, "batch": b, "waves": int(w), "rays": cnt, "median_ms": round(ms, 3),
                              "grays": round(cnt / ms / 1e6, 3)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
