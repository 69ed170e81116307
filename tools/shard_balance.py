#!/usr/bin/env python3
"""Load balance of the N-way tile split, measured on one GPU.

bench.py shards the frame by tiles (tile t -> rank t mod N)
and each rank renders its shard with no data-path collective, then the slot
buffers are gathered to rank 0.  Strong scaling over N GPUs is bounded by the
slowest shard: this renders every shard (r, N) alone on the one GPU of the box,
at the bench config, and reports per N

    max_ms / mean_ms          shard imbalance
    full_ms / (N * max_ms)    predicted strong-scaling efficiency of the render
                              (1.0 = the slowest shard takes exactly 1/N)

plus the gather's bytes per rank.  It is not a scaling curve (the driver's
SCALE run is): a shard alone on a whole GPU has the whole chip to itself, as it
would on its own GPU.  Films of the shards are also checked against the full
frame (bit-identical slots: the RNG is keyed by the global pixel).

    python tools/shard_balance.py --scene cornell --ns 2,4,8 --reps 2
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell", choices=["cornell", "cornell_1m"])
    ap.add_argument("--res", default="1920x1080")
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--ns", default="2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--tile", type=int, default=32)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import bench
    import first_raytracer_amd as frt
    nx, ny = (int(v) for v in a.res.split("x"))
    workdir = tempfile.gettempdir()   # the generated 1M-triangle OBJ (33 MB) stays out of gpurun_out/
    kind, obj, name = bench.scene_spec(a.scene, workdir)
    hs = frt.HostScene.from_spec({"objects": [{"obj": obj, "geo": True}], "camera": frt.CORNELL_CAMERA,
                                  "world": "list"}, nx / ny)
    ctx = frt.Context(0)
    hs.build_bvh_gpu(ctx, "gsah")                    # the bench's tree (binned SAH on the GPU)
    ctx.upload(hs)

    def render(index, count):
        p = frt.RenderParams.make(nx, ny, a.spp, seed=0, tile_size=a.tile, shard_index=index, shard_count=count)
        film = np.zeros((ny, nx, 3), np.float32)
        best = None
        for _ in range(a.reps):
            f, st = ctx.render(p, np.zeros((ny, nx, 3), np.float32))
            best = st if best is None or st.kernel_ms < best.kernel_ms else best
            film = f
        return film, best

    render(0, 1)                                     # warm-up
    full, stf = render(0, 1)
    out = {"scene": name, "res": a.res, "spp": a.spp, "tile": a.tile, "full_ms": round(stf.kernel_ms, 2),
           "full_rays": int(stf.rays), "per_n": []}
    print(json.dumps({"full_ms": stf.kernel_ms, "rays": stf.rays}), file=sys.stderr, flush=True)
    for n in (int(v) for v in a.ns.split(",")):
        ms, rays, films = [], [], np.zeros_like(full)
        for r in range(n):
            f, st = render(r, n)
            ms.append(st.kernel_ms)
            rays.append(int(st.rays))
            films += f
            print(json.dumps({"n": n, "r": r, "ms": st.kernel_ms}), file=sys.stderr, flush=True)
        slots = frt.shard_slots(frt.RenderParams.make(nx, ny, a.spp, tile_size=a.tile, shard_index=0, shard_count=n))
        mx, mean = max(ms), float(np.mean(ms))
        out["per_n"].append({
            "n": n, "shard_ms": [round(x, 2) for x in ms], "max_ms": round(mx, 2), "mean_ms": round(mean, 2),
            "imbalance_max_over_mean": round(mx / mean, 4),
            "predicted_render_efficiency": round(stf.kernel_ms / (n * mx), 4),
            "predicted_speedup": round(stf.kernel_ms / mx, 3),
            "rays_sum_over_full": round(sum(rays) / stf.rays, 6),
            "films_identical": bool(np.array_equal(films, full)),
            "gather_bytes_per_rank": int(len(slots) * 12)})
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
