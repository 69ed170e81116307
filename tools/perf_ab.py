#!/usr/bin/env python3
"""A/B timing of kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Prints per-variant median/min
kernel ms and Grays/s as JSON lines.

  python tools/perf_ab.py [--scene cornell|cornell_1m|veach] [--spp 64] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--res", default="1920x1080")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="default,no_lds")
    args = ap.parse_args()
    import torch  # noqa: F401  (single HIP runtime)
    import first_raytracer_amd as frt
    sys.path.insert(0, ROOT)
    from bench import scene_spec
    nx, ny = (int(v) for v in args.res.split("x"))
    kind, obj, name = scene_spec(args.scene, "/tmp")
    ctx = frt.Context(0)
    ctx.upload(frt.HostScene(kind, obj, nx / ny))
    variants = {"default": 0, "no_lds": frt.FRT_FLAG_NO_LDS_SCENE, "waves5": frt.FRT_FLAG_WAVES5}
    chosen = [v for v in args.variants.split(",") if v in variants]
    res = {v: [] for v in chosen}
    rays = {}
    film = None
    for r in range(args.rounds + 1):
        for v in chosen:
            film, st = ctx.render(frt.RenderParams.make(nx, ny, args.spp, seed=0, flags=variants[v]), film)
            if r > 0:
                res[v].append(st.kernel_ms)
            rays[v] = st.rays
    for v in chosen:
        ms = res[v]
        print(json.dumps({"scene": args.scene, "variant": v, "spp": args.spp, "median_ms": statistics.median(ms),
                          "min_ms": min(ms), "grays_per_s": rays[v] / (statistics.median(ms) * 1e-3) / 1e9,
                          "rays": rays[v]}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
