#!/usr/bin/env python3
"""C3 probe: veach_mis (main.cpp:281-314) as a list world (the reference's,
hitable_list) against the same primitives under a BVH (the reference's
commented-out alternatives, main.cpp:311-312), both rendered by the fp64
kernels.  Reports kernel ms per variant and the films' RMSE against each
other: a BVH answers the list's closest hit except at exact-t ties between
primitives, so the films should agree to the noise-free level.

    python tools/veach_bvh_probe.py --spp 256 --rounds 2
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def f32(x):
    return float(np.float32(x))


def veach_spec(obj, world):
    def light(c, r, e):
        return {"sphere": c, "radius": r, "material": {"type": "diffuse_light", "emit": (e, e, e)},
                "where": "both"}
    return {"objects": [{"obj": obj},
                        light((10, 10, 4), 0.5, 800.0),
                        light((f32(-1.25), 0, 0), f32(0.1), 100.0),
                        light((f32(-3.75), 0, 0), f32(0.03333), f32(901.803)),
                        light((f32(1.25), 0, 0), f32(0.3), f32(11.1111)),
                        light((f32(3.75), 0, 0), f32(0.9), 1.23457)],
            "camera": {"lookfrom": (0, 2, 15), "lookat": (0, -2, 2.5), "vup": (0, 1, 0), "vfov": 28.0,
                       "aperture": 0.0, "focus": 50.0},
            "world": world}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--res", default="1920x1080")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch  # noqa: F401
    import first_raytracer_amd as frt
    import bench
    nx, ny = (int(v) for v in a.res.split("x"))
    kind, obj, _ = bench.scene_spec("veach", "/tmp")
    scenes = {"ref_list": frt.HostScene(kind, obj, nx / ny),
              "spec_list": frt.HostScene.from_spec(veach_spec(obj, "list"), nx / ny),
              "spec_bvh": frt.HostScene.from_spec(veach_spec(obj, "bvh"), nx / ny),
              "ref_sah": frt.HostScene(kind, obj, nx / ny)}
    scenes["ref_sah"].build_bvh_sah()
    ctxs = {}
    for k, hs in scenes.items():
        c = frt.Context(0)
        c.set_precision("fp64")
        c.upload(hs)
        ctxs[k] = c
    res = {k: [] for k in scenes}
    films, rays = {}, {}
    for r in range(a.rounds + 1):
        for k, c in ctxs.items():
            p = frt.RenderParams.make(nx, ny, a.spp, seed=0)
            f, st = c.render(p, np.zeros((ny, nx, 3), np.float32))
            if r > 0:
                res[k].append(st.kernel_ms)
            films[k], rays[k] = np.asarray(f), st.rays
            print(json.dumps({"k": k, "ms": st.kernel_ms, "fp64": st.fp64, "lds": st.scene_in_lds,
                              "depth": st.bvh_depth}), file=sys.stderr, flush=True)
    base = films["ref_list"]
    for k in scenes:
        d = films[k] - base
        print(json.dumps({"variant": k, "median_ms": statistics.median(res[k]), "rays": int(rays[k]),
                          "grays_per_s": rays[k] / statistics.median(res[k]) / 1e6,
                          "rmse_vs_ref_list": float(np.sqrt(np.mean(d * d))),
                          "max_abs_vs_ref_list": float(np.abs(d).max()),
                          "pixels_differing": int((np.abs(d).max(axis=2) > 0).sum())}), flush=True)
    for c in ctxs.values():
        c.close()


if __name__ == "__main__":
    main()
