#!/usr/bin/env python3
"""A/B of the list-world (veach_mis, C3) kernel variants in ONE process,
interleaved rounds: precision (fp64 / fp32).  Prints one JSON line per
variant: median kernel ms, Grays/s.  (Round 3 also timed a per-prim box test
and a 2-wave fp64 register cap here, both since removed:
profiles/r03/r03c_ab_veach_listbox_f64waves.jsonl.)

  python tools/ab_veach.py [--spp 256] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {"fp64": "fp64", "fp32": "fp32"}   # name: frt_set_precision


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    args = ap.parse_args()
    import torch  # noqa: F401  (single HIP runtime)
    import first_raytracer_amd as frt
    obj = os.path.join(ROOT, "tests", "golden", "scenes", "veach_mi.obj")
    nx, ny = 1920, 1080
    hs = frt.HostScene("veach_mis", obj, nx / ny)
    names = args.variants.split(",")
    ctxs, res = {}, {v: [] for v in names}
    for v in names:
        c = frt.Context(0, precision=VARIANTS[v])
        c.upload(hs)
        ctxs[v] = c
    film = np.zeros((ny, nx, 3), np.float32)
    ref = None
    for r in range(args.rounds + 1):
        for v in names:
            f, st = ctxs[v].render(frt.RenderParams.make(nx, ny, args.spp, seed=1), film)
            if r > 0:
                res[v].append((st.kernel_ms, st.rays, st.fp64))
            if ref is None:
                ref = f.copy()
    for v in names:
        ms = statistics.median(x[0] for x in res[v])
        print(json.dumps({"variant": v, "median_ms": round(ms, 2), "grays": round(res[v][0][1] / ms / 1e6, 3),
                          "fp64": res[v][0][2], "spp": args.spp}), flush=True)


if __name__ == "__main__":
    import numpy as np
    main()
