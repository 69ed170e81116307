#!/usr/bin/env python3
"""Register-cap hazard: the films of one library (FRT_LIB_PATH) on the conductor
scene of tools/caps_table.py, saved for offline comparison -- every (cap,
max_depth) of one plan, plus a normals render for the primary hits.  The bounce
at which capped and uncapped films first differ, and how the wrong pixels
differ (per channel, by ratio), say which shading quantity is wrong.

    FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_fail.so python tools/caps_films.py --out films.npz
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--flags", type=int, default=17)
    ap.add_argument("--caps", default="0,4,5,6")
    ap.add_argument("--depths", default="1,2,3,4,6,33")
    ap.add_argument("--res", default="64x48")
    ap.add_argument("--spp", default="1,16")
    ap.add_argument("--seed", type=int, default=12)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import first_raytracer_amd as frt
    import scene_specs as SS
    nx, ny = (int(v) for v in a.res.split("x"))
    spec = SS.cornell_conductors("beckmann", "ggx", "bvh")
    ctx = frt.Context(0)
    ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
    out = {}
    for spp in (int(s) for s in a.spp.split(",")):
        for d in (int(v) for v in a.depths.split(",")):
            for w in a.caps.split(","):
                os.environ["FRT_MATS_WAVES"] = w
                film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=a.seed, max_depth=d, flags=a.flags))
                out[f"s{spp}_d{d}_w{w}"] = np.asarray(film, np.float32).reshape(ny, nx, 3)
                print(spp, d, w, int(st.waves_cap), int(st.rays), flush=True)
        os.environ["FRT_MATS_WAVES"] = "0"
        film, _ = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=a.seed, flags=a.flags,
                                                   integrator=frt.FRT_INTEGRATOR_NORMALS))
        out[f"s{spp}_normals"] = np.asarray(film, np.float32).reshape(ny, nx, 3)
    ctx.close()
    np.savez_compressed(a.out, **out)


if __name__ == "__main__":
    main()
