#!/usr/bin/env python3
"""Register-cap table: the conductor scene of tests/test_gpu_conductors.py
(test_register_caps_agree) rendered under every FRT_MATS_WAVES cap and plan,
against the oracle, without stopping at the first bad film.  The library is
the one FRT_LIB_PATH names (default: the in-tree libfrt.so), so builds that
differ only in compiler options can be compared in one call.  One JSON line
per (plan, cap): rmse vs the oracle, pixels differing from the plan's
uncapped film, the mean signed error, ray counts.

    FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_x.so python tools/caps_table.py --tag x
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--flags", default="0,16,17")
    ap.add_argument("--caps", default="0,3,4,5,6")
    ap.add_argument("--res", default="64x48")
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--seed", type=int, default=12)
    ap.add_argument("--scene", default="conductors", choices=["conductors", "lambert"],
                    help="lambert: tessellated Cornell (lambertian kernels; caps by FRT_FLAG_WAVES*)")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import first_raytracer_amd as frt
    import oracle
    import scene_specs as SS
    nx, ny = (int(v) for v in a.res.split("x"))
    ctx = frt.Context(0)
    if a.scene == "conductors":
        spec = SS.cornell_conductors("beckmann", "ggx", "bvh")
        ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, a.spp, seed=a.seed)
        ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
        cap_flags = {w: 0 for w in a.caps.split(",")}
    else:                       # the lambertian kernels' caps come from flags: compiler's own, 5, 6
        obj = os.path.join(ROOT, "tests", "golden", "scenes", "CornellBox-Original.obj")
        tess = os.path.join("/tmp", "caps_tess.obj")
        frt.write_tessellated_obj(obj, 16, tess)
        ref, cnt = oracle.OracleScene("cornell_box_obj", tess, nx / ny).render(nx, ny, a.spp, seed=a.seed)
        ctx.upload(frt.HostScene("cornell_box_obj", tess, nx / ny))
        cap_flags = {"4": frt.FRT_FLAG_WAVES4, "5": frt.FRT_FLAG_WAVES5, "6": frt.FRT_FLAG_WAVES6}
    ref = np.asarray(ref, np.float64).reshape(-1, 3)
    for flags in (int(f) for f in a.flags.split(",")):
        base = None
        for w, cf in cap_flags.items():
            os.environ["FRT_MATS_WAVES"] = w
            film, st = ctx.render(frt.RenderParams.make(nx, ny, a.spp, seed=a.seed, flags=flags | cf))
            f = np.asarray(film, np.float64).reshape(-1, 3)
            if base is None:
                base = f
            d = f - ref
            print(json.dumps({"tag": a.tag, "lib": os.environ.get("FRT_LIB_PATH", "libfrt.so"), "flags": flags,
                              "cap": int(st.waves_cap), "rmse": float(np.sqrt(np.mean(d ** 2))),
                              "mean_err": float(d.mean()),
                              "px_diff_vs_first_cap": int((np.abs(f - base).max(axis=1) > 1e-6).sum()),
                              "rays": int(st.rays), "oracle_rays": int(cnt.rays)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
