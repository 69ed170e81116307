#!/usr/bin/env python3
"""Probe: the conductor test scene (tests/scene_specs.py cornell_conductors,
beckmann sphere + ggx cube) rendered by every plan x register cap against
the oracle; prints RMSE and ray counts per (flags, FRT_MATS_WAVES)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402
import first_raytracer_amd as frt  # noqa: E402
import oracle  # noqa: E402
import scene_specs as SS  # noqa: E402

spec = SS.cornell_conductors("beckmann", "ggx", "bvh")
nx, ny, spp = 96, 72, 32
ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=11)
ctx = frt.Context(0)
ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
flag_sets = [int(x) for x in os.environ.get("PROBE_FLAGS", "1,17,0").split(",")]
caps = os.environ.get("PROBE_CAPS", "0,4,5,6").split(",")
for flags in flag_sets:
    for w in caps:
        if w == "-":
            os.environ.pop("FRT_MATS_WAVES", None)
        else:
            os.environ["FRT_MATS_WAVES"] = w
        film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=11, flags=flags))
        e = float(np.sqrt(np.mean((film.reshape(-1, 3).astype(np.float64) - ref) ** 2)))
        print("flags", flags, "waves", w, "cap", st.waves_cap, "lds", st.scene_in_lds, "rmse", e, "rays", st.rays,
              cnt.rays, flush=True)
