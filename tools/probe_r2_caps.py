#!/usr/bin/env python3
"""Round-2 register-cap hazard, reproduced on a round-2 source state with its
6-wave specular kernels enabled (built out of tree into
first_raytracer_amd/build/r2/first_raytracer_amd/, with that round's ctypes
binding).  The conductor scene (tests/scene_specs.py cornell_conductors) on
the HBM binary plan (flags 17) and the HBM 4-wide plan (flags 1) at caps 5
and 6 against the oracle; then, for the first diverging pixel, which samples
of it differ between the two caps (spp 1 renders with sample_offset).

    PYTHONPATH=first_raytracer_amd/build/r2 python tools/probe_r2_caps.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.append(ROOT)
sys.path.append(os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402
import first_raytracer_amd as frt  # noqa: E402
import oracle  # noqa: E402
import scene_specs as SS  # noqa: E402

print("binding", frt.__file__, flush=True)
spec = SS.cornell_conductors("beckmann", "ggx", "bvh")
nx, ny, spp = 96, 72, 32
ref, cnt = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=11)
ctx = frt.Context(0)
ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
films = {}
for flags in (17, 1, 0):
    for w in ("5", "6"):
        os.environ["FRT_MATS_WAVES"] = w
        film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=11, flags=flags))
        e = float(np.sqrt(np.mean((film.reshape(-1, 3).astype(np.float64) - ref) ** 2)))
        films[(flags, w)] = film.copy()
        print("flags", flags, "waves", w, "cap", st.waves_cap, "rmse", e, "rays", st.rays, cnt.rays, flush=True)
for flags in (17, 1):
    a, b = films[(flags, "5")].reshape(-1, 3), films[(flags, "6")].reshape(-1, 3)
    d = np.abs(a.astype(np.float64) - b).max(axis=1)
    bad = np.nonzero(d > 1e-6)[0]
    print("flags", flags, "pixels differing between caps 5 and 6:", len(bad), "nan:", int(np.isnan(b).any(axis=1).sum()),
          flush=True)
    if len(bad) == 0:
        continue
    worst = bad[np.argsort(-d[bad])[:3]]
    for pix in worst:
        px, py = int(pix % nx), int(pix // nx)
        print(f"  pixel ({px},{py}) cap5 {a[pix]} cap6 {b[pix]} oracle {ref[pix]}", flush=True)
    pix = int(worst[0])
    diffs = []
    for s in range(spp):
        out = {}
        for w in ("5", "6"):
            os.environ["FRT_MATS_WAVES"] = w
            f, _ = ctx.render(frt.RenderParams.make(nx, ny, 1, seed=11, flags=flags, sample_offset=s))
            out[w] = f.reshape(-1, 3)[pix].astype(np.float64)
        if np.abs(out["5"] - out["6"]).max() > 1e-6:
            diffs.append((s, out["5"].tolist(), out["6"].tolist()))
    print("  samples that differ (sample, cap5, cap6):", diffs[:8], flush=True)
ctx.close()
