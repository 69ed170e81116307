#!/usr/bin/env python3
"""Diagnostic: render one scene under every kernel variant (LDS/HBM, BVH2/BVH4,
register caps, shading thresholds) and compare each film with the oracle and
with the LDS/BVH2 film.  python tools/diag_variants.py [tess]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import first_raytracer_amd as frt  # noqa: E402
import oracle  # noqa: E402

tess = int(sys.argv[1]) if len(sys.argv) > 1 else 16
obj = os.path.join(ROOT, "tests/golden/scenes/CornellBox-Original.obj")
dst = "/tmp/diag_tess.obj"
frt.write_tessellated_obj(obj, tess, dst)
nx, ny, spp = 64, 48, 8
hs = frt.HostScene("cornell_box_obj", dst, nx / ny)
ref, _ = oracle.OracleScene("cornell_box_obj", dst, nx / ny).render(nx, ny, spp, seed=21)
ctx = frt.Context(0)
ctx.upload(hs)
F = frt
variants = {
    "lds": 0, "hbm4": F.FRT_FLAG_NO_LDS_SCENE, "hbm2": F.FRT_FLAG_NO_LDS_SCENE | F.FRT_FLAG_BVH2,
    "hbm4_w4": F.FRT_FLAG_NO_LDS_SCENE | F.FRT_FLAG_WAVES4,
    "hbm2_w4": F.FRT_FLAG_NO_LDS_SCENE | F.FRT_FLAG_BVH2 | F.FRT_FLAG_WAVES4,
    "lds_w4": F.FRT_FLAG_WAVES4,
}
base = None
for tm in ("0", "16"):
    os.environ["FRT_TRAV_MIN"] = tm
    for name, fl in variants.items():
        f, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=21, flags=fl))
        if base is None:
            base = f
        e = float(np.sqrt(np.mean((f.astype(np.float64).reshape(-1, 3) - ref.reshape(-1, 3)) ** 2)))
        nd = int((np.abs(f - base).reshape(-1, 3).max(1) > 0).sum())
        print(f"trav{tm:>2} {name:8s} rmse_vs_oracle={e:.3e} pixels_differing_from_lds={nd:5d} rays={st.rays} "
              f"plan=(lds={st.scene_in_lds} w={st.waves_cap} stack={st.stack_entries} depth={st.bvh_depth})",
              flush=True)
ctx.close()
