#!/usr/bin/env python3
"""Throughput of the material kernels (MATS mask: textures, phong / metal /
dielectric, rough conductor) next to the lambertian-only kernel, on the
builder scenes of tests/scene_specs.py at 1080p.  One JSON line per scene:
rays / kernel time (HIP events inside libfrt.so), best of --rounds.

  python tools/perf_mats.py [--spp 64] [--rounds 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import first_raytracer_amd as frt  # noqa: E402
import scene_specs as SS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--flags", default="0", help="comma list of FRT_FLAG_* values to A/B (e.g. 0,8,4)")
    a = ap.parse_args()
    nx, ny = 1920, 1080
    scenes = {
        "cornell_lambertian": {"objects": [{"obj": SS.CORNELL_OBJ, "geo": True}], "camera": SS.CORNELL_CAM},
        "cornell_conductors": SS.cornell_conductors(),
        "cornell_textured": SS.cornell_textured(),
        # one material set each (the kernel the launcher picks: kMatsTex / kMatsSpec)
        "cornell_checker_floor": {"objects": SS.cornell_textured()["objects"][:2], "camera": SS.CORNELL_CAM},
        "cornell_mirror": {"objects": [{"obj": os.path.join(ROOT, "tests", "golden", "scenes", "CornellBox-Mirror.obj"),
                                        "geo": True}], "camera": SS.CORNELL_CAM},
    }
    ctx = frt.Context(0)
    for name, spec in scenes.items():
        hs = frt.HostScene.from_spec(spec, nx / ny)
        hs.build_bvh_sah()
        ctx.upload(hs)
        for flags in (int(f) for f in a.flags.split(",")):
            run(ctx, name, nx, ny, a, flags)
    ctx.close()


def run(ctx, name, nx, ny, a, flags):
    if True:
        p = frt.RenderParams.make(nx, ny, a.spp, seed=1, flags=flags)
        ctx.render(p)                                  # warm-up
        best = None
        for _ in range(a.rounds):
            _, st = ctx.render(p)
            rays = st.camera_rays + st.extension_rays + st.shadow_rays
            mrs = rays / (st.kernel_ms * 1e3)
            if best is None or mrs > best[0]:
                best = (mrs, st.kernel_ms, rays, st.waves_cap, st.scene_in_lds)
        print(json.dumps({"scene": name, "flags": flags, "spp": a.spp, "Mrays_s": round(best[0], 1), "kernel_ms": round(best[1], 3),
                          "rays": int(best[2]), "waves_cap": int(best[3]), "scene_in_lds": int(best[4])}), flush=True)


if __name__ == "__main__":
    main()
