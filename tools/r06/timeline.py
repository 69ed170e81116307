#!/usr/bin/env python3
"""(Record of round 6, stage x; the FRT_EXP_TIMELINE knob was removed after it.)
Per-wave timeline of path_megakernel (experiment build with FRT_EXP_TIMELINE=1,
loaded with FRT_LIB_PATH): its frt_stats ray fields carry sums over waves of
(entry -> first exhausted grab in shader-clock ticks, the same in 100-MHz
ticks, first exhausted grab -> exit, entry -> exit): the mean clock of the main
phase and per-wave mean durations.  Prints the per-wave means in ms beside the
launch's event time, for a few configurations."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    import first_raytracer_amd as frt
    from bench import scene_spec
    nx, ny = 1920, 1080
    for scene, spps in (("cornell", (16, 64, 512)), ("cornell_1m", (64, 512))):
        kind, obj, name = scene_spec(scene, "/tmp")
        hs = frt.HostScene.from_spec({"objects": [{"obj": obj, "geo": True}], "camera": frt.CORNELL_CAMERA,
                                      "world": "list"}, nx / ny)
        ctx = frt.Context(0)
        hs.build_bvh_gpu(ctx, "gsah")
        ctx.upload(hs)
        for spp in spps:
            for rep in range(3):
                film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=0))
            nw = 256 * 4 * st.waves_cap          # 256 CUs, one wave per SIMD per 256-thread block
            ms = lambda v: round(v / nw * 1e-5, 3)    # per-wave mean, 100-MHz ticks -> ms
            out = {"scene": scene, "spp": spp, "kernel_ms": round(st.kernel_ms, 3), "waves": nw,
                   "main_phase_clock_ghz": round(st.camera_rays / st.extension_rays * 0.1, 4),
                   "mean_to_exhausted_ms": ms(st.extension_rays),
                   "mean_drain_ms": ms(st.shadow_rays), "mean_total_ms": ms(st.samples)}
            print(json.dumps(out), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
