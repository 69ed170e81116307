#!/usr/bin/env python3
"""Per-phase lane occupancy of path_megakernel from the diagnostic build
(make -C first_raytracer_amd exp NAME=diag DEFS=-DFRT_DIAG):

  FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_diag.so python tools/diag_phases.py [--scene cornell_1m] [--spp 32]

Counter pairs (wave trips, active lanes summed over trips): 0 BVH4Q node
iterations, 1 leaf primitive tests, 2 binary node iterations, 3 step-loop
iterations (tracing lanes), 4 shading passes (lanes shading), 6 outer-loop
iterations, 5 PSS-MLT accept / reject lanes, 7 octant-plan stack entries skipped by pop culling (entry
distance beyond the closest hit: each was a node visit or a leaf test before
round 5); cycles (s_memtime, per wave, summed): 16 step loop, 17 shading,
18 refill + ray setup (PSS-MLT: queue + next proposal; 19 accept / reject +
splats, 20 accepted-row materialisation).  Timing under instrumentation is perturbed; the lane
counts are exact.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--res", default="1920x1080")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--integrator", default="path", choices=["path", "pssmlt"],
                    help="pssmlt: --spp = mutations per pixel over --chains chains")
    ap.add_argument("--chains", type=int, default=1 << 18)
    args = ap.parse_args()
    import torch  # noqa: F401
    import first_raytracer_amd as frt
    from bench import scene_spec
    nx, ny = (int(v) for v in args.res.split("x"))
    kind, obj, name = scene_spec(args.scene, "/tmp")
    if kind == "cornell_box_obj":
        hs = frt.HostScene.from_spec({"objects": [{"obj": obj, "geo": True}], "camera": frt.CORNELL_CAMERA,
                                      "world": "list"}, nx / ny)
        hs.build_bvh_sah()
    else:
        hs = frt.HostScene(kind, obj, nx / ny)
    ctx = frt.Context(0)
    ctx.upload(hs)
    if args.integrator == "pssmlt":
        p = frt.RenderParams.pssmlt(nx, ny, args.spp, args.chains, seed=0)
        p.flags = args.flags
    else:
        p = frt.RenderParams.make(nx, ny, args.spp, seed=0, flags=args.flags)
    ctx.render(p)
    film, st = ctx.render(p)
    buf = (ctypes.c_ulonglong * 24)()
    frt.lib().frt_diag_read(buf)
    v = list(buf)
    names = {0: "bvh4_node", 1: "leaf_prim", 2: "bvh2_node", 3: "step", 4: "shade", 5: "accept", 6: "outer",
             7: "culled_pop"}
    out = {"scene": args.scene, "spp": args.spp, "rays": st.rays, "kernel_ms": st.kernel_ms,
           "waves_cap": st.waves_cap, "stack": st.stack_entries}
    for k, n in names.items():
        trips, lanes = v[2 * k], v[2 * k + 1]
        out[n] = {"trips": trips, "lanes": lanes, "util": lanes / (64.0 * trips) if trips else None,
                  "per_ray": lanes / st.rays}
    cyc = {"step": v[16], "shade": v[17], "refill": v[18]}
    if args.integrator == "pssmlt":   # PSS-MLT: 18 = queue + next proposal; 19 accept / splats; 20 rows
        cyc.update({"accept_splat": v[19], "materialise": v[20]})
    out["integrator"] = args.integrator
    tot = sum(cyc.values())
    out["cycles_share"] = {k: c / tot for k, c in cyc.items()} if tot else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
