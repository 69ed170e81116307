#!/usr/bin/env python3
"""A/B timing of kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Prints per-variant median/min
kernel ms and Grays/s as JSON lines.

  python tools/perf_ab.py [--scene cornell|cornell_1m|veach] [--spp 64] [--rounds 5]
                          [--variants default,waves5,default/leaf1]

A variant is FLAG[+FLAG...][/leafN][/travN][/descN][/grabN][/sptN][/spiN]: render flags (travN sets
FRT_TRAV_MIN=N, descN FRT_MIN_DESC=N for its renders), on a scene uploaded with
FRT_LEAF_SIZE=N (one context per leaf size; default = the library default).
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("FRT_PKG_ROOT"):   # another revision's package (its binding + libfrt.so), same-call A/B
    sys.path.insert(0, os.environ["FRT_PKG_ROOT"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--res", default="1920x1080")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="default,no_lds")
    ap.add_argument("--bvh", default="sah", choices=["host", "sah", "ploc", "lbvh", "gsah"],
                    help="sah: binned SAH tree (bench default); host: the reference topology; "
                         "ploc / lbvh: the GPU builders")
    ap.add_argument("--integrator", default="path", choices=["path", "ao", "normals", "pssmlt"],
                    help="pssmlt: --spp = mutations per pixel, --chains chains")
    ap.add_argument("--chains", type=int, default=1 << 18)
    ap.add_argument("--save-films", default="", help="npz of each variant's last film (cross-library checks)")
    ap.add_argument("--env", default="", help="constant environment r,g,b (AO: 1,1,1 unless given)")
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (single HIP runtime)
    import first_raytracer_amd as frt
    sys.path.insert(0, ROOT)
    from bench import scene_spec
    nx, ny = (int(v) for v in args.res.split("x"))
    kind, obj, name = scene_spec(args.scene, "/tmp")
    names = {"default": 0, "no_lds": frt.FRT_FLAG_NO_LDS_SCENE, "waves4": frt.FRT_FLAG_WAVES4,
             "waves5": frt.FRT_FLAG_WAVES5, "waves6": frt.FRT_FLAG_WAVES6, "bvh2": frt.FRT_FLAG_BVH2,
             "no_oct": frt.FRT_FLAG_NO_OCT, "fp32": frt.FRT_FLAG_FP32}
    flags = {}
    for v in args.variants.split(","):
        parts = v.split("/")[0].split("+")
        if all(p in names for p in parts):
            flags[v.split("/")[0]] = sum(names[p] for p in parts)
    chosen = [v for v in args.variants.split(",") if v.split("/")[0] in flags]

    def opt(v, key):
        return next((o[len(key):] for o in v.split("/")[1:] if o.startswith(key)), "")

    if args.bvh != "host" and kind == "cornell_box_obj":
        hs = frt.HostScene.from_spec({"objects": [{"obj": obj, "geo": True}], "camera": frt.CORNELL_CAMERA,
                                      "world": "list"}, nx / ny)
        if args.bvh == "sah":
            hs.build_bvh_sah()
        else:
            bctx = frt.Context(0)
            print(json.dumps({"bvh": args.bvh, "build_ms": hs.build_bvh_gpu(bctx, args.bvh),
                              "depth": hs.info.bvh_depth}), file=sys.stderr, flush=True)
    else:
        hs = frt.HostScene(kind, obj, nx / ny)
    integ = {"path": 0, "ao": frt.FRT_INTEGRATOR_AO, "normals": frt.FRT_INTEGRATOR_NORMALS,
             "pssmlt": None}[args.integrator]
    env = args.env or ("1,1,1" if args.integrator == "ao" else "")
    if env:
        hs.set_env([float(x) for x in env.split(",")])
    ctxs = {}
    for v in chosen:   # one context per upload-time option (leaf size)
        leaf = opt(v, "leaf")
        if leaf not in ctxs:
            if leaf:
                os.environ["FRT_LEAF_SIZE"] = leaf
            else:
                os.environ.pop("FRT_LEAF_SIZE", None)
            ctxs[leaf] = frt.Context(0)
            ctxs[leaf].upload(hs)
    os.environ.pop("FRT_LEAF_SIZE", None)
    res = {v: [] for v in chosen}
    rays = {}
    films = {}
    last = {}
    for r in range(args.rounds + 1):
        for v in chosen:
            leaf = opt(v, "leaf")
            for key, env in (("trav", "FRT_TRAV_MIN"), ("desc", "FRT_MIN_DESC"), ("grab", "FRT_GRAB"),
                             ("spt", "FRT_SPI_TARGET")):
                if opt(v, key):
                    os.environ[env] = opt(v, key)
                else:
                    os.environ.pop(env, None)
            spi = int(opt(v, "spi") or 0)       # samples per work item (0: automatic)
            if integ is None:
                p = frt.RenderParams.pssmlt(nx, ny, args.spp, args.chains, seed=0)
                p.flags = flags[v.split("/")[0]]
            else:
                p = frt.RenderParams.make(nx, ny, args.spp, seed=0, flags=flags[v.split("/")[0]],
                                           samples_per_item=spi, integrator=integ)
            films[leaf], st = ctxs[leaf].render(p, films.get(leaf))
            if args.save_films:
                last[v] = np.array(films[leaf], copy=True)
            if r > 0:
                res[v].append(st.kernel_ms)
            rays[v] = st.rays
    for v in chosen:
        ms = res[v]
        print(json.dumps({"scene": args.scene, "variant": v, "spp": args.spp, "median_ms": statistics.median(ms),
                          "min_ms": min(ms), "grays_per_s": rays[v] / (statistics.median(ms) * 1e-3) / 1e9,
                          "rays": rays[v]}), flush=True)
    if len(films) > 1:   # upload-time options change addresses only: the films must be identical
        keys = list(films)
        print(json.dumps({"films_identical": {str(k): bool(np.array_equal(np.asarray(films[k]),
                                                                               np.asarray(films[keys[0]])))
                                              for k in keys[1:]}}), flush=True)
    if args.save_films:
        np.savez(args.save_films, **last)
    for c in ctxs.values():
        c.close()


if __name__ == "__main__":
    main()
