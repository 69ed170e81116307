#!/usr/bin/env python3
"""Register-cap fault, per path vertex: an experiment build with
FRT_DBG_CAPTURE (frt_dbg_set / frt_dbg_read) records the path state of one
(pixel, sample) before and after each shading step and after each shadow
ray.  Renders the conductor scene (tools/caps_table.py) on one plan at a
good and a bad cap, picks the pixel that differs most, and prints the first
sample whose records differ, record by record.

    FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_fail_dbg.so python tools/caps_dbg.py --flags 17 --good 0 --bad 4
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
NAMES = ["tag", "depth", "prim", "t", "u", "v", "ro.x", "ro.y", "ro.z", "rd.x", "rd.y", "rd.z",
         "beta.x", "beta.y", "beta.z", "L.x", "L.y", "L.z", "nee.x", "nee.y", "nee.z",
         "nxt_d.x", "nxt_d.y", "nxt_d.z", "prev_pdf", "shadow", "term", "prev_spec",
         "prev_p.x", "prev_p.y", "prev_p.z", "pad"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", type=int, default=17)
    ap.add_argument("--good", default="0")
    ap.add_argument("--bad", default="4")
    ap.add_argument("--pixels", type=int, default=3)
    a = ap.parse_args()
    import torch  # noqa: F401
    import first_raytracer_amd as frt
    import oracle
    import scene_specs as SS
    nx, ny, spp = 64, 48, 16
    spec = SS.cornell_conductors("beckmann", "ggx", "bvh")
    ref, _ = oracle.OracleScene.from_spec(spec, nx / ny).render(nx, ny, spp, seed=12)
    ref = np.asarray(ref, np.float64).reshape(-1, 3)
    ctx = frt.Context(0)
    ctx.upload(frt.HostScene.from_spec(spec, nx / ny))
    lib = frt._lib
    lib.frt_dbg_set.argtypes = [ctypes.c_int, ctypes.c_int]
    buf = (ctypes.c_float * (32 * 256))()
    n = ctypes.c_int()

    def render(cap, pix=-1, s=-1):
        os.environ["FRT_MATS_WAVES"] = cap
        assert lib.frt_dbg_set(pix, s) == 0
        film, st = ctx.render(frt.RenderParams.make(nx, ny, spp, seed=12, flags=a.flags))
        assert lib.frt_dbg_read(buf, ctypes.byref(n)) == 0
        recs = np.frombuffer(buf, np.float32).reshape(256, 32)[: n.value].copy()
        return np.asarray(film, np.float64).reshape(-1, 3), recs

    fg, _ = render(a.good)
    fb, _ = render(a.bad)
    print("rmse good", float(np.sqrt(np.mean((fg - ref) ** 2))), "bad", float(np.sqrt(np.mean((fb - ref) ** 2))), flush=True)
    d = np.abs(fg - fb).max(axis=1)
    bad = np.nonzero(d > 1e-6)[0]
    print("pixels differing:", len(bad), flush=True)
    for pix in bad[np.argsort(-d[bad])][: a.pixels]:
        pix = int(pix)
        print(f"pixel {pix} ({pix % nx},{pix // nx}) good {fg[pix]} bad {fb[pix]} oracle {ref[pix]}", flush=True)
        for s in range(spp):
            _, rg = render(a.good, pix, s)
            _, rb = render(a.bad, pix, s)
            if rg.shape == rb.shape and np.array_equal(rg, rb):
                continue
            print(f"  sample {s}: {len(rg)} / {len(rb)} records", flush=True)
            for k in range(max(len(rg), len(rb))):
                g = rg[k] if k < len(rg) else None
                b = rb[k] if k < len(rb) else None
                if g is not None and b is not None and np.array_equal(g, b):
                    print(f"    rec {k} tag {int(g[0])} depth {int(g[1])}: same", flush=True)
                    continue
                print(f"    rec {k} DIFFERS", flush=True)
                for j, nm in enumerate(NAMES):
                    gv = None if g is None else float(g[j])
                    bv = None if b is None else float(b[j])
                    if gv != bv:
                        print(f"      {nm:9s} good {gv!r:>24} bad {bv!r:>24}", flush=True)
                break
            break
    ctx.close()


if __name__ == "__main__":
    main()
