#!/usr/bin/env python3
"""Golden images: converged renders of the oracle, the fp64 C
restatement of path::Li (oracle/), committed as small fixtures.

  cornell_64x64_16384spp.pfm          CornellBox-Original, 64x64, 16384 spp, seed 1000
  cornell_256x256_1024spp_blocks.json the 256x256 1024 spp render as 8x8-pixel block means
  veach_96x64_1024spp.pfm             veach_mis (C3 geometry), 96x64, 1024 spp, seed 1000

Run from the repo root after `make -C oracle`:  python tests/golden/make_golden_images.py
The images are linear radiance, PFM rows y = 0 first (image.h:89-118)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
SCENES = os.path.join(HERE, "scenes")
SEED = 1000


def write_pfm(path, img):
    h, w, _ = img.shape
    with open(path, "wb") as f:
        f.write(b"PF\n%d %d\n-1\n" % (w, h))
        f.write(np.ascontiguousarray(img, "<f4").tobytes())


def render(kind, obj, nx, ny, spp):
    t = time.time()
    out, cnt = oracle.OracleScene(kind, obj, nx / ny).render(nx, ny, spp, seed=SEED)
    print(f"{kind} {nx}x{ny} {spp}spp: {time.time() - t:.1f}s, {cnt.rays} rays", flush=True)
    return out.reshape(ny, nx, 3)


def main():
    cornell = os.path.join(SCENES, "CornellBox-Original.obj")
    veach = os.path.join(SCENES, "veach_mi.obj")
    img = render("cornell_box_obj", cornell, 64, 64, 16384)
    write_pfm(os.path.join(HERE, "cornell_64x64_16384spp.pfm"), img)
    img = render("cornell_box_obj", cornell, 256, 256, 1024)
    blocks = img.reshape(32, 8, 32, 8, 3).mean(axis=(1, 3))
    json.dump({"scene": "cornell_box_obj", "nx": 256, "ny": 256, "spp": 1024, "seed": SEED, "block": 8,
               "generator": "oracle (fp64 C restatement of path::Li), tests/golden/make_golden_images.py",
               "mean": img.reshape(-1, 3).mean(0).tolist(),
               "block_means": blocks.round(7).tolist()},
              open(os.path.join(HERE, "cornell_256x256_1024spp_blocks.json"), "w"))
    img = render("veach_mis", veach, 96, 64, 1024)
    write_pfm(os.path.join(HERE, "veach_96x64_1024spp.pfm"), img)


if __name__ == "__main__":
    main()
