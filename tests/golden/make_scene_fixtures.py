#!/usr/bin/env python3
"""Copy the scene DATA the hot-path configs need into tests/golden/scenes/.

CornellBox-Original (public domain, Williams College 2011; see
first_ray/CornellBox/copyright.txt) and veach_mi are data, not code.  The GPU
box has no /root/reference, so the parity tests and bench.py read these
copies.  Tokens are kept verbatim (float parsing follows Assimp's
fast_atoreal_move token by token); comments and blank lines are dropped and
whitespace is normalised.
"""
import os

REF = "/root/reference/first_ray"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
FILES = ["CornellBox/CornellBox-Original.obj", "CornellBox/CornellBox-Original.mtl",
         "veach_mi/veach_mi.obj", "veach_mi/veach_mi.mtl",
         # modified_phong variants (Ks != 0, opacity 1: mesh_loader.cpp:78-100)
         "CornellBox/CornellBox-Glossy-Floor.obj",
         "CornellBox/CornellBox-Glossy.mtl",   # the mtllib CornellBox-Glossy-Floor.obj names
         "CornellBox/CornellBox-Sphere.obj", "CornellBox/CornellBox-Sphere.mtl",
         "CornellBox/CornellBox-Mirror.obj", "CornellBox/CornellBox-Mirror.mtl"]


def normalise(text):
    out = []
    for line in text.splitlines():
        line = line.split("#", 1)[0].strip()
        if line:
            out.append(" ".join(line.split()))
    return "\n".join(out) + "\n"


def main():
    os.makedirs(DST, exist_ok=True)
    for rel in FILES:
        with open(os.path.join(REF, rel)) as f:
            data = normalise(f.read())
        with open(os.path.join(DST, os.path.basename(rel)), "w") as f:
            f.write("# scene data from jammm/first_raytracer first_ray/%s (normalised)\n" % rel)
            f.write(data)
        print("wrote", os.path.basename(rel))


if __name__ == "__main__":
    main()
