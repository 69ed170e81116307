#!/usr/bin/env python3
"""TEST INFRASTRUCTURE.  Regenerate tests/golden/kat_ref.json from the reference.

Builds oracle/_ref/ref_kat from the reference sources (`make -C oracle ref`,
needs /root/reference), runs it with HOME pointed at a scratch dir (the
reference's PFM writer prefixes $HOME, image.h:94-98) and stores every case as
hex-float strings, so the restatement can be checked bit for bit:

    {"tri_hit": [[ins...], [outs...]], ...,  "pfm": {"nx":..,"ny":..,"data":[..],"bytes_hex":".."}}

Usage: python3 oracle/gen_golden.py [ncases]
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    subprocess.check_call(["make", "-s", "-C", HERE, "ref"])
    with tempfile.TemporaryDirectory() as home:
        env = dict(os.environ, HOME=home)
        out = subprocess.check_output([os.path.join(HERE, "_ref", "ref_kat"), str(n)], env=env, text=True)
        # metal / rough_conductor: own program (util.h sincos, see ref_kat_conductor.cpp)
        out += subprocess.check_output([os.path.join(HERE, "_ref", "ref_kat_conductor"), str(n)], env=env,
                                       text=True, timeout=60)
        cases = {}
        pfm = None
        for line in out.splitlines():
            if "|" not in line:
                continue  # the reference's "Filename is now ..." chatter
            head, tail = line.split("|", 1)
            kind, *ins = head.split()
            outs = tail.split()
            if kind == "pfm":
                with open(os.path.join(home, outs[0]), "rb") as f:
                    raw = f.read()
                nx, ny = int(float.fromhex(ins[0])), int(float.fromhex(ins[1]))
                pfm = {"nx": nx, "ny": ny, "data": ins[2:], "bytes_hex": raw.hex()}
                continue
            cases.setdefault(kind, []).append([ins, outs])
    cases["pfm"] = pfm
    cases["_meta"] = {
        "generator": "oracle/ref_kat.cpp + ref_kat_conductor.cpp (built from /root/reference/first_ray sources by oracle/Makefile `ref`)",
        "ncases": n,
        "format": "hex floats (float.fromhex); per kind: [inputs, outputs]",
    }
    dst = os.path.join(ROOT, "tests", "golden", "kat_ref.json")
    with open(dst, "w") as f:
        json.dump(cases, f, separators=(",", ":"))
    print("wrote", dst, os.path.getsize(dst), "bytes;", {k: len(v) for k, v in cases.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
