#!/usr/bin/env python3
"""HBM traffic per megakernel launch from rocprofv3 FETCH_SIZE / WRITE_SIZE
passes (separate runs), corrected as MI355X_MICROARCH.md "HBM [CDNA4]"
prescribes: FETCH_SIZE (KiB, TCC_EA0_RDREQ x 64 B) reports half the bytes of
128-B requests on gfx950, so it is doubled; WRITE_SIZE is taken as is.

  python tools/pmc_traffic.py <fetch_dir> <write_dir> <key> <out.json>

Updates profiles/pmc_traffic.json[key] (bench.py reads it as roofline.traffic)."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    out = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        out[k] = out.get(k, 0.0) + float(r["Counter_Value"])
    return out


def main():
    fdir, wdir, key, dst = sys.argv[1:5]
    f = per_dispatch(fdir, "FETCH_SIZE")
    w = per_dispatch(wdir, "WRITE_SIZE")
    kern = {}
    for src, name, scale in ((f, "FETCH_SIZE", 1.0), (w, "WRITE_SIZE", 1.0)):
        for (did, kname), v in src.items():
            short = kname.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            kern.setdefault(short, {}).setdefault(name, []).append(v * scale)
    summary = {}
    for k, v in kern.items():
        fe = max(v.get("FETCH_SIZE", [0.0]))
        wr = max(v.get("WRITE_SIZE", [0.0]))
        summary[k] = {"FETCH_SIZE_KiB": fe, "WRITE_SIZE_KiB": wr,
                      "hbm_bytes_corrected": 2.0 * fe * 1024 + wr * 1024}
    mk = [k for k in summary if "megakernel" in k]
    out = {"round": 1, "key": key, "fetch_dir": fdir, "write_dir": wdir,
           "correction": "hbm_bytes = 2 * FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM [CDNA4]); per launch",
           "kernels": summary}
    if mk:
        out["megakernel"] = mk[0]
        out["megakernel_hbm_bytes_per_launch"] = summary[mk[0]]["hbm_bytes_corrected"]
        tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        t = json.load(open(tp)) if os.path.exists(tp) else {}
        t[key] = out["megakernel_hbm_bytes_per_launch"]
        json.dump(t, open(tp, "w"), indent=1, sort_keys=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
