#!/usr/bin/env python3
"""Per-ray PMC figures of the megakernel for bench.py's roofline, from
rocprofv3 --pmc passes of ONE bench command (each pass its own run):

  python tools/roofline_pmc.py KEY --sq DIR --fetch DIR --write DIR --bench BENCH.json
         [--f64 DIR] [--tcc DIR] [--copy-to profiles/r03]

KEY is "<integrator>:<scene>:<nx>x<ny>" (bench.py's key).  From the LAST
*_megakernel dispatch of each pass (counters summed over dimensions):
  valu_insts_per_ray  = SQ_INSTS_VALU / rays per launch
  valu_lane_util      = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)
  hbm_bytes_per_ray   = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 / rays per launch
  valu_issue_per_ray  = (SQ_INSTS_VALU + F64 FMA/ADD/MUL + 3 x F64 TRANS) / rays
                        (--f64 pass: an fp64 FMA/ADD/MUL wave-instruction issues at
                        half the fp32 rate on MI355X, 78.6 vs 157.3 TFLOP/s vector,
                        so it takes two fp32 issue slots; an fp64 transcendental
                        (rcp/sqrt/rsq_f64) is weighted four; without the pass
                        valu_issue_per_ray = valu_insts_per_ray)
  l2_hit_rate         = TCC_HIT / (TCC_HIT + TCC_MISS)   (--tcc pass)
  wait_frac           = SQ_WAIT_ANY / SQ_WAVE_CYCLES     (--wait pass: the share of
                        wave cycles spent waiting in s_waitcnt)
  clock_ghz           = GRBM_GUI_ACTIVE / 8 / dispatch ns (--clock pass: the clock the chip
                        ran the launch at; rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs,
                        MI355X_MICROARCH.md "DVFS give-back")
  --clock-only: add just the --clock figures to KEY's existing record.
FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is doubled as MI355X_MICROARCH.md
"HBM [CDNA4]" prescribes for gfx950 (it tallies 128-B requests at 64 B).
The rays per launch come from the bench JSON the passes printed (every pass
renders the same frame; the ray count is deterministic).  Updates
profiles/roofline_pmc.json[KEY]; --copy-to keeps the CSVs under profiles/.
"""
import argparse
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_megakernel(d):
    path = os.path.join(d, "run_counter_collection.csv")
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        if "megakernel" not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    if not per:
        sys.exit(f"no megakernel dispatch in {path}")
    last = max(per)
    return names[last], dict(per[last]), path


def dispatch_ns(path, did=None):
    """End - Start timestamp of the last megakernel dispatch in a counter CSV."""
    rows = [r for r in csv.DictReader(open(path)) if "megakernel" in r["Kernel_Name"]]
    last = max(int(r["Dispatch_Id"]) for r in rows) if did is None else did
    r = next(r for r in rows if int(r["Dispatch_Id"]) == last)
    return float(r["End_Timestamp"]) - float(r["Start_Timestamp"])


def clock_fields(d):
    _, gr, p = last_megakernel(d)
    ns = dispatch_ns(p)
    return {"GRBM": gr, "clock_dispatch_ms": ns * 1e-6, "clock_ghz": gr["GRBM_GUI_ACTIVE"] / 8.0 / ns}, p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("--sq", default="")
    ap.add_argument("--fetch", default="")
    ap.add_argument("--write", default="")
    ap.add_argument("--bench", default="")
    ap.add_argument("--clock", default="")
    ap.add_argument("--clock-only", action="store_true")
    ap.add_argument("--f64", default="")
    ap.add_argument("--tcc", default="")
    ap.add_argument("--wait", default="")
    ap.add_argument("--copy-to", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "roofline_pmc.json"))
    a = ap.parse_args()
    if a.clock_only:
        t = json.load(open(a.out))
        fields, p = clock_fields(a.clock)
        if a.copy_to:
            os.makedirs(a.copy_to, exist_ok=True)
            dst = os.path.join(a.copy_to, f"pmc_{a.key.replace(':', '_')}_clock.csv")
            shutil.copy(p, dst)
            p = os.path.relpath(dst, ROOT)
        t[a.key].update(fields)
        t[a.key]["source"] = t[a.key]["source"].split(", " + p)[0] + ", " + p
        json.dump(t, open(a.out, "w"), indent=1, sort_keys=True)
        print(json.dumps(fields, indent=1))
        return
    if not (a.sq and a.fetch and a.write and a.bench):
        sys.exit("--sq, --fetch, --write and --bench are required (or --clock-only)")
    line = [l for l in open(a.bench) if l.startswith("{")][-1]
    b = json.loads(line)
    rays = b["roofline"]["rays_per_launch"]
    kname, sq, p_sq = last_megakernel(a.sq)
    _, fe, p_fe = last_megakernel(a.fetch)
    _, wr, p_wr = last_megakernel(a.write)
    fetch_b = 2.0 * fe["FETCH_SIZE"] * 1024.0
    write_b = wr["WRITE_SIZE"] * 1024.0
    rec = {
        "kernel": kname.replace("(anonymous namespace)::", "").split("(")[0],
        "rays_per_launch": rays,
        "SQ": sq, "FETCH_SIZE_KiB": fe["FETCH_SIZE"], "WRITE_SIZE_KiB": wr["WRITE_SIZE"],
        "valu_insts_per_ray": sq["SQ_INSTS_VALU"] / rays,
        "valu_lane_util": sq["SQ_THREAD_CYCLES_VALU"] / (64.0 * sq["SQ_ACTIVE_INST_VALU"]),
        "hbm_bytes_per_ray": (fetch_b + write_b) / rays,
        "read_bytes_per_ray": fetch_b / rays, "write_bytes_per_ray": write_b / rays,
        "correction": "hbm = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), MI355X_MICROARCH.md HBM [CDNA4]",
    }
    passes = [("sq", p_sq), ("fetch", p_fe), ("write", p_wr)]
    issue = sq["SQ_INSTS_VALU"]
    if a.f64:
        _, f6, p_f6 = last_megakernel(a.f64)
        passes.append(("f64", p_f6))
        arith = sum(f6.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("FMA", "ADD", "MUL"))
        trans = f6.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
        rec.update({"F64": f6, "f64_insts_per_ray": (arith + trans) / rays})
        issue += arith + 3.0 * trans
    rec["valu_issue_per_ray"] = issue / rays
    if a.tcc:
        _, tc, p_tc = last_megakernel(a.tcc)
        passes.append(("tcc", p_tc))
        rec.update({"TCC": tc, "l2_hit_rate": tc["TCC_HIT"] / max(1.0, tc["TCC_HIT"] + tc["TCC_MISS"])})
    if a.wait:
        _, wt, p_wt = last_megakernel(a.wait)
        passes.append(("wait", p_wt))
        rec.update({"WAIT": wt, "wait_frac": wt["SQ_WAIT_ANY"] / max(1.0, wt["SQ_WAVE_CYCLES"])})
    if a.clock:
        fields, p_ck = clock_fields(a.clock)
        passes.append(("clock", p_ck))
        rec.update(fields)
    srcs = []
    for tag, p in passes:
        if a.copy_to:
            os.makedirs(a.copy_to, exist_ok=True)
            dst = os.path.join(a.copy_to, f"pmc_{a.key.replace(':', '_')}_{tag}.csv")
            shutil.copy(p, dst)
            p = os.path.relpath(dst, ROOT)
        srcs.append(p)
    rec["source"] = ", ".join(srcs)
    t = json.load(open(a.out)) if os.path.exists(a.out) else {}
    t[a.key] = rec
    json.dump(t, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
