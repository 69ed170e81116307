#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs for the megakernels: per pass
directory, the LAST dispatch of each *_megakernel (the timed round), counters
summed over dimensions.  Derived: lane utilisation of VALU issue
(SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)), mean VMEM latency in
cycles (SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM_RD), L2 hit rate.

  python tools/pmc_summary.py gpurun_out/pmc2 [--json out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict


def load(d):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in rows:
        if "megakernel" not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    if not per:
        return None, {}
    last = max(per)
    return names[last], dict(per[last])


def main():
    root = sys.argv[1]
    out = {}
    groups = defaultdict(dict)
    for sub in sorted(os.listdir(root)):
        p = os.path.join(root, sub)
        if not os.path.isdir(p) or not os.path.exists(os.path.join(p, "run_counter_collection.csv")):
            continue
        name, c = load(p)
        key = sub.rsplit("_", 1)[0]
        groups[key].update(c)
        groups[key]["kernel"] = name
    for key, c in groups.items():
        d = {k: v for k, v in c.items()}
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_THREAD_CYCLES_VALU" in c:
            d["valu_lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
        if "SQ_INST_LEVEL_VMEM" in c and c.get("SQ_INSTS_VMEM_RD"):
            d["vmem_latency_cyc"] = c["SQ_INST_LEVEL_VMEM"] / c["SQ_INSTS_VMEM_RD"]
        if "SQ_INST_LEVEL_LDS" in c and c.get("SQ_INSTS_LDS"):
            d["lds_latency_cyc"] = c["SQ_INST_LEVEL_LDS"] / c["SQ_INSTS_LDS"]
        if "TCC_HIT_sum" in c:
            d["l2_hit"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
            d["wait_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
            d["valu_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        out[key] = d
        print(key, d.get("kernel", "")[:90])
        for k in ("valu_lane_util", "vmem_latency_cyc", "lds_latency_cyc", "l2_hit", "wait_frac",
                  "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_BUSY_CYCLES",
                  "TCC_EA0_RDREQ_sum", "TCC_REQ_sum"):
            if k in d:
                print(f"   {k:20s} {d[k]:.4g}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
