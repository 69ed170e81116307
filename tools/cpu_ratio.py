#!/usr/bin/env python3
"""the CPU baseline's restatement-to-reference time ratio.

Times the oracle (oracle/frt_oracle.c, the fp64 C restatement bench.py's
cpu_baseline runs) single-threaded on C1 -- CornellBox-Original 256x256 x 16
spp, full frame, path::Li -- in this container, and relates it to SURVEY.md
section 6's measurement of first_ray itself on the same container and config:
2.14 Mrays/s on one thread (12.60 M rays in 5.89 s; path.cpp:4-116 driven by
integrator.h:19-45).  Writes profiles/r06/cpu_ratio.json, which bench.py reads
to put a "first_ray on this host" estimate beside cpu_baseline.  (Round 6
re-timed the oracle side on the current RNG; first_ray's side stays the
survey's probe: first_ray needs cpp-taskflow and GLFW, absent from this image,
and the task rules forbid building the reference against stand-ins.)

    python tools/cpu_ratio.py [--reps 5]
"""
import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

FIRST_RAY_MRAYS_1T = 2.14       # SURVEY.md section 6, same container, C1
FIRST_RAY_RAYS = 12.60e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    obj = os.path.join(ROOT, "tests", "golden", "scenes", "CornellBox-Original.obj")
    sc = oracle.OracleScene("cornell_box_obj", obj, 1.0)
    runs = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        _, cnt = sc.render(256, 256, 16, seed=0, nthreads=1)
        dt = time.perf_counter() - t0
        runs.append({"seconds": dt, "rays": cnt.rays, "mrays": cnt.rays / dt / 1e6})
    med = statistics.median(r["mrays"] for r in runs)
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    out = {
        "config": "C1: CornellBox-Original 256x256 x 16 spp, full frame, path::Li, 1 thread",
        "oracle_mrays_1thread": round(med, 3), "oracle_runs": runs,
        "oracle_rays": runs[0]["rays"], "first_ray_rays": FIRST_RAY_RAYS,
        "first_ray_mrays_1thread": FIRST_RAY_MRAYS_1T,
        "ratio_port_over_first_ray": round(med / FIRST_RAY_MRAYS_1T, 3),
        "host": {"cpu": cpu, "machine": platform.machine()},
        "source": "SURVEY.md section 6 (first_ray, same container, g++ -O3 -march=native, 1 thread)",
        "measured": time.strftime("round 6, %Y-%m-%d"),
        "oracle_spread": [round(min(r["mrays"] for r in runs), 3), round(max(r["mrays"] for r in runs), 3)],
    }
    dst = os.path.join(ROOT, "profiles", "r06", "cpu_ratio.json")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("oracle_mrays_1thread", "ratio_port_over_first_ray")}))


if __name__ == "__main__":
    main()
