#!/usr/bin/env python3
"""PSS-MLT start-up bias of the reference's algorithm, on the CPU oracle only
(oracle/ora_mlt_render: pssmlt.cpp restated, chains started from a uniform
state with no burn-in, pssmlt.cpp:301-365).  The image mean of the MLT film,
with the normaliser b's bootstrap noise divided out (reference b from 10^7
paths), against the oracle's path tracer at pssmlt's depth cap, for growing
chain lengths at a fixed chain count.  A transient of the chains shows as a
bias that shrinks with the chain length; the GPU kernel runs the same chains
(tests/test_gpu_pssmlt.py), so this is the reference's behaviour, not a GPU
effect.  Test infrastructure: imports the oracle.

    python tools/mlt_startup_bias.py > profiles/r04/mlt_startup_bias.json
"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import oracle
    import bench
    nx, ny, chains, threads = 32, 24, 96, min(16, os.cpu_count() or 1)
    kind, obj, name = bench.scene_spec("cornell", "/tmp")
    sc = oracle.OracleScene(kind, obj, nx / ny)
    ref = sc.render(nx, ny, 4096, seed=5, nthreads=threads, max_depth=bench.MLT_MAX_PATH)[0]
    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(lambda k: sc.mlt_bootstrap(nx, ny, seed=1234 + 7919 * k, n_init=625000), range(16)))
    b_ref = float(np.mean(parts))
    rm = float(ref.reshape(-1, 3).mean(0).mean())
    rows = []
    for steps in (2048, 8192, 32768, 131072):
        errs = []
        for seed in (7, 8, 9, 10):
            film, b, _ = sc.mlt_render(nx, ny, chains, steps, seed=seed, nthreads=threads)
            errs.append(float(film.reshape(-1, 3).mean(0).mean() * b_ref / b / rm - 1.0))
        rows.append({"steps_per_chain": steps, "mean_rel_err_b_corrected": float(np.mean(errs)),
                     "per_seed": errs})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"scene": name, "res": f"{nx}x{ny}", "chains": chains, "path_reference_spp": 4096,
                      "max_depth": bench.MLT_MAX_PATH, "b_ref": b_ref, "b_ref_paths": 16 * 625000,
                      "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
