#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X path integrator on the BASELINE.json config
(CornellBox-Original, 1920x1080, 512 spp, path + NEE + MIS), with the image
tiles sharded over N GPUs (one process per GPU, RCCL gather of the tile
radiance to rank 0 over xGMI), plus the roofline of the path megakernel and
the CPU baseline (the fp64 C restatement, oracle/, timed on this host's cores).

The same JSON line carries the north-star run (BASELINE.json north_star, SURVEY
§8(d) C4): the 1,005,858-triangle tessellated Cornell box at 1920x1080 / 512
spp, sharded the same way, timed the same way, with its own RMSE against the
oracle and its own roofline ("north_star": {...}).  It also carries BASELINE.json's
configs[2] and [4] as blocks "c3" (veach_mi 1080p 1024 spp, the fp64 list-world
kernel) and "c5" (PSS-MLT on CornellBox 1080p, 512 mutations per pixel, 2^18
chains), each timed the same way (3 frames after 1 warm-up) with its own RMSE
against the oracle (C5: path-exact on a chain shard of the config), roofline
and CPU figure, so the driver's default run measures four of the five configs
(C1 is the reference's own CPU plumbing case).

One "step" = one full frame: every rank renders its tiles (tile t -> rank
t mod N) into HBM, then the per-rank slot buffers are gathered to rank 0,
which scatters them into the film.  Scene build and upload happen before the
timed region.

    python bench.py [--gpus N --steps K --warmup W] [--scene cornell|cornell_1m|veach|sphere]

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec + RMSE vs CPU ref, CornellBox 1080p 512spp, 1/2/4/8 MI355X"
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
# MI355X_MICROARCH.md: HBM3E 8.0 TB/s; 256 CUs x 4 SIMD-32 at 2.4 GHz, a wave64
# VALU instruction issues over 2 cycles -> 1228.8 G wave-instructions/s; LDS
# aggregate ~150 TB/s for ds_read_b64/b128
HBM_PEAK_GBS = 8000.0
VALU_PEAK_CLOCK_GHZ = 2.4
VALU_PEAK_GINST = 256 * 4 * VALU_PEAK_CLOCK_GHZ / 2.0
LDS_PEAK_GBS = 150000.0
L2_XCD_BYTES = 4 << 20          # one XCD's L2 (MI355X_MICROARCH.md)
NODE_BYTES, TRI_BYTES, RAY_BYTES = 32, 48, 32   # B_ray = 32 V + 48 T + 32
NS_TARGET_MRAYS = 1000.0                        # north_star: >= 1 Gray/s on one MI355X


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Heartbeat:
    """A line on stderr every `every` s while rank 0 runs long oracle work (the
    oracle's C calls release the GIL), so a long CPU phase is not silent."""

    def __init__(self, what, every=30.0):
        import threading
        self.what, self.every, self.t0 = what, every, time.perf_counter()
        self.stop = threading.Event()
        self.th = threading.Thread(target=self.run, daemon=True)

    def run(self):
        while not self.stop.wait(self.every):
            log(f"bench: {self.what} running, {time.perf_counter() - self.t0:.0f} s")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv, script=None, env=None, poll_s=0.5):
    """`bench.py --gpus N` without a launcher (no WORLD_SIZE in the
    environment): start N rank processes of this script with RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT, as torchrun
    would, and wait for them.  The parent never touches the GPU (it only counts
    devices, which does not initialise HIP on this image), so the children are
    fresh processes, not exec'd replacements.  Returns 0 when every rank exits
    0; when one fails, the others are terminated (by their own PIDs) and its
    exit code is returned, so a run with fewer than N working ranks cannot print
    a line."""
    import subprocess
    script = script or os.path.abspath(__file__)
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=e))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(poll_s)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                log(f"bench: rank {procs.index(p)} exited with {code}; stopping the other ranks")
                for q in live:
                    q.terminate()
    for p in procs:
        p.wait()
    return rc


def check_world(gpus, world, backend, n_devices):
    """The rank set must be the one asked for: WORLD_SIZE == --gpus, and with
    RCCL one device per rank (gloo rehearsals may share devices).  Returns an
    error message or None."""
    if world != gpus:
        return f"--gpus {gpus} but WORLD_SIZE {world}: refusing to measure a different rank count"
    if n_devices < 1:
        return "no GPU visible"
    if backend == "nccl" and n_devices < world:
        return f"--gpus {world} needs {world} GPUs for RCCL, {n_devices} visible"
    return None


def host_cpus():
    """CPUs this process may use: its affinity mask, capped by the cgroup CPU
    quota (a GPU box shares a large host; nproc reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def scene_spec(name, workdir, tag=""):
    """(scene kind, OBJ path, label).  cornell_1m is generated on first use;
    `tag` keeps concurrent ranks on their own files."""
    if name == "cornell":
        return "cornell_box_obj", os.path.join(SCENES, "CornellBox-Original.obj"), "CornellBox-Original"
    if name == "veach":
        return "veach_mis", os.path.join(SCENES, "veach_mi.obj"), "veach_mi"
    if name == "sphere":   # modified_phong spheres (specular branch)
        return "cornell_box_obj", os.path.join(SCENES, "CornellBox-Sphere.obj"), "CornellBox-Sphere"
    if name == "cornell_1m":
        import first_raytracer_amd as frt
        dst = os.path.join(workdir, f"cornell_1m_k172{tag}.obj")
        if not os.path.exists(dst):
            frt.write_tessellated_obj(os.path.join(SCENES, "CornellBox-Original.obj"), 172, dst)
        return "cornell_box_obj", dst, "cornell_1m (k=172, 1,005,858 tris)"
    raise ValueError(name)


def load_profile(fname, key):
    path = os.path.join(ROOT, "profiles", fname)
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f).get(key)
    return None


def cpu_baseline(kind, obj, nx, ny, spp, seed, npix, threads, film, seconds, integrator=0, env=None, min_frac=0.0):
    """The oracle (fp64 C restatement) on a bounded pixel sample of the same
    frame and RNG streams: CPU Mrays/s, reference traversal counters (for
    B_ray) and the RMSE of the GPU film on those pixels.  npix = 0: calibrate
    on growing samples (from 512 pixels) until one takes about `seconds` of CPU
    work; the CPU rate comes from that run.  The RMSE sample then grows, if
    needed, with more evenly spaced pixels to cover at least `min_frac` of the
    frame (the rate stays bounded by `seconds`; the extra pixels'
    time is reported as rmse_extra_seconds)."""
    import oracle
    sc = oracle.OracleScene(kind, obj, nx / ny)
    if env is not None:
        sc.set_env(env)

    def run(n):
        pix = np.unique(np.linspace(0, nx * ny - 1, n).astype(np.int32))
        t0 = time.perf_counter()
        out, cnt = sc.render(nx, ny, spp, seed=seed, pixels=pix, nthreads=threads, integrator=integrator)
        return pix, out, cnt, time.perf_counter() - t0

    if npix > 0:
        pix, out, cnt, dt = run(npix)
    else:                                   # grow the sample until it takes >= seconds/2
        npix = 512
        while True:
            pix, out, cnt, dt = run(npix)
            if dt >= 0.5 * seconds or npix >= nx * ny:
                break
            npix = int(min(nx * ny, npix * min(16.0, max(2.0, seconds / max(dt, 1e-3)))))
    rays = cnt.rays
    n_timed = len(pix)
    extra_s = 0.0
    min_pix = int(min_frac * nx * ny)
    if len(pix) < min_pix:                  # RMSE coverage: more evenly spaced pixels, not timed
        more = np.setdiff1d(np.unique(np.linspace(0, nx * ny - 1, min_pix).astype(np.int32)), pix)
        t0 = time.perf_counter()
        out2, _ = sc.render(nx, ny, spp, seed=seed, pixels=more, nthreads=threads, integrator=integrator)
        extra_s = time.perf_counter() - t0
        pix, out = np.concatenate([pix, more]), np.concatenate([out, out2])
    gpu = film.reshape(-1, 3)[pix].astype(np.float64)
    rmse = float(np.sqrt(np.mean((gpu - out) ** 2)))
    # fp32 vs fp64 rounding occasionally sends one sample down another branch
    # (a silhouette, the light's edge); such a pixel differs by ~radiance/spp.
    # Reported apart so a systematic error would show in rmse_converged.
    dev = np.abs(gpu - out).max(axis=1)
    bad = dev > 1e-3
    rmse_conv = float(np.sqrt(np.mean((gpu[~bad] - out[~bad]) ** 2))) if (~bad).any() else None
    return {
        "mrays": rays / dt / 1e6, "seconds": dt, "rays": rays, "npix": n_timed, "rmse_pixels": int(len(pix)),
        "V": cnt.node_visits / rays, "T": (cnt.tri_tests + cnt.sphere_tests) / rays,
        "rays_per_sample": rays / cnt.samples, "rmse": rmse,
        "diverged_pixels": int(bad.sum()), "rmse_converged": rmse_conv, "rmse_extra_seconds": round(extra_s, 2),
    }


def cpu_baseline_mlt(ctx, r, mpp, n_chains, seed, threads, seconds, shards=0):
    """C5's CPU baseline and path-exact parity in one: the oracle's PSS-MLT
    (pssmlt.cpp restated in fp64) on the chains of shard (0, K) of the config
    itself -- every one of them runs the config's full mutation count -- with K
    halved from 1024 (a power of two, at least 16) until the oracle's run takes
    about `seconds`; the GPU renders the same shard for the comparison
    (mlt_shard_parity).  `r` is the measured render (bench.Runner.measure):
    its scene must still be the one uploaded to ctx.  A request with fewer
    mutations than chains (0 steps per chain) has no chain to compare: the
    parity is None, with a note."""
    nx, ny = r["nx"], r["ny"]
    if mpp * nx * ny // n_chains <= 0:
        return {"mrays": None, "seconds": 0.0, "rays": 0, "npix": 0, "V": None, "T": None, "parity": None,
                "sample": "none", "note": (f"{mpp} mutations/pixel x {nx}x{ny} < {n_chains} chains: 0 mutations "
                                           f"per chain, no path-exact parity")}
    K = shards if shards > 0 else 1024      # shards = 1: every chain of the frame (no estimate)
    while True:
        par = mlt_shard_parity(ctx, r["kind"], r["obj"], nx, ny, mpp, n_chains, K, seed, threads, env=r["env"])
        dt = par["oracle_seconds"]
        if shards > 0 or dt >= 0.5 * seconds or K <= 16 or K >= n_chains:
            break
        K = max(16, K >> max(1, min(4, int(math.ceil(math.log2(seconds / max(dt, 1e-3)))))))
    par.pop("gpu_film")
    return {"mrays": par["oracle_mrays"], "seconds": dt, "rays": par["rays_oracle"], "npix": 0,
            "V": par["oracle_counters"]["V"], "T": par["oracle_counters"]["T"], "parity": par,
            "sample": (f"the {par['chains']} chains c = 0 mod {K} of the config's {n_chains}, "
                       f"{par['steps_per_chain']} mutations each")}


def mlt_shard_parity(ctx, kind, obj, nx, ny, mpp, n_chains, shard_count, seed, threads, shard_index=0,
                     n_init=10000, flags=0, env=None):
    """C5 path-exact parity at the config itself: the GPU
    renders shard (shard_index, shard_count) of the PSS-MLT request -- the
    chains c = shard_index + j * shard_count of n_chains, each with the
    config's full mutation count -- and the oracle's pssmlt.cpp restatement
    (ora_mlt_render_shard, fp64) runs the same chains on the same counter-RNG
    streams.  Returns the comparison and the oracle's CPU timing (the C5 CPU
    baseline: the reference algorithm on a bounded sample of the same chains).

    * chains: a chain is path-exact when its trajectory fingerprint (accepted
      proposals, sum of the accepted steps' indices) equals the oracle's.
      fp32 rounding can flip one accept or one hit decision and send a chain
      elsewhere until both copies accept the same large step (whose state is
      the RNG's alone), so `diverged_chains` counts the chains whose
      fingerprints differ;
    * film: the shard films (splats scaled as in the full render) compared
      per pixel and in 8x8-block means, with their means;
    * rays: camera + extension + shadow counts."""
    import oracle
    import first_raytracer_amd as frt
    film = np.zeros((ny, nx, 3), np.float32)
    film, st = ctx.render(frt.RenderParams.pssmlt(nx, ny, mpp, n_chains, seed=seed, bootstrap=n_init,
                                                  shard_index=shard_index, shard_count=shard_count, flags=flags), film)
    n_local = int(st.work_items)
    u_gpu, fp_gpu = ctx.mlt_chain_state(0, n_local)
    steps = mpp * nx * ny // n_chains
    sc = oracle.OracleScene(kind, obj, nx / ny)
    if env is not None:                       # the GPU scene's environment (bench --env)
        sc.set_env(env)
    t0 = time.perf_counter()
    ref, b, cnt, fp_ora, u_ora = sc.mlt_render_shard(nx, ny, n_chains, steps, shard_index, shard_count, seed=seed,
                                                     n_init=n_init, nthreads=threads)
    dt = time.perf_counter() - t0
    same = np.all(fp_gpu == fp_ora, axis=1)
    g, o = film.astype(np.float64), ref
    du = np.abs(u_gpu.astype(np.float64) - u_ora).max(axis=1) if n_local else np.zeros(0)
    bs = 8
    gb = g[: ny // bs * bs, : nx // bs * bs].reshape(ny // bs, bs, nx // bs, bs, 3).mean(axis=(1, 3))
    ob = o[: ny // bs * bs, : nx // bs * bs].reshape(ny // bs, bs, nx // bs, bs, 3).mean(axis=(1, 3))
    peak = float(np.abs(o).max())
    rmse = float(np.sqrt(np.mean((g - o) ** 2)))
    return {
        "shard": [shard_index, shard_count], "chains": n_local, "n_chains": n_chains, "steps_per_chain": steps,
        "samples_gpu": int(st.samples), "samples_oracle": int(cnt.samples),
        "rays_gpu": int(st.rays), "rays_oracle": int(cnt.rays),
        "rays_rel_diff": float(abs(int(st.rays) - int(cnt.rays)) / max(1, int(cnt.rays))),
        "path_exact_chains": int(same.sum()), "diverged_chains": int((~same).sum()),
        "diverged_frac": float((~same).mean()) if n_local else 0.0,
        "accepts_gpu": int(fp_gpu[:, 0].astype(np.int64).sum()), "accepts_oracle": int(fp_ora[:, 0].astype(np.int64).sum()),
        "state_maxdiff_path_exact": float(du[same].max()) if same.any() else None,
        "film_rmse": rmse, "film_peak": peak, "film_rmse_over_peak": rmse / max(1.0, peak),
        # the K shard films sum to the full film and their errors are independent (disjoint
        # chains), so the full frame's squared error is about K x one shard's
        "full_frame_rmse_est": rmse * math.sqrt(shard_count),
        "film_rel_l2": float(np.linalg.norm(g - o) / max(np.linalg.norm(o), 1e-30)),
        "block8_rel_l2": float(np.linalg.norm(gb - ob) / max(np.linalg.norm(ob), 1e-30)),
        "mean_gpu": [float(x) for x in g.reshape(-1, 3).mean(0)], "mean_oracle": [float(x) for x in o.reshape(-1, 3).mean(0)],
        "mean_rel_diff": float(g.mean() / o.mean() - 1.0) if o.mean() > 0 else None,
        "b_oracle": float(b),
        "oracle_seconds": dt, "oracle_mrays": cnt.rays / dt / 1e6, "oracle_threads": threads,
        "oracle_counters": {"V": cnt.node_visits / max(1, cnt.rays), "T": (cnt.tri_tests + cnt.sphere_tests) / max(1, cnt.rays)},
        "gpu_film": film,
    }


MLT_MAX_PATH = 10     # pssmlt.h MaxPathLength: pssmlt::Li traces depths 0..10 (pssmlt.cpp:151)


def mlt_block_rmse(kind, obj, nx, ny, film, threads, seconds, spp=256, block=8, seed=0, n_init=10000,
                   max_blocks=None, env=None):
    """C5's "RMSE vs CPU ref".  PSS-MLT (pssmlt.cpp) and path::Li estimate the
    same image with different samples, so no stream is shared and no pixel is
    path-exact at 1080p (chains run ~4000 mutations; pssmlt.cpp has no
    burn-in, so chains also carry start-up bias, ~0 % at this length).  The
    comparison is statistical: 8x8-block means of the GPU's PSS-MLT film
    against the oracle's fp64 path::Li with pssmlt's depth cap (max_depth 10)
    at `spp` per pixel on an evenly spaced sample of blocks, grown until it
    takes about `seconds`.  The oracle renders its samples in two independent
    halves (two frame seeds); oracle_noise = RMSE(half1 - half2) / 2 is the
    reference's own noise on the block means.
    PSS-MLT's image is scaled by its normaliser b, the mean scalar
    contribution of N_Init = 10^4 bootstrap paths (pssmlt.cpp:303-312): the
    whole image inherits b's sampling error (several % on Cornell, where
    camera paths that see the light score ~17).  The oracle recomputes the b
    this render used (same bootstrap streams) and a reference b from 10^7
    paths of other streams; `b_factor` = b_ref / b_used undoes the
    normalisation noise, so the remaining error is the chains' own.  The light's
    blocks (radiance ~17) carry most of the squared error of both estimators,
    so the gates are on the b-corrected film: the median per-block relative
    error |g - r| / (r + 0.01) <= 0.05 and the mean over the sampled blocks
    within 2 % (tests/test_gpu_pssmlt.py::test_block_means_match_oracle_path).
    `rmse` is the plain RMSE of the block means (linear radiance, uncorrected);
    `rmse_b_corrected` the same after the b correction."""
    import oracle
    sc = oracle.OracleScene(kind, obj, nx / ny)
    if env is not None:
        sc.set_env(env)
    bx, by = nx // block, ny // block
    img = np.asarray(film, np.float64).reshape(ny, nx, 3)

    def run(nb):
        ids = np.unique(np.linspace(0, bx * by - 1, nb).astype(np.int64))
        x0, y0 = (ids % bx) * block, (ids // bx) * block
        d = np.arange(block)
        pix = ((y0[:, None, None] + d[None, :, None]) * nx + (x0[:, None, None] + d[None, None, :])).reshape(-1)
        t0 = time.perf_counter()
        halves = [sc.render(nx, ny, spp // 2, seed=s, pixels=pix.astype(np.int32), nthreads=threads,
                            max_depth=MLT_MAX_PATH)[0].reshape(len(ids), block * block, 3).mean(axis=1)
                  for s in (0x5EED0001, 0x5EED0002)]
        gpu = img[(y0[:, None, None] + d[None, :, None]), (x0[:, None, None] + d[None, None, :])]
        return ids, halves, gpu.reshape(len(ids), block * block, 3).mean(axis=1), time.perf_counter() - t0

    nb = bx * by if max_blocks is None else min(bx * by, max_blocks)
    if seconds > 0:
        nb = min(nb, 64)
    while True:
        ids, (h1, h2), g, dt = run(nb)
        if seconds <= 0 or dt >= 0.5 * seconds or nb >= bx * by:
            break
        nb = int(min(bx * by, nb * min(16.0, max(2.0, seconds / max(dt, 1e-3)))))
    b_used = sc.mlt_bootstrap(nx, ny, seed=seed, n_init=n_init)
    # reference b: 16 x 625,000 paths of independent streams on `threads` host
    # threads (the oracle call releases the GIL): relative noise ~0.4 %
    # (a single path's sc has relative std ~13 on Cornell), against 1.3 % at 10^6
    from concurrent.futures import ThreadPoolExecutor
    n_ref_parts, n_ref_each = 16, 625000
    with ThreadPoolExecutor(max_workers=max(1, min(threads, n_ref_parts))) as ex:
        parts = list(ex.map(lambda k: sc.mlt_bootstrap(nx, ny, seed=(seed ^ 0x5EEDB00F) + 7919 * k,
                                                       n_init=n_ref_each), range(n_ref_parts)))
    b_ref = float(np.mean(parts))
    bf = b_ref / b_used
    ref = 0.5 * (h1 + h2)
    rmse = float(np.sqrt(np.mean((g - ref) ** 2)))
    gc = g * bf
    rel = np.abs(gc - ref) / (ref + 0.01)
    rel_noise = np.abs(h1 - h2) / 2.0 / (ref + 0.01)
    return {"rmse": rmse, "rmse_b_corrected": float(np.sqrt(np.mean((gc - ref) ** 2))),
            "oracle_noise_rmse": float(np.sqrt(np.mean((h1 - h2) ** 2))) / 2.0,
            "rel_block_err_median": float(np.median(rel)), "rel_block_err_p95": float(np.percentile(rel, 95)),
            "oracle_rel_noise_median": float(np.median(rel_noise)),
            "mean_rel_err": float(g.mean() / ref.mean() - 1.0),
            "mean_rel_err_b_corrected": float(gc.mean() / ref.mean() - 1.0),
            "b_used": b_used, "b_ref": b_ref, "b_factor": bf, "n_init": n_init,
            "b_ref_paths": n_ref_parts * n_ref_each, "b_ref_rel_noise": float(np.std(parts) / np.mean(parts) / 4.0),
            "blocks": int(len(ids)), "block": block, "block_frac": round(len(ids) / (bx * by), 4),
            "oracle_spp": spp, "max_depth": MLT_MAX_PATH, "seconds": round(dt, 1),
            "tolerance": {"rel_block_err_median": 0.05, "mean_rel_err_b_corrected": 0.02}}


def roofline(integrator, key, world, res, V, T, shared_device=False):
    """Roofline of the dominant kernel (the megakernel) for this config.

    The bound follows where the scene lives (DESIGN.md §7 "Roofline"):
    * scene in LDS (Cornell, 5 KiB) or a cache-resident list world (veach,
      ~20 KiB, read through L1/L2): the kernel issues divergent VALU work;
      HBM carries only the per-(chunk, slot) partial sums.  bound "valu":
      achieved = VALU issue slots per launch (PMC SQ_INSTS_VALU per ray, fp64
      FMA/ADD/MUL counted twice and fp64 transcendentals four times when the
      kernel computes in fp64 -- tools/roofline_pmc.py valu_issue_per_ray --
      x rays per launch) / launch time, peak = 1228.8 G fp32 wave-slots/s.
    * scene in HBM (cornell_1m, ~150 MB): bound "hbm": achieved = HBM bytes per
      launch from the PMC passes (2 x FETCH_SIZE + WRITE_SIZE per ray, the
      gfx950 correction of MI355X_MICROARCH.md) x rays per launch / launch time.
    The per-ray PMC figures come from profiles/roofline_pmc.json (made by
    tools/roofline_pmc.py from the rocprofv3 CSVs named there); the launch time
    and ray count are this run's.  The SURVEY §8(d) algorithmic bytes
    (B_ray = 32 V + 48 T + 32 on the reference's tree) are reported beside it."""
    launch_s = res["avg_kernel_ms"] * 1e-3
    rays = res["rays_per_launch"]
    pmc = load_profile("roofline_pmc.json", f"{integrator}:{key}" + (":fp64" if res.get("fp64") else ""))
    valu_bound = res["scene_in_lds"] or res["scene_bytes"] <= L2_XCD_BYTES   # LDS or L2-resident scene
    out = {"kernel": "mlt_megakernel" if integrator == "pssmlt" else "path_megakernel",
           "rays_per_launch": int(rays), "avg_launch_ms": round(res["avg_kernel_ms"], 3),
           "scene_residency": "lds" if res["scene_in_lds"] else ("l2" if valu_bound else "hbm"),
           "scene_bytes": int(res["scene_bytes"]), "launch": res["launch"]}
    algo = None
    if V is not None:
        b_ray = NODE_BYTES * V + TRI_BYTES * T + RAY_BYTES
        algo = rays * b_ray / launch_s / 1e9
        out.update({"algorithmic_bytes_per_ray": round(b_ray, 1), "V_node": round(V, 3), "T_tri": round(T, 3),
                    "algorithmic_GBps": round(algo, 1)})
    if pmc is not None:
        out["pmc_source"] = pmc.get("source")
        if pmc.get("valu_lane_util") is not None:
            out["valu_lane_util"] = round(pmc["valu_lane_util"], 4)
        hbm = pmc.get("hbm_bytes_per_ray")
        hbm_gbs = rays * hbm / launch_s / 1e9 if hbm is not None else None
        issue = pmc.get("valu_issue_per_ray", pmc.get("valu_insts_per_ray"))
        if pmc.get("l2_hit_rate") is not None:
            out["l2_hit_rate"] = round(pmc["l2_hit_rate"], 4)
        if pmc.get("write_bytes_per_ray") is not None and integrator != "pssmlt":
            # WRITE_SIZE per launch (scratch spills included) against the launch's algorithmic
            # output: one 12-B (chunk, slot) partial sum per work item
            out["written_bytes_per_launch"] = int(rays * pmc["write_bytes_per_ray"])
            out["output_bytes_per_launch"] = int(res.get("work_items", 0)) * 12
        if valu_bound and issue is not None:
            ach = rays * issue / launch_s / 1e9
            out.update({"bound": "valu", "achieved": round(ach, 1), "peak": VALU_PEAK_GINST, "unit": "Ginst/s",
                        "frac": round(ach / VALU_PEAK_GINST, 4),
                        "traffic": None if hbm is None else int(rays * hbm),
                        "hbm_GBps": None if hbm_gbs is None else round(hbm_gbs, 1),
                        "lds_frac": None if algo is None else round(algo / LDS_PEAK_GBS, 4)})
        elif hbm is not None:
            # FETCH_SIZE counts L2 misses; on gfx950 those include Infinity-Cache hits
            # (MI355X_MICROARCH.md), and cornell_1m's 99 MB scene fits the 256 MB
            # Infinity Cache: the counted bytes are an upper bound on HBM bytes, and
            # the kernel is latency-bound (wait_frac), not bandwidth-bound
            out.update({"bound": "hbm", "achieved": round(hbm_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(hbm_gbs / HBM_PEAK_GBS, 4), "traffic": int(rays * hbm),
                        "counts_infinity_cache_hits": True,
                        "traffic_basis": "2 x FETCH_SIZE + WRITE_SIZE: L2-miss bytes, served by the Infinity "
                                         "Cache or HBM (the counters do not split them)",
                        "algorithmic_over_traffic": None if algo is None else round(algo / hbm_gbs, 3)})
            if issue is not None:
                out["valu_issue_frac"] = round(rays * issue / launch_s / 1e9 / VALU_PEAK_GINST, 4)
        if pmc.get("wait_frac") is not None:
            # SQ_WAIT_ANY / SQ_WAVE_CYCLES: share of wave cycles spent in s_waitcnt
            out["wait_frac"] = round(pmc["wait_frac"], 4)
        if pmc.get("clock_ghz"):
            # the clock the chip ran this kernel at (GRBM_GUI_ACTIVE, profiled launch): the
            # VALU peak above is priced at 2.4 GHz; at the running clock the issue rate is
            # the same fraction of a lower peak (MI355X_MICROARCH.md "DVFS give-back")
            ck = pmc["clock_ghz"]
            out["clock_ghz"] = round(ck, 3)
            vf = out.get("frac") if out.get("bound") == "valu" else out.get("valu_issue_frac")
            if vf is not None:
                out["valu_issue_frac_at_clock"] = round(vf * VALU_PEAK_CLOCK_GHZ / ck, 4)
    if shared_device and out.get("frac") is not None:
        # ranks sharing one device (gloo rehearsal): a rank's launch time is not
        # the time of a launch that has the chip, so no fraction of its peak
        for k in ("achieved", "frac", "valu_issue_frac", "lds_frac", "valu_issue_frac_at_clock"):   # chip peaks
            if k in out:
                out[k] = None
        out["basis"] = "ranks share one device (rehearsal): no roofline"
    if "bound" not in out:
        # no counter profile for this config: no roofline.  The algorithmic bytes
        # (algorithmic_GBps above) are not one: L1 / L2 / the Infinity Cache / LDS
        # serve most node reads, so priced against HBM they exceed the peak.
        out.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None,
                    "traffic": None, "basis": "no PMC profile for this config (tools/roofline_pmc.py)"})
    return out


class Runner:
    """Per-process GPU state: the rank, the device, the collectives."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        n_dev = torch.cuda.device_count()
        err = check_world(args.gpus, self.world, args.backend, n_dev)
        if err:
            log(f"bench: {err}")
            sys.exit(2)
        self.gloo = args.backend == "gloo"
        # ranks sharing one device (a gloo rehearsal on a smaller box): the
        # timings are real, but each rank has only part of the chip, so no
        # roofline fraction is reported
        self.shared_device = self.world > n_dev
        if self.gloo:
            local = local % n_dev
        if self.world > 1:
            torch.cuda.set_device(local)
            if self.gloo:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        self.local = local
        self.dev = torch.device("cuda", local)
        import first_raytracer_amd as frt
        self.frt = frt
        self.ctx = frt.Context(local)

    def all_reduce(self, t, op=None):
        """RCCL on device tensors; the gloo rehearsal stages through the host."""
        kw = {} if op is None else {"op": op}
        if self.gloo:
            h = t.cpu()
            self.dist.all_reduce(h, **kw)
            t.copy_(h)
        else:
            self.dist.all_reduce(t, **kw)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def gather_ranks(self, x):
        """Every rank's float x, as a list on every rank (one all-reduce of a
        world-sized vector; per-rank timings for the line at N > 1)."""
        torch = self.torch
        v = torch.zeros(self.world, dtype=torch.float64, device=self.dev)
        v[self.rank] = float(x)
        if self.world > 1:
            self.all_reduce(v)
        return [float(t) for t in v.cpu()]

    def measure(self, args, scene, spp, steps, warmup, bvh_arg, integrator=None, precision=None, env=None):
        """Build + upload `scene`, then W warmup and K timed frames (barrier +
        synchronize on both sides, max over ranks).  `integrator`, `precision`
        and `env` default to the command line's (the configuration blocks pass
        their own)."""
        torch, frt = self.torch, self.frt
        integrator = integrator or args.integrator
        precision = precision or args.precision
        nx, ny = (int(x) for x in args.res.lower().split("x"))
        workdir = tempfile.gettempdir()   # the generated 1M-triangle OBJ (33 MB) stays out of gpurun_out/
        kind, obj, scene_name = scene_spec(scene, workdir, tag=f"_r{self.rank}")
        t0 = time.perf_counter()
        gpu_build_ms = None
        bvh = bvh_arg if kind == "cornell_box_obj" else "host"   # veach: list world, no BVH
        if bvh in ("gpu", "ploc", "lbvh", "sah"):    # OBJ load only; the BVH is built below
            hs = frt.HostScene.from_spec({"objects": [{"obj": obj, "geo": True}], "camera": frt.CORNELL_CAMERA,
                                          "world": "list"}, nx / ny)
        else:
            hs = frt.HostScene(kind, obj, nx / ny)   # OBJ load + reference-topology BVH build (host)
        if env is None and integrator == "ao":
            env = (1.0, 1.0, 1.0)                    # the scenes' black environment would make every AO sample 0
        if env is not None:
            hs.set_env(env)
        integ = {"path": frt.FRT_INTEGRATOR_PATH, "ao": frt.FRT_INTEGRATOR_AO,
                 "normals": frt.FRT_INTEGRATOR_NORMALS}.get(integrator, frt.FRT_INTEGRATOR_PSSMLT)
        ctx = self.ctx
        ctx.set_precision(precision)                 # read by the upload below (fp64 records) and the renders
        if bvh == "sah":
            hs.build_bvh_sah()                       # binned SAH on the host (in host_build_s)
        if bvh in ("gpu", "ploc", "lbvh"):
            algo = "gsah" if bvh == "gpu" else bvh
            hs.build_bvh_gpu(ctx, algo)              # warm-up build (kernels load on first use)
            tg = time.perf_counter()
            gpu_build_ms = hs.build_bvh_gpu(ctx, algo)   # binned SAH / PLOC / Karras on the device (frt_lbvh.hip)
            t0 += time.perf_counter() - tg           # count one build in host_build_s
        t1 = time.perf_counter()
        ctx.upload(hs)                               # flatten + leaf collapse + BVH4Q + copy to HBM
        t2 = time.perf_counter()
        world, rank = self.world, self.rank
        if integrator == "pssmlt":
            # chains shard over ranks (chain c -> rank c mod N); splat films are summed
            params = frt.RenderParams.pssmlt(nx, ny, spp, args.chains, seed=args.seed,
                                             shard_index=rank, shard_count=world)
            mlt_film = torch.zeros(nx * ny * 3, dtype=torch.float32, device=self.dev)
        else:
            params = frt.RenderParams.make(nx, ny, spp, seed=args.seed, tile_size=args.tile,
                                           shard_index=rank, shard_count=world, integrator=integ)
            from first_raytracer_amd.dist import TileGather
            tgather = TileGather(nx, ny, args.tile, world, rank, self.dev, stage_cpu=self.gloo)
        stream = torch.cuda.current_stream(self.dev)
        ev = []                                      # (start, end) events around each timed step's collective

        def step(timed=False):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if integrator == "pssmlt":
                st = ctx.render_device(params, mlt_film.data_ptr(), stream.cuda_stream)
                if timed:
                    e0.record(stream)
                if world > 1:
                    self.all_reduce(mlt_film)        # RCCL sum of the per-rank splat films
            else:
                st = ctx.render_device(params, tgather.my_slots.data_ptr(), stream.cuda_stream)
                if timed:
                    e0.record(stream)
                tgather.gather()   # RCCL gather of the tile slots to rank 0, which scatters them into its film
            if timed:
                e1.record(stream)
                ev.append((e0, e1))
            return st

        for _ in range(warmup):
            step()
        torch.cuda.synchronize(self.dev)
        self.barrier()
        t_start = time.perf_counter()
        rays = 0
        kernel_ms = []
        last = None
        for k in range(steps):
            st = step(timed=True)
            rays += st.rays
            kernel_ms.append(st.kernel_ms)
            last = st
            log(f"rank {rank} {scene} {integrator} step {k}: {st.rays / 1e9:.3f} Grays, kernel {st.kernel_ms:.1f} ms")
        torch.cuda.synchronize(self.dev)
        self.barrier()
        elapsed = time.perf_counter() - t_start
        my_elapsed = elapsed
        gather_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if ev else 0.0
        per_rank = None
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.dev)
            self.all_reduce(t, op=self.dist.ReduceOp.MAX)
            elapsed = float(t.item())
            r = torch.tensor([float(rays)], dtype=torch.float64, device=self.dev)
            self.all_reduce(r, op=self.dist.ReduceOp.SUM)
            rays = int(r.item())
            per_rank = {"kernel_ms": [round(x, 3) for x in self.gather_ranks(np.mean(kernel_ms))],
                        "collective_ms": [round(x, 3) for x in self.gather_ranks(gather_ms)],
                        "elapsed_s": [round(x, 4) for x in self.gather_ranks(my_elapsed)],
                        "rays_per_step": [int(x) for x in self.gather_ranks(last.rays)]}
        film = None
        if rank == 0:
            film = (mlt_film if integrator == "pssmlt" else tgather.film).cpu().numpy()
        return {
            "scene": scene, "scene_name": scene_name, "kind": kind, "obj": obj, "nx": nx, "ny": ny, "spp": spp,
            "steps": steps, "warmup": warmup, "elapsed": elapsed, "rays": rays, "value": rays / elapsed / 1e6,
            "integrator": integrator, "integ": integ, "env": env, "bvh": bvh, "gpu_build_ms": gpu_build_ms,
            "setup_s": t2 - t0, "build_s": t1 - t0, "upload_s": t2 - t1,
            "avg_kernel_ms": float(np.mean(kernel_ms)), "rays_per_launch": last.rays,
            "collective_ms": gather_ms, "per_rank": per_rank,
            "samples_per_launch": last.samples, "work_items": int(last.work_items), "scene_in_lds": last.scene_in_lds,
            "scene_bytes": last.scene_bytes,
            "launch": {"waves_cap": int(last.waves_cap), "stack": int(last.stack_entries),
                       "bvh_depth": int(last.bvh_depth)},
            "fp64": bool(last.fp64),
            "film": film,
        }


BVH_NAMES = {"gpu": "binned SAH (GPU, 32 bins per axis)", "ploc": "PLOC (GPU)", "lbvh": "linear BVH (GPU)",
             "sah": "binned SAH (host, 32 bins per axis)",
             "host": "create_bvh (reference topology)"}


def parse_env(text):
    return tuple(float(x) for x in text.split(",")) if text else None


def count_devices_no_hip():
    """GPUs this process may use, counted through amdsmi (torch's own amdsmi
    count, which honours the *_VISIBLE_DEVICES variables) WITHOUT initialising
    HIP: the parent of `bench.py --gpus N` starts N rank processes and must
    not have touched the GPU (torch.cuda.device_count()
    falls back to hipGetDeviceCount when amdsmi fails).  None when amdsmi
    cannot count."""
    import torch
    try:
        n = int(torch.cuda._device_count_amdsmi())
    except Exception:           # no amdsmi, or a torch without that helper
        return None
    return n if n >= 0 else None


def launch_ranks(args, argv, count=count_devices_no_hip):
    """`bench.py --gpus N` without a launcher: check the device count with
    amdsmi only, assert that HIP is still uninitialised, then start the N
    ranks (spawn_ranks).  Returns the exit code (2 = refused)."""
    n_dev = count()
    if n_dev is None:
        log("bench: cannot count GPUs without initialising HIP (amdsmi unavailable); "
            "start the ranks with torchrun instead")
        return 2
    err = check_world(args.gpus, args.gpus, args.backend, n_dev)
    if err:
        log(f"bench: {err}")
        return 2
    import torch
    assert not torch.cuda.is_initialized(), "HIP initialised in the launcher before the ranks start"
    return spawn_ranks(args.gpus, argv)


def cpu_line(cpu, threads, nproc, sample):
    return {"value": round(cpu["mrays"], 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "host_nproc": nproc, "sample": sample}


def path_rmse_detail(cpu, nx, ny):
    return {"pixels": cpu["rmse_pixels"], "pixel_frac": round(cpu["rmse_pixels"] / (nx * ny), 4),
            "diverged_pixels": cpu["diverged_pixels"], "rmse_converged": cpu["rmse_converged"],
            "diverged_threshold": 1e-3, "extra_oracle_seconds": cpu["rmse_extra_seconds"]}


def block_common(r, world):
    """The fields every configuration block shares with the headline line."""
    out = {"value": round(r["value"], 1), "unit": "Mrays/s", "n_gpus": world, "steps": r["steps"],
           "warmup": r["warmup"], "ms_per_step": round(r["elapsed"] / r["steps"] * 1e3, 2),
           "dtype": "f64" if r["fp64"] else "f32", "rays_per_step": int(r["rays"] // r["steps"]),
           "bvh": BVH_NAMES[r["bvh"]], "setup_s": round(r["setup_s"], 2),
           "collective_ms": round(r["collective_ms"], 3),
           "image_mean": [round(float(x), 6) for x in r["film"].reshape(-1, 3).mean(0)]}
    if r["per_rank"] is not None:
        out["per_rank"] = r["per_rank"]
    return out


def first_ray_estimate(cpu_mrays):
    """cpu_baseline / (the port's 1-thread Mrays/s on C1 over first_ray's), or None."""
    rec = None
    for rnd in ("r06", "r03"):
        path = os.path.join(ROOT, "profiles", rnd, "cpu_ratio.json")
        if os.path.exists(path):
            with open(path) as f:
                rec = json.load(f)
            break
    if not rec or not rec.get("ratio_port_over_first_ray"):
        return None
    ratio = rec["ratio_port_over_first_ray"]
    return {"value": round(cpu_mrays / ratio, 3), "unit": "Mrays/s", "ratio_port_over_first_ray": ratio,
            "oracle_mrays_1thread_median": rec.get("oracle_mrays_1thread"),
            "basis": ("cpu_baseline / ratio; ratio = the oracle's 1-thread Mrays/s on C1 (CornellBox 256x256x16, "
                      f"median of {len(rec.get('oracle_runs', []))} runs, {rec.get('measured', 'round 3')}) over "
                      "first_ray's 2.14 Mrays/s (SURVEY.md section 6, the survey's probe build in the same "
                      "container; tools/cpu_ratio.py). first_ray itself does not run here: path.cpp needs "
                      "cpp-taskflow and GLFW, which this image lacks, and the task rules forbid building the "
                      "reference against stand-ins; nothing of the reference travels to the GPU box. Assumes "
                      "first_ray scales like the port; as written its shared ray counters scale negatively "
                      "(1.25 Mrays/s on 8 threads, SURVEY section 6)")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell", choices=["cornell", "cornell_1m", "veach", "sphere"])
    ap.add_argument("--res", default="1920x1080")
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--bvh", default="gpu", choices=["gpu", "sah", "host", "ploc", "lbvh"],
                    help="gpu (default): binned SAH tree built on the GPU (frt_lbvh.hip); sah: the same rule on "
                         "the host; host: the reference's create_bvh topology (exact-t ties resolved in its "
                         "order); ploc / lbvh: PLOC clustering / the Karras linear BVH on the GPU. List-world "
                         "scenes (veach) ignore it")
    ap.add_argument("--cpu-pixels", type=int, default=0, help="pixels in the CPU-baseline sample (0: calibrated)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target CPU-baseline duration when calibrated")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every CPU this process may use (host_cpus)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--north-star", default="auto", choices=["auto", "on", "off"],
                    help="auto: with the default config (cornell, path) also run cornell_1m 1080p/512spp")
    ap.add_argument("--ns-steps", type=int, default=3, help="timed frames of the north-star run")
    ap.add_argument("--ns-pixels", type=int, default=32768, help="oracle pixel sample for the north-star RMSE")
    ap.add_argument("--configs", default="auto", choices=["auto", "on", "off"],
                    help="auto: with the default config also run BASELINE's C3 (veach_mi 1080p 1024 spp) and C5 "
                         "(PSS-MLT on CornellBox 1080p, 512 mutations/pixel) as blocks \"c3\" and \"c5\"")
    ap.add_argument("--cfg-steps", type=int, default=3, help="timed frames of each configuration block")
    ap.add_argument("--cfg-cpu-seconds", type=float, default=10.0,
                    help="target oracle duration of each configuration block's CPU baseline / parity")
    ap.add_argument("--c3-min-pixels", type=int, default=16384, help="oracle pixels of the C3 block's RMSE (at least)")
    ap.add_argument("--rmse-min-frac", type=float, default=0.25,
                    help="the calibrated CPU sample covers at least this fraction of the frame's pixels")
    ap.add_argument("--precision", default="auto", choices=["auto", "fp32", "fp64"],
                    help="frt_set_precision: auto = fp64 for list worlds (veach), fp32 for BVH worlds")
    ap.add_argument("--pfm", default="", help="write the rank-0 film here")
    ap.add_argument("--integrator", default="path", choices=["path", "pssmlt", "ao", "normals"],
                    help="pssmlt: C5 config, --spp = mutations per pixel; ao (ao.cpp), normals (debug_renderer.h)")
    ap.add_argument("--env", default="", help="constant environment r,g,b (default: the scene's; 1,1,1 for ao)")
    ap.add_argument("--chains", type=int, default=1 << 18, help="PSS-MLT chains (all ranks)")
    ap.add_argument("--mlt-shards", type=int, default=0,
                    help="PSS-MLT path-exact parity on shard (0, K) of the chains; 0: K calibrated to "
                         "--cpu-seconds, 1: every chain (the full-frame RMSE, no estimate)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N-rank path with host-staged collectives (e.g. ranks sharing one GPU)")
    ap.add_argument("--rmse-pixels-multi", type=int, default=32768,
                    help="N > 1: oracle pixel sample for rank 0's RMSE (no CPU timing at N > 1)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here, before anything touches the GPU
        sys.exit(launch_ranks(args, sys.argv[1:]))

    R = Runner(args)
    world, rank = R.world, R.rank
    threads = args.cpu_threads or host_cpus()
    timed_cpu = world == 1          # the CPU baseline is timed at N = 1 only; the RMSE is computed at every N
    nproc = os.cpu_count()
    res = R.measure(args, args.scene, args.spp, args.steps, args.warmup, args.bvh, env=parse_env(args.env))
    mlt_cpu = None
    if args.integrator == "pssmlt" and rank == 0 and not args.no_cpu_baseline:
        # the path-exact parity renders shard chains on R.ctx: it runs now, while R.ctx
        # still holds this line's scene (not after the north-star upload)
        with Heartbeat("PSS-MLT parity (oracle)"):
            mlt_cpu = cpu_baseline_mlt(R.ctx, res, args.spp, args.chains, args.seed, threads, args.cpu_seconds,
                                       shards=args.mlt_shards)
    default = (args.scene == "cornell" and args.integrator == "path" and args.res == "1920x1080"
               and args.spp == 512)
    do_ns = args.north_star == "on" or (args.north_star == "auto" and default)
    ns = R.measure(args, "cornell_1m", 512, args.ns_steps, 1, args.bvh, integrator="path", precision="auto") \
        if do_ns else None
    do_cfg = args.configs == "on" or (args.configs == "auto" and default)
    c3 = c5 = c5_cpu = None
    if do_cfg:
        # BASELINE configs[2] and [4]: the driver's default run measures them too
        c3 = R.measure(args, "veach", 1024, args.cfg_steps, 1, args.bvh, integrator="path", precision="auto")
        c5 = R.measure(args, "cornell", 512, args.cfg_steps, 1, args.bvh, integrator="pssmlt", precision="auto")
        if rank == 0 and not args.no_cpu_baseline:
            with Heartbeat("C5 parity (oracle)"):
                c5_cpu = cpu_baseline_mlt(R.ctx, c5, 512, args.chains, args.seed, threads, args.cfg_cpu_seconds)

    beat = Heartbeat("oracle RMSE / CPU baseline") if rank == 0 else None
    if beat is not None:
        beat.__enter__()
    if rank == 0:
        nx, ny = res["nx"], res["ny"]
        key = f"{args.scene}:{nx}x{ny}"
        cpu = None
        if not args.no_cpu_baseline:
            if args.integrator == "pssmlt":
                cpu = mlt_cpu
                if cpu is not None:
                    cpu["mlt_rmse"] = mlt_block_rmse(res["kind"], res["obj"], nx, ny, res["film"], threads,
                                                     args.cpu_seconds, seed=args.seed, env=res["env"])
                    # "RMSE vs CPU ref": the same chains on the oracle (path-exact up to
                    # fp32-diverged chains), as the full-frame estimate from one shard
                    cpu["rmse"] = cpu["parity"]["full_frame_rmse_est"] if cpu["parity"] else None
            elif timed_cpu:
                cpu = cpu_baseline(res["kind"], res["obj"], nx, ny, args.spp, args.seed, args.cpu_pixels, threads,
                                   res["film"], args.cpu_seconds, integrator=res["integ"], env=res["env"],
                                   min_frac=args.rmse_min_frac)
            else:
                cpu = cpu_baseline(res["kind"], res["obj"], nx, ny, args.spp, args.seed, args.rmse_pixels_multi,
                                   threads, res["film"], 0.0, integrator=res["integ"], env=res["env"])
        ts = load_profile("traversal_stats.json", key)
        V, T = (cpu["V"], cpu["T"]) if cpu is not None else (ts["V"], ts["T"]) if ts is not None else (None, None)
        li_name = {"path": "path::Li", "ao": "ao::Li", "normals": "normals_renderer::Li"}.get(args.integrator)
        sname = res["scene_name"]
        workload = {"path": f"{sname} {nx}x{ny} {args.spp}spp path+NEE+MIS",
                    "ao": f"{sname} {nx}x{ny} {args.spp}spp ambient occlusion (ao.cpp)",
                    "normals": f"{sname} {nx}x{ny} {args.spp}spp shading normals (debug_renderer.h)",
                    "pssmlt": f"{sname} {nx}x{ny} PSS-MLT {args.spp} mutations/pixel, {args.chains} chains"
                    }[args.integrator]
        film_np = res["film"]
        line = {
            "metric": METRIC, "value": round(res["value"], 1), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(res["elapsed"] / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64" if res["fp64"] else "f32", "data": "synthetic",
            "config": {"workload": workload,
                       "integrator": args.integrator, "scene": args.scene,
                       "nx": nx, "ny": ny, "spp": args.spp, "seed": args.seed, "tile": args.tile,
                       "env": res["env"], "precision": args.precision,
                       "parallelism": (f"chains-interleaved x{world} + rccl all-reduce" if args.integrator == "pssmlt"
                                       else f"tiles-interleaved x{world} + rccl gather to rank 0")},
            "rmse": None if cpu is None else cpu["rmse"],
            "rmse_detail": None if cpu is None else {
                "basis": ("rmse = full_frame_rmse_est of path_exact: the GPU's and the oracle's films of the same "
                          "chain shard (the config's own chains and mutation count), sqrt(K) x the shard-film RMSE; "
                          "statistical = 8x8-block means against the oracle's path tracer (a different estimator)"),
                "path_exact": cpu["parity"], "statistical": cpu["mlt_rmse"]} if "mlt_rmse" in cpu else
            path_rmse_detail(cpu, nx, ny),
            "mutations_per_step": int(res["samples_per_launch"]) if args.integrator == "pssmlt" else None,
            "rays_per_step": int(res["rays"] // args.steps),
            "setup_s": round(res["setup_s"], 2), "host_build_s": round(res["build_s"], 2),
            "upload_s": round(res["upload_s"], 2),
            "bvh": BVH_NAMES[res["bvh"]],
            "gpu_build_ms": None if res["gpu_build_ms"] is None else round(res["gpu_build_ms"], 3),
            "value_per_gpu": round(res["value"] / world, 1),
            "collective_ms": round(res["collective_ms"], 3),
            "image_mean": [round(float(x), 6) for x in film_np.reshape(-1, 3).mean(0)],
            "roofline": roofline(args.integrator, key, world, res, V, T, R.shared_device),
            "cpu_baseline": None if (cpu is None or not timed_cpu or (args.integrator == "pssmlt"
                                                                      and not cpu["parity"])) else cpu_line(
                cpu, threads, nproc,
                (f"{cpu['npix']} evenly spaced pixels of the same {nx}x{ny} frame at {args.spp} spp "
                 f"({cpu['rays']} rays, {cpu['seconds']:.1f} s) on {threads} threads (every CPU this "
                 f"process may use; the host reports {nproc}); fp64 C restatement of {li_name}")
                if args.integrator != "pssmlt" else
                (f"PSS-MLT {cpu['sample']} on the same {nx}x{ny} frame ({cpu['rays']} rays, "
                 f"{cpu['seconds']:.1f} s) on {threads} threads; fp64 C restatement of pssmlt.cpp")),
        }
        if res["per_rank"] is not None:
            line["per_rank"] = res["per_rank"]
        if line["cpu_baseline"] is not None:
            est = first_ray_estimate(cpu["mrays"])
            if est is not None:
                line["cpu_baseline"]["first_ray_estimate"] = est
        if ns is not None:
            nkey = f"cornell_1m:{ns['nx']}x{ns['ny']}"
            ncpu = None
            if not args.no_cpu_baseline:      # a fixed pixel sample, timed; the RMSE at every N
                ncpu = cpu_baseline(ns["kind"], ns["obj"], ns["nx"], ns["ny"], 512, args.seed, args.ns_pixels,
                                    threads, ns["film"], 0.0)
            nts = load_profile("traversal_stats.json", nkey)
            nV, nT = ((ncpu["V"], ncpu["T"]) if ncpu is not None else (nts["V"], nts["T"]) if nts is not None
                      else (None, None))
            blk = {"workload": f"{ns['scene_name']} {ns['nx']}x{ns['ny']} 512spp path+NEE+MIS"}
            blk.update(block_common(ns, world))
            blk.update({
                "target": f">= {NS_TARGET_MRAYS:.0f} Mrays/s on one MI355X",
                "target_met": bool(ns["value"] / world >= NS_TARGET_MRAYS),
                "rmse": None if ncpu is None else ncpu["rmse"],
                "rmse_detail": None if ncpu is None else {
                    "pixels": ncpu["rmse_pixels"], "diverged_pixels": ncpu["diverged_pixels"],
                    "rmse_converged": ncpu["rmse_converged"], "diverged_threshold": 1e-3,
                    "oracle_mrays": round(ncpu["mrays"], 3), "oracle_threads": threads},
                "roofline": roofline("path", nkey, world, ns, nV, nT, R.shared_device),
                "cpu_baseline": None if (ncpu is None or not timed_cpu) else cpu_line(
                    ncpu, threads, nproc,
                    f"the RMSE sample: {ncpu['npix']} evenly spaced pixels of the same frame at 512 spp "
                    f"({ncpu['rays']} rays, {ncpu['seconds']:.1f} s) on {threads} threads; fp64 C restatement "
                    f"of path::Li over the reference-topology BVH")})
            line["north_star"] = blk
        if c3 is not None:
            c3x, c3y = c3["nx"], c3["ny"]
            ccpu = None
            if not args.no_cpu_baseline:
                min_frac = min(1.0, args.c3_min_pixels / (c3x * c3y))
                if timed_cpu:
                    ccpu = cpu_baseline(c3["kind"], c3["obj"], c3x, c3y, 1024, args.seed, 0, threads, c3["film"],
                                        args.cfg_cpu_seconds, integrator=c3["integ"], min_frac=min_frac)
                else:
                    ccpu = cpu_baseline(c3["kind"], c3["obj"], c3x, c3y, 1024, args.seed, args.c3_min_pixels,
                                        threads, c3["film"], 0.0, integrator=c3["integ"])
            ckey = f"veach:{c3x}x{c3y}"
            blk = {"workload": f"{c3['scene_name']} {c3x}x{c3y} 1024spp path+NEE+MIS (BASELINE configs[2], "
                               f"list world, {'fp64' if c3['fp64'] else 'fp32'} kernel: precision auto)"}
            blk.update(block_common(c3, world))
            blk.update({
                "rmse": None if ccpu is None else ccpu["rmse"],
                "rmse_detail": None if ccpu is None else path_rmse_detail(ccpu, c3x, c3y),
                "roofline": roofline("path", ckey, world, c3, None if ccpu is None else ccpu["V"],
                                     None if ccpu is None else ccpu["T"], R.shared_device),
                "cpu_baseline": None if (ccpu is None or not timed_cpu) else cpu_line(
                    ccpu, threads, nproc,
                    f"{ccpu['npix']} evenly spaced pixels of the same frame at 1024 spp ({ccpu['rays']} rays, "
                    f"{ccpu['seconds']:.1f} s) on {threads} threads; fp64 C restatement of path::Li")})
            line["c3"] = blk
        if c5 is not None:
            par = c5_cpu["parity"] if c5_cpu is not None else None
            blk = {"workload": f"{c5['scene_name']} {c5['nx']}x{c5['ny']} PSS-MLT 512 mutations/pixel, "
                               f"{args.chains} chains (BASELINE configs[4])"}
            blk.update(block_common(c5, world))
            blk.update({
                "mutations_per_step": int(c5["samples_per_launch"]),
                "rmse": None if not par else par["full_frame_rmse_est"],
                "rmse_detail": None if c5_cpu is None else {
                    "basis": ("full_frame_rmse_est: the GPU's and the oracle's films of the same chain shard (the "
                              "config's own chains, each with the config's full mutation count), sqrt(K) x the "
                              "shard-film RMSE; a chain is path-exact when its trajectory fingerprint equals the "
                              "oracle's"),
                    "path_exact": par, "note": c5_cpu.get("note")},
                "roofline": roofline("pssmlt", f"cornell:{c5['nx']}x{c5['ny']}", world, c5,
                                     None if not par else par["oracle_counters"]["V"],
                                     None if not par else par["oracle_counters"]["T"], R.shared_device),
                "cpu_baseline": None if (not par or not timed_cpu) else cpu_line(
                    c5_cpu, threads, nproc,
                    f"PSS-MLT {c5_cpu['sample']} ({c5_cpu['rays']} rays, {c5_cpu['seconds']:.1f} s) on "
                    f"{threads} threads; fp64 C restatement of pssmlt.cpp")})
            line["c5"] = blk
        if R.gloo:
            line["config"]["parallelism"] += " (gloo host-staged rehearsal)"
        if args.pfm:
            R.frt.write_pfm(args.pfm, film_np.reshape(ny, nx, 3))
        beat.__exit__()
        print(json.dumps(line), flush=True)
    R.ctx.close()
    if world > 1:
        R.dist.destroy_process_group()


if __name__ == "__main__":
    main()
