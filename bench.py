#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X path integrator on the BASELINE.json config
(CornellBox-Original, 1920x1080, 512 spp, path + NEE + MIS), with the image
tiles sharded over N GPUs (one process per GPU, RCCL all-gather of the tile
radiance over xGMI), plus the roofline of the path megakernel and the CPU
baseline (the fp64 C restatement, oracle/, timed on this host's cores).

One "step" = one full frame: every rank renders its tiles (tile t -> rank
t mod N) into HBM, then the per-rank slot buffers are all-gathered and rank 0
scatters them into the film.  Scene upload and BVH build happen before the
timed region.

    python bench.py [--gpus N --steps K --warmup W] [--scene cornell|cornell_1m|veach]

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec + RMSE vs CPU ref, CornellBox 1080p 512spp, 1/2/4/8 MI355X"
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
LDS_PEAK_GBS = 150000.0   # ds_read_b128 aggregate, MI355X_MICROARCH.md §LDS
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
NODE_BYTES, TRI_BYTES, RAY_BYTES = 32, 48, 32   # B_ray = 32 V + 48 T + 32


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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


def load_traversal_stats(key):
    path = os.path.join(ROOT, "profiles", "traversal_stats.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f).get(key)
    return None


def cpu_baseline(kind, obj, nx, ny, spp, seed, npix, threads, film, seconds, integrator=0, env=None):
    """The oracle (fp64 C restatement) on a bounded pixel sample of the same
    frame and RNG streams: CPU Mrays/s, reference traversal counters (for
    B_ray) and the RMSE of the GPU film on those pixels.  npix = 0: calibrate
    on growing samples (from 512 pixels) until one takes about `seconds` of CPU work."""
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
    gpu = film.reshape(-1, 3)[pix].astype(np.float64)
    rmse = float(np.sqrt(np.mean((gpu - out) ** 2)))
    # fp32 vs fp64 rounding occasionally sends one sample down another branch
    # (a silhouette, the light's edge); such a pixel differs by ~radiance/spp.
    # Reported apart so a systematic error would show in rmse_converged.
    dev = np.abs(gpu - out).max(axis=1)
    bad = dev > 1e-3
    rmse_conv = float(np.sqrt(np.mean((gpu[~bad] - out[~bad]) ** 2))) if (~bad).any() else None
    return {
        "mrays": rays / dt / 1e6, "seconds": dt, "rays": rays, "npix": len(pix),
        "V": cnt.node_visits / rays, "T": (cnt.tri_tests + cnt.sphere_tests) / rays,
        "rays_per_sample": rays / cnt.samples, "rmse": rmse,
        "diverged_pixels": int(bad.sum()), "rmse_converged": rmse_conv,
    }


def cpu_baseline_mlt(kind, obj, nx, ny, seed, threads, seconds):
    """The oracle's PSS-MLT on a bounded sample of the same frame: chains x 512
    mutations, the chain count grown (from 256) until a run takes about
    `seconds` of CPU work."""
    import oracle
    sc = oracle.OracleScene(kind, obj, nx / ny)
    steps = 512

    def run(chains):
        t0 = time.perf_counter()
        _, _, cnt = sc.mlt_render(nx, ny, chains, steps, seed=seed, n_init=10000, nthreads=threads)
        return cnt, time.perf_counter() - t0

    chains = 256
    while True:                             # grow the sample until it takes >= seconds/2
        cnt, dt = run(chains)
        if dt >= 0.5 * seconds or chains >= 1 << 20:
            break
        chains = int(min(1 << 20, chains * min(16.0, max(2.0, seconds / max(dt, 1e-3)))))
    return {"mrays": cnt.rays / dt / 1e6, "seconds": dt, "rays": cnt.rays, "npix": 0,
            "V": cnt.node_visits / cnt.rays, "T": (cnt.tri_tests + cnt.sphere_tests) / cnt.rays,
            "rmse": None, "sample": f"{chains} chains x {steps} mutations"}


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
    ap.add_argument("--bvh", default="sah", choices=["host", "gpu", "sah"],
                    help="sah (default): binned SAH tree (host); host: the reference's create_bvh topology "
                         "(exact-t ties resolved in its order); gpu: linear BVH built on the GPU (frt_lbvh.hip). "
                         "List-world scenes (veach) ignore it")
    ap.add_argument("--cpu-pixels", type=int, default=0, help="pixels in the CPU-baseline sample (0: calibrated)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline duration when calibrated")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pfm", default="", help="write the rank-0 film here")
    ap.add_argument("--integrator", default="path", choices=["path", "pssmlt", "ao", "normals"],
                    help="pssmlt: C5 config, --spp = mutations per pixel; ao (ao.cpp), normals (debug_renderer.h)")
    ap.add_argument("--env", default="", help="constant environment r,g,b (default: the scene's; 1,1,1 for ao)")
    ap.add_argument("--chains", type=int, default=1 << 18, help="PSS-MLT chains (all ranks)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N-rank path with host-staged collectives (e.g. ranks sharing one GPU)")
    args = ap.parse_args()
    nx, ny = (int(x) for x in args.res.lower().split("x"))

    import torch
    import torch.distributed as dist

    import first_raytracer_amd as frt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    gloo = args.backend == "gloo"
    if gloo:
        local = local % torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    def all_reduce(t, op=None):
        """RCCL on device tensors; the gloo rehearsal stages through the host."""
        kw = {} if op is None else {"op": op}
        if gloo:
            h = t.cpu()
            dist.all_reduce(h, **kw)
            t.copy_(h)
        else:
            dist.all_reduce(t, **kw)

    workdir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else "/tmp"
    kind, obj, scene_name = scene_spec(args.scene, workdir, tag=f"_r{rank}")
    t0 = time.perf_counter()
    gpu_build_ms = None
    bvh = args.bvh if kind == "cornell_box_obj" else "host"   # veach: list world, no BVH
    if bvh in ("gpu", "sah"):                    # OBJ load only; the BVH is built below
        hs = frt.HostScene.from_spec({"objects": [{"obj": obj, "geo": True}], "camera": frt.CORNELL_CAMERA,
                                      "world": "list"}, nx / ny)
    else:
        hs = frt.HostScene(kind, obj, nx / ny)   # OBJ load + reference-topology BVH build (host)
    env = None
    if args.env:
        env = tuple(float(x) for x in args.env.split(","))
    elif args.integrator == "ao":
        env = (1.0, 1.0, 1.0)                    # the scenes' black environment would make every AO sample 0
    if env is not None:
        hs.set_env(env)
    integ = {"path": frt.FRT_INTEGRATOR_PATH, "ao": frt.FRT_INTEGRATOR_AO,
             "normals": frt.FRT_INTEGRATOR_NORMALS}.get(args.integrator, frt.FRT_INTEGRATOR_PSSMLT)
    ctx = frt.Context(local)
    if bvh == "sah":
        hs.build_bvh_sah()                       # binned SAH on the host (in host_build_s)
    if bvh == "gpu":
        hs.build_bvh_gpu(ctx)                    # warm-up build (hipcub kernels load on first use)
        tg = time.perf_counter()
        gpu_build_ms = hs.build_bvh_gpu(ctx)     # Morton + radix sort + Karras + refit (frt_lbvh.hip)
        t0 += time.perf_counter() - tg           # count one build in host_build_s
    t1 = time.perf_counter()
    ctx.upload(hs)                               # flatten + leaf collapse + BVH4Q + copy to HBM
    t2 = time.perf_counter()
    build_s, upload_s, setup_s = t1 - t0, t2 - t1, t2 - t0

    if args.integrator == "pssmlt":
        # chains shard over ranks (chain c -> rank c mod N); splat films are summed
        params = frt.RenderParams.pssmlt(nx, ny, args.spp, args.chains, seed=args.seed,
                                         shard_index=rank, shard_count=world)
        mlt_film = torch.zeros(nx * ny * 3, dtype=torch.float32, device=dev)

        class _Film:
            film = mlt_film
        tg = _Film()
    else:
        params = frt.RenderParams.make(nx, ny, args.spp, seed=args.seed, tile_size=args.tile,
                                       shard_index=rank, shard_count=world, integrator=integ)
        from first_raytracer_amd.dist import TileGather
        tg = TileGather(nx, ny, args.tile, world, rank, dev, stage_cpu=gloo)
    stream = torch.cuda.current_stream(dev)

    def step():
        if args.integrator == "pssmlt":
            st = ctx.render_device(params, mlt_film.data_ptr(), stream.cuda_stream)
            if world > 1:
                all_reduce(mlt_film)        # RCCL sum of the per-rank splat films
            return st
        st = ctx.render_device(params, tg.my_slots.data_ptr(), stream.cuda_stream)
        tg.gather()       # RCCL all-gather of the tile slots, rank 0 scatters into its film
        return st

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_start = time.perf_counter()
    rays = 0
    kernel_ms = []
    last = None
    for k in range(args.steps):
        st = step()
        rays += st.rays
        kernel_ms.append(st.kernel_ms)
        last = st
        log(f"rank {rank} step {k}: {st.rays / 1e9:.3f} Grays, kernel {st.kernel_ms:.1f} ms")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([float(rays)], dtype=torch.float64, device=dev)
        all_reduce(r, op=dist.ReduceOp.SUM)
        rays = int(r.item())

    if rank == 0:
        value = rays / elapsed / 1e6
        film_np = tg.film.cpu().numpy()
        key = f"{args.scene}:{nx}x{ny}"
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            if args.integrator == "pssmlt":
                cpu = cpu_baseline_mlt(kind, obj, nx, ny, args.seed, threads, args.cpu_seconds)
            else:
                cpu = cpu_baseline(kind, obj, nx, ny, args.spp, args.seed, args.cpu_pixels, threads, film_np,
                                   args.cpu_seconds, integrator=integ, env=env)
            cpu["threads"] = threads
        ts = load_traversal_stats(key)
        if cpu is not None:
            V, T = cpu["V"], cpu["T"]
        elif ts is not None:
            V, T = ts["V"], ts["T"]
        else:
            V = T = None
        avg_kernel_s = float(np.mean(kernel_ms)) * 1e-3
        rays_per_launch = last.rays
        roofline = None
        if V is not None:
            b_ray = NODE_BYTES * V + TRI_BYTES * T + RAY_BYTES
            achieved = rays_per_launch * b_ray / avg_kernel_s / 1e9
            traffic = None
            pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                with open(pmc) as f:
                    traffic = json.load(f).get(f"{args.integrator}:{key}:n{world}")
            roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "kernel": "mlt_megakernel" if args.integrator == "pssmlt" else "path_megakernel",
                        "bytes_per_ray": round(b_ray, 1),
                        "V_node": round(V, 3), "T_tri": round(T, 3), "rays_per_launch": int(rays_per_launch),
                        "avg_launch_ms": round(avg_kernel_s * 1e3, 3),
                        # where the algorithmic bytes are served from: an LDS-resident scene is not
                        # HBM-bound (frac can exceed 1); its LDS-read peak is ~150 TB/s (MI355X_MICROARCH.md §LDS)
                        "scene_residency": "lds" if last.scene_in_lds else "hbm",
                        "scene_bytes": int(last.scene_bytes),
                        "lds_frac": round(achieved / LDS_PEAK_GBS, 4) if last.scene_in_lds else None,
                        "launch": {"waves_cap": int(last.waves_cap), "stack": int(last.stack_entries),
                                   "bvh_depth": int(last.bvh_depth)}}
        li_name = {"path": "path::Li", "ao": "ao::Li", "normals": "normals_renderer::Li"}.get(args.integrator)
        workload = {"path": f"{scene_name} {nx}x{ny} {args.spp}spp path+NEE+MIS",
                    "ao": f"{scene_name} {nx}x{ny} {args.spp}spp ambient occlusion (ao.cpp)",
                    "normals": f"{scene_name} {nx}x{ny} {args.spp}spp shading normals (debug_renderer.h)",
                    "pssmlt": f"{scene_name} {nx}x{ny} PSS-MLT {args.spp} mutations/pixel, {args.chains} chains"
                    }[args.integrator]
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": workload,
                       "integrator": args.integrator, "scene": args.scene,
                       "nx": nx, "ny": ny, "spp": args.spp, "seed": args.seed, "tile": args.tile,
                       "env": env,
                       "parallelism": (f"chains-interleaved x{world} + rccl all-reduce" if args.integrator == "pssmlt"
                                       else f"tiles-interleaved x{world} + rccl all-gather")},
            "rmse": None if cpu is None else cpu["rmse"],
            "rmse_detail": None if cpu is None or "diverged_pixels" not in cpu else {
                "pixels": cpu["npix"], "diverged_pixels": cpu["diverged_pixels"],
                "rmse_converged": cpu["rmse_converged"], "diverged_threshold": 1e-3},
            "mutations_per_step": int(last.samples) if args.integrator == "pssmlt" else None,
            "rays_per_step": int(rays // args.steps),
            "setup_s": round(setup_s, 2), "host_build_s": round(build_s, 2), "upload_s": round(upload_s, 2),
            "bvh": {"gpu": "gpu-lbvh", "sah": "binned SAH (host)"}.get(bvh, "create_bvh (reference topology)"),
            "gpu_build_ms": None if gpu_build_ms is None else round(gpu_build_ms, 3),
            "value_per_gpu": round(value / world, 1),
            "image_mean": [round(float(x), 6) for x in film_np.reshape(-1, 3).mean(0)],
            "roofline": roofline,
            "cpu_baseline": None if cpu is None else {
                "value": round(cpu["mrays"], 3), "unit": "Mrays/s", "cores": cpu["threads"], "kind": "port",
                "sample": (f"{cpu['npix']} evenly spaced pixels of the same {nx}x{ny} frame at {args.spp} spp "
                           f"({cpu['rays']} rays, {cpu['seconds']:.1f} s); fp64 C restatement of {li_name}")
                if args.integrator != "pssmlt" else
                          (f"PSS-MLT {cpu['sample']} on the same {nx}x{ny} frame ({cpu['rays']} rays, "
                           f"{cpu['seconds']:.1f} s); fp64 C restatement of pssmlt.cpp")},
        }
        if gloo:
            line["config"]["parallelism"] += " (gloo host-staged rehearsal)"
        if args.pfm:
            frt.write_pfm(args.pfm, film_np.reshape(ny, nx, 3))
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
