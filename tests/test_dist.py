"""Multi-GPU path logic on CPU: tile sharding over N ranks + the all-gather /
scatter of first_raytracer_amd.dist.TileGather, world_size 2 and 3 with the
gloo backend (the GPU run uses the same code with RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, nx, ny, tile, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import first_raytracer_amd as frt
    from first_raytracer_amd.dist import TileGather
    tg = TileGather(nx, ny, tile, world, rank, torch.device("cpu"))
    # "render": slot value = 3*pixel + channel for this rank's slots
    slots = frt.shard_slots(frt.RenderParams.make(nx, ny, 1, tile_size=tile, shard_index=rank, shard_count=world))
    vals = np.zeros((tg.max_slots, 3), np.float32)
    ok = slots >= 0
    vals[:len(slots)][ok] = (3 * slots[ok, None] + np.arange(3)).astype(np.float32)
    tg.my_slots.copy_(torch.from_numpy(vals.reshape(-1)))
    film = tg.gather()
    if rank == 0:
        q.put(film.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nx,ny,tile", [(2, 96, 72, 32), (3, 100, 37, 16)])
def test_tile_gather_reassembles_frame(world, nx, ny, tile):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, nx, ny, tile, q)) for r in range(world)]
    for p in procs:
        p.start()
    film = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(film, np.arange(nx * ny * 3, dtype=np.float32))
