#!/usr/bin/env python3
"""One-GPU check of the collectives bench.py uses at N > 1 over the "nccl"
(RCCL) backend: a world of one rank on cuda:0 runs dist.gather into views of
one device buffer (TileGather's call), all_reduce and barrier, and checks the
results.  A world of one exercises the torch/RCCL call path and argument
handling that the 8-GPU driver run depends on; it cannot measure xGMI.

  python tools/nccl_gather_check.py
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from first_raytracer_amd.dist import TileGather
    dev = torch.device("cuda", 0)
    n = 1 << 20
    src = torch.arange(n, dtype=torch.float32, device=dev)
    out = torch.zeros(n, dtype=torch.float32, device=dev)
    dist.gather(src, list(out.view(1, -1).unbind(0)), dst=0)
    torch.cuda.synchronize()
    assert torch.equal(out, src), "gather"
    t = torch.ones(16, device=dev)
    dist.all_reduce(t)
    assert float(t.sum()) == 16.0, "all_reduce"
    g = TileGather(64, 48, 32, 1, 0, dev)
    g.my_slots.copy_(torch.arange(g.my_slots.numel(), dtype=torch.float32, device=dev))
    film = g.gather()
    assert film.shape[0] == 64 * 48 * 3 and torch.isfinite(film).all()
    dist.barrier()
    dist.destroy_process_group()
    print("nccl gather/all_reduce/barrier OK", torch.__version__, flush=True)


if __name__ == "__main__":
    main()
