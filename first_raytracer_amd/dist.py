"""Tile sharding + the one collective of the multi-GPU path.

Tile t of the frame belongs to rank t mod N (frt_render_params.shard_index /
shard_count).  Each rank renders its tiles into a slot buffer in HBM; the
buffers (padded to the largest shard) are gathered to rank 0 with
torch.distributed -- RCCL grouped send/recv over xGMI with the "nccl"
backend, gloo in the CPU tests -- and rank 0 scatters the slots into the film
(viewer::fout_image order, y = 0 bottom).  Only rank 0 receives: N-1 buffers
cross the links once (SURVEY.md §8(e) "gather to rank 0"), not N(N-1) as an
all-gather would move.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import RenderParams, shard_slots


def shard_layout(nx, ny, tile, world):
    """(slot counts per rank, padded slot->pixel map of all ranks concatenated)."""
    maps = [shard_slots(RenderParams.make(nx, ny, 1, tile_size=tile, shard_index=r, shard_count=world))
            for r in range(world)]
    max_slots = max(len(m) for m in maps)
    padded = np.full((world, max_slots), -1, np.int64)
    for r, m in enumerate(maps):
        padded[r, :len(m)] = m
    return [len(m) for m in maps], padded.reshape(-1)


class TileGather:
    """Gather of per-rank slot buffers to rank 0 + scatter into rank 0's film."""

    def __init__(self, nx, ny, tile, world, rank, device, stage_cpu=False):
        """stage_cpu: gather through host copies (a gloo rehearsal of the GPU
        path on one device; RCCL gathers device buffers directly)."""
        self.nx, self.ny, self.world, self.rank = nx, ny, world, rank
        self.stage_cpu = stage_cpu
        counts, slot_pix = shard_layout(nx, ny, tile, world)
        self.max_slots = max(counts)
        self.my_slots = torch.zeros(self.max_slots * 3, dtype=torch.float32, device=device)
        self.gathered = (torch.zeros(world * self.max_slots * 3, dtype=torch.float32, device=device)
                         if world > 1 and rank == 0 else None)
        self.film = torch.zeros(nx * ny * 3, dtype=torch.float32, device=device) if rank == 0 else None
        if rank == 0:
            sp = torch.from_numpy(slot_pix).to(device)
            self.valid = sp >= 0
            self.dst = sp[self.valid]

    def _gather_list(self, buf):
        return list(buf.view(self.world, -1).unbind(0)) if self.rank == 0 else None

    def gather(self):
        """Collective: every rank calls it after rendering into self.my_slots."""
        src = self.my_slots
        if self.world > 1:
            if self.stage_cpu:
                g = torch.empty(self.world * self.max_slots * 3, dtype=torch.float32) if self.rank == 0 else None
                dist.gather(self.my_slots.cpu(), self._gather_list(g) if g is not None else None, dst=0)
                if self.rank == 0:
                    self.gathered.copy_(g)
            else:
                dist.gather(self.my_slots, self._gather_list(self.gathered), dst=0)
            src = self.gathered
        if self.rank == 0:
            self.film.view(-1, 3)[self.dst] = src.view(-1, 3)[self.valid]
        return self.film
