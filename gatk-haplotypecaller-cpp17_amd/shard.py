"""Multi-GPU sharding of a pair batch.

Every (read, hap) pair is independent, so a batch splits across ranks with no
exchange during compute. Shards are balanced by cells (R*H), not pair count:
pairs are sorted by cells and dealt in snake order (0..N-1, N-1..0, ...),
which keeps every rank within one pair's cells of the mean. The only
collective is the gather of per-pair results to rank 0 (RCCL over xGMI with
the nccl backend; gloo in the CPU tests).
"""
from __future__ import annotations

import numpy as np


def shard_pairs(R, H, world: int):
    """Return a list of `world` int64 index arrays (each sorted ascending)."""
    n = len(R)
    if world <= 1:
        return [np.arange(n, dtype=np.int64)]
    cells = np.asarray(R, np.int64) * np.asarray(H, np.int64)
    order = np.argsort(-cells, kind="stable")
    pos = np.arange(n, dtype=np.int64)
    lap, k = np.divmod(pos, world)
    rank_of = np.where(lap % 2 == 0, k, world - 1 - k)
    out = []
    for r in range(world):
        out.append(np.sort(order[rank_of == r]))
    return out


def shard_cells(R, H, shards):
    cells = np.asarray(R, np.int64) * np.asarray(H, np.int64)
    return [int(cells[s].sum()) for s in shards]


def gather_results(dist, local: dict, shards, rank: int, world: int, device=None):
    """Gather per-pair result tensors of every rank to rank 0 and put them back
    in batch order. local: name -> 1-D torch tensor of this rank's shard
    (length >= len(shards[rank])). Returns name -> full tensor on rank 0, None
    elsewhere. Uses dist.gather (RCCL gather); shards are padded to the largest."""
    import torch

    nmax = max(len(s) for s in shards)
    full = {}
    for name, t in local.items():
        buf = t
        if buf.numel() < nmax:
            buf = torch.zeros(nmax, dtype=t.dtype, device=t.device)
            buf[: t.numel()] = t
        else:
            buf = buf[:nmax].contiguous()
        glist = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, gather_list=glist, dst=0)
        if rank == 0:
            n = sum(len(s) for s in shards)
            out = torch.empty(n, dtype=t.dtype, device=buf.device)
            for r, s in enumerate(shards):
                idx = torch.as_tensor(s, device=buf.device)
                out[idx] = glist[r][: len(s)]
            full[name] = out
    return full if rank == 0 else None
