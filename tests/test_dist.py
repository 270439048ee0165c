"""CPU: the multi-GPU data path (shard by cells -> per-rank compute -> gather to
rank 0) with the gloo backend at world size 2 and 4. The per-rank compute here
is the oracle standing in for the HIP engine (no GPU in this container); the
sharding and gather code is exactly what bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import shard
import workloads as W


def test_shards_partition_and_balance():
    b = W.config("S2", 20_000)
    for world in (1, 2, 3, 8):
        s = shard.shard_pairs(b["R"], b["H"], world)
        allidx = np.concatenate(s)
        assert len(allidx) == len(b["R"]) and len(np.unique(allidx)) == len(b["R"])
        cells = shard.shard_cells(b["R"], b["H"], s)
        cmax = int((b["R"].astype(np.int64) * b["H"]).max())
        assert max(cells) - min(cells) <= cmax


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    b = W.config("S2", 600)
    shards = shard.shard_pairs(b["R"], b["H"], world)
    sub = W.subset(b, shards[rank])
    res = oracle.Oracle().pairs(sub, nthreads=1)
    local = {"raw_f32": torch.from_numpy(res["raw_f32"]),
             "raw_f64": torch.from_numpy(res["raw_f64"])}
    full = shard.gather_results(dist, local, shards, rank, world)
    if rank == 0:
        ref = oracle.Oracle().pairs(b, nthreads=1)
        ok = (np.array_equal(full["raw_f32"].numpy().view(np.uint32), ref["raw_f32"].view(np.uint32))
              and np.array_equal(full["raw_f64"].numpy().view(np.uint64), ref["raw_f64"].view(np.uint64)))
        out_q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gather_reassembles_batch_order(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok
