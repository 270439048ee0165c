"""GPU: bench.py's multi-rank path (one process per rank, shard by cells, the
device pass on a created stream, gather to rank 0, reassembly) run with two
and with eight ranks on the one GPU over gloo — the path the driver's 8-GPU
run takes over RCCL (BASELINE configs[3]: the full 1M-pair S2 batch sharded
eight ways). The last step writes into NaN-poisoned outputs, so the gathered
results must come from that run; the reassembled batch is compared with a
single-process run of the whole batch and with the oracle."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_two_rank_gloo_check_is_bit_exact(tmp_path, oracle_lib):
    npz = tmp_path / "gathered.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--pairs", "20000", "--dist-backend", "gloo",
           "--no-cpu", "--no-extra", "--check", "2000", "--check-out", str(npz)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["multi_rank_check"] == "2000 pairs bit-exact", out.get("multi_rank_check")
    got = np.load(npz)
    b = W.config("S2", 20_000)
    ref = oracle_lib.pairs(b, nthreads=16)
    assert np.array_equal(got["raw_f32"].view(np.uint32), ref["raw_f32"].view(np.uint32))
    m = ref["rescued"].astype(bool)
    assert np.array_equal(got["raw_f64"][m].view(np.uint64), ref["raw_f64"][m].view(np.uint64))
    assert (got["raw_f64"][~m] == 0).all()


def test_rccl_path_one_rank_overlapped_gather_is_bit_exact(tmp_path, oracle_lib):
    # The RCCL path the 8-GPU run takes (nccl process group, two output sets,
    # the gather of step k on its own stream overlapping step k + 1's pass,
    # NaN-poisoned last step), exercised at one rank on the one GPU.
    npz = tmp_path / "gathered.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--force-dist", "--steps", "3", "--warmup", "2", "--pairs", "20000",
           "--no-cpu", "--no-extra", "--check", "2000", "--check-out", str(npz)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["multi_rank_check"] == "2000 pairs bit-exact", out.get("multi_rank_check")
    assert "overlapping" in out["gather"]
    got = np.load(npz)
    ref = oracle_lib.pairs(W.config("S2", 20_000), nthreads=16)
    assert np.array_equal(got["raw_f32"].view(np.uint32), ref["raw_f32"].view(np.uint32))


@pytest.fixture(scope="module")
def s2_full_single(engine):
    """The whole S2 batch (configs[2]) in one process on one device slot."""
    b = W.config("S2")
    bt = engine.Batch(b)
    bt.run()
    r = bt.results()
    bt.close()
    return b, r


def test_configs3_eight_ranks_full_s2_is_bit_exact(tmp_path, oracle_lib, s2_full_single):
    """BASELINE configs[3]'s own workload through the HIP path: bench.py at 8
    ranks (gloo on the one GPU: the same sharding, per-rank batches, stream
    ordering and reassembly as the RCCL run) over the full 1M-pair S2 batch,
    the last step into NaN-poisoned outputs. The reassembled 1M raw results
    equal the single-process run bit for bit, and a 3 000-pair sample the oracle."""
    b, single = s2_full_single
    npz = tmp_path / "gathered8.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--steps", "2", "--warmup", "1", "--dist-backend", "gloo",
           "--no-cpu", "--no-extra", "--check", "3000", "--check-out", str(npz)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 8 and out["config"]["pairs"] == 1_000_000
    assert out["multi_rank_check"] == "3000 pairs bit-exact", out.get("multi_rank_check")
    got = np.load(npz)
    assert np.array_equal(got["raw_f32"].view(np.uint32), single["raw_f32"].view(np.uint32))
    assert np.array_equal(got["raw_f64"].view(np.uint64), single["raw_f64"].view(np.uint64))
    idx = np.sort(np.random.default_rng(11).choice(1_000_000, 3000, replace=False))
    ref = oracle_lib.pairs(W.subset(b, idx), nthreads=16)
    assert np.array_equal(got["raw_f32"][idx].view(np.uint32), ref["raw_f32"].view(np.uint32))
    m = ref["rescued"].astype(bool)
    assert np.array_equal(got["raw_f64"][idx][m].view(np.uint64), ref["raw_f64"][m].view(np.uint64))


def test_eight_device_slots_full_s2_is_bit_exact(engine, s2_full_single):
    """The library's own multi-GPU path (hc_phmm_init_devices) with eight
    device slots on the one GPU over the full S2 batch: split by cells into
    eight parts on eight streams, bit-identical to one slot."""
    b, single = s2_full_single
    engine.shutdown()
    engine.init_devices([0] * 8)
    try:
        assert engine.device_count() == 8
        bt = engine.Batch(b)
        st0 = bt.stats()
        assert st0.n_devices == 8
        bt.run()
        r = bt.results()
        bt.close()
        for k in single:
            assert np.array_equal(np.ascontiguousarray(r[k]).view(np.uint8),
                                  np.ascontiguousarray(single[k]).view(np.uint8)), k
        got = engine.pairs(b)   # the call path on 8 slots: 8 parts, device-planned, one per slot
        for k in single:
            assert np.array_equal(np.ascontiguousarray(got[k]).view(np.uint8),
                                  np.ascontiguousarray(single[k]).view(np.uint8)), k
    finally:
        engine.shutdown()
        engine.init(0)
