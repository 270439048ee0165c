"""GPU: bench.py's multi-rank path (one process per rank, shard by cells, the
device pass on a created stream, gather to rank 0, reassembly) run with two
ranks on the one GPU over gloo — the path the driver's 8-GPU run takes over
RCCL. The last step writes into NaN-poisoned outputs, so the gathered results
must come from that run; the reassembled batch is compared with the oracle."""
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
