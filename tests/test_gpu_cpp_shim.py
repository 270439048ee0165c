"""GPU: the C++ drop-in (include/hc_pairhmm.hpp, hc::MI355XPairHMM) and the
reference's accelerator slot (shacc_pairhmm::calculate) called from a compiled
C++ program with SAMRecord/Haplotype stand-ins, checked bit for bit against the
oracle's compute_likelihoods semantics (intel_pairhmm.hpp:24-56)."""
import os
import struct
import subprocess

import numpy as np
import pytest

import hcphmm
import workloads as W

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_dropin_region(tmp_path, oracle_lib):
    exe = tmp_path / "shim_region"
    libdir = os.path.dirname(hcphmm.LIB_PATH)
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "shim_region.cpp"), "-L", libdir, "-lhcpairhmm",
                    "-Wl,-rpath," + libdir, "-o", str(exe)], check=True)
    reads, haps = W.region(n_reads=60, n_haps=6, seed=77)
    # a few junk reads so the filter removes some, and one read longer than 200 bp
    rng = np.random.default_rng(1)
    for k in (3, 17, 41):
        rs = W.ACGT[rng.integers(0, 4, 150)].tobytes()
        reads[k] = (rs,) + reads[k][1:]
    long_hap = haps[0] + haps[1][:100]
    haps[2] = long_hap
    lr = long_hap[10:240]
    reads[5] = (lr, bytes([60]) * len(lr), b"I" * len(lr), b"I" * len(lr), b"+" * len(lr))
    blob = struct.pack("<ii", len(reads), len(haps))
    for r in reads:
        blob += struct.pack("<i", len(r[0])) + r[0] + struct.pack("<i", len(r[1])) + r[1]
    for h in haps:
        blob += struct.pack("<i", len(h)) + h
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    fin.write_bytes(blob)
    subprocess.run([str(exe), str(fin), str(fout)], check=True, timeout=120)
    data = fout.read_bytes()
    kept = struct.unpack("<i", data[:4])[0]
    nR, nH = len(reads), len(haps)
    mask = np.frombuffer(data[4:4 + nR], np.uint8).astype(bool)
    off = 4 + nR
    L = np.frombuffer(data[off:off + 8 * kept * nH], np.float64).reshape(kept, nH)
    off += 8 * kept * nH
    shacc = np.frombuffer(data[off:off + 4 * nR * nH], np.float32).reshape(nR, nH)

    flat = W.region_flat(reads, haps)
    raw = oracle_lib.pairs(flat, nthreads=8)["loglik"].reshape(nR, nH)
    refn, keep = oracle_lib.normalize(raw, np.array([len(r[0]) for r in reads], np.int32))
    assert kept == int(keep.sum()) and kept < nR
    assert np.array_equal(mask, keep)
    assert np.array_equal(L.view(np.uint64), refn[keep].view(np.uint64))
    assert np.array_equal(shacc, raw.astype(np.float32))
