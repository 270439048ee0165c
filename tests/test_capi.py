"""CPU: the C-ABI library loads, exports every declared symbol, and its host
side (LUTs, argument checks) is correct without a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import hcphmm


@pytest.fixture(scope="module")
def built():
    hcphmm.ensure_built()
    return hcphmm.lib()


def test_build_id_matches_tree(built):
    """The loaded binary says which sources it was built from
    (hc_phmm_build_id), and they are this tree's."""
    bid = hcphmm.build_id()
    assert set(bid) >= {"kernel", "lib", "git"}
    tree = hcphmm.tree_hashes()
    assert bid["kernel"] == tree["kernel"] and bid["lib"] == tree["lib"], (bid, tree)
    assert re.fullmatch(r"[0-9a-f]{16}", bid["kernel"]) and re.fullmatch(r"[0-9a-f]{16}", bid["lib"])


def test_exports_every_declared_symbol(built):
    syms = hcphmm.declared_symbols()
    assert len(syms) >= 14
    out = subprocess.run(["nm", "-D", "--defined-only", hcphmm.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_library_has_gfx950_code_object(built):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", hcphmm.LIB_PATH],
                         capture_output=True, text=True)
    text = out.stdout + out.stderr
    if out.returncode != 0 or "gfx" not in text:
        data = open(hcphmm.LIB_PATH, "rb").read()
        assert b"gfx950" in data
    else:
        assert "gfx950" in text


def test_struct_layout_matches_shacc(built):
    # shacc_pairhmm::Read {int; 5 x const char*} / Haplotype {int; const char*}
    assert ctypes.sizeof(hcphmm.Read) == 48
    assert hcphmm.Read.bases.offset == 8
    assert ctypes.sizeof(hcphmm.Hap) == 16


def test_engine_luts_match_reference(built, golden):
    L = hcphmm.get_luts()
    for k in L:
        assert np.array_equal(L[k].view(np.uint8), golden[k].view(np.uint8)), k


def test_no_silent_fallback_without_gpu(built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(hcphmm.PairHMMError) as e:
        hcphmm.init()
    assert e.value.code == hcphmm.ENODEV
    b = {"read_off": np.zeros(1, np.int64), "R": np.ones(1, np.int32),
         "hap_off": np.zeros(1, np.int64), "H": np.ones(1, np.int32)}
    for k in ("rs", "q", "ins", "dels", "gcp", "hap"):
        b[k] = np.array([65], np.uint8)
    with pytest.raises(hcphmm.PairHMMError):
        hcphmm.pairs(b)


def test_cpp_shim_compiles(tmp_path):
    """include/hc_pairhmm.hpp (the IntelPairHMM drop-in) compiles against a
    stand-in of the caller's SAMRecord/Haplotype shape and links."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "shim.cpp"
    src.write_text(r'''
#include "hc_pairhmm.hpp"
#include <string>
#include <string_view>
#include <vector>
struct SAMRecord { std::string SEQ, QUAL;
  static inline const std::string GOP = std::string(200, 'I');
  static inline const std::string GCP = std::string(200, '+');
  auto insertionGOP() const { return std::string_view{GOP}.substr(0, SEQ.size()); }
  auto deletionGOP() const { return std::string_view{GOP}.substr(0, SEQ.size()); }
  auto overallGCP() const { return std::string_view{GCP}.substr(0, SEQ.size()); }
  auto size() const { return SEQ.size(); } };
struct Haplotype { std::string bases; };
int main() {
  std::vector<Haplotype> h{{"ACGT"}, {"ACGA"}};
  std::vector<SAMRecord> r{{"ACG", "III"}};
  hc::MI355XPairHMM phmm;
  try { auto L = phmm.compute_likelihoods(h, r); return int(L.size()) - 1; }
  catch (const std::exception&) { return 0; }
}
''')
    exe = tmp_path / "shim"
    subprocess.run(["g++", "-std=c++17", "-I", os.path.join(root, "include"), str(src),
                    "-L", os.path.dirname(hcphmm.LIB_PATH), "-lhcpairhmm",
                    "-Wl,-rpath," + os.path.dirname(hcphmm.LIB_PATH), "-o", str(exe)], check=True)
    assert exe.exists()


def test_flat_record_nibble_packing():
    """Flat calls upload base codes as nibbles (flat_plan.cpp pack_nibbles,
    AVX2 with a scalar tail): ConvertChar codes (pairhmm_common.h:26-44: A0 C1
    T2 G3 N4, every other byte 0), two per byte, even index in the low nibble;
    every byte value and every length around the 64-byte vector step."""
    import ctypes as C
    import hcphmm
    L = hcphmm.lib()
    L.hcx_pack_nibbles.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    L.hcx_pack_nibbles.restype = None
    code = np.zeros(256, np.uint8)
    for ch, v in ((b"C", 1), (b"T", 2), (b"G", 3), (b"N", 4)):
        code[ch[0]] = v
    rng = np.random.default_rng(0)
    for n in list(range(0, 140)) + [255, 256, 257, 1000, 4096]:
        s = rng.integers(0, 256, n, dtype=np.uint8)
        if n >= 256:
            s[:256] = np.arange(256, dtype=np.uint8)
        c = code[s]
        exp = np.zeros((n + 1) // 2, np.uint8)
        exp[:] = c[0::2]
        exp[: n // 2] |= c[1::2] << 4
        got = np.full((n + 1) // 2 + 8, 0xEE, np.uint8)
        L.hcx_pack_nibbles(s.ctypes.data, n, got.ctypes.data)
        assert np.array_equal(got[: (n + 1) // 2], exp), n
        assert (got[(n + 1) // 2:] == 0xEE).all(), n   # nothing written past the record field


def test_flat_record_compact_fields():
    """Compact flat records (flat_plan.cpp, kernels.hpp kFmtRead1B /
    kFmtHap2b): a read with no 'N' whose qualities (& 127) lie in [33, 97)
    goes as ((q & 127) - 33) << 2 | code per base (codes A0 C1 T2 G3, every
    other byte 0 as ConvertChar), else it is refused; a hap with no 'N' as
    2-bit codes, 4 per byte (base k in bits 2(k % 4) of byte k / 4). Every
    byte value and the lengths around the 32-byte vector step."""
    import ctypes as C
    L = hcphmm.lib()
    L.hcx_pack_read_1b.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.hcx_pack_hap_2b.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    code = np.zeros(256, np.uint8)
    for ch, v in ((b"C", 1), (b"T", 2), (b"G", 3), (b"N", 4)):
        code[ch[0]] = v
    rng = np.random.default_rng(1)
    nonN = np.array([x for x in range(256) if x != ord("N")], np.uint8)
    for n in list(range(1, 100)) + [127, 128, 129, 255, 256, 1000, 2049]:
        b = rng.choice(nonN, n)
        if n >= 255:
            b[:255] = nonN
        q = (rng.integers(33, 97, n) | (rng.integers(0, 2, n) << 7)).astype(np.uint8)   # bit 7 ignored
        got = np.full(n + 8, 0xEE, np.uint8)
        assert L.hcx_pack_read_1b(q.ctypes.data, b.ctypes.data, n, got.ctypes.data) == 1, n
        qm = (q & 127).astype(np.int32)
        exp = (((qm - 33) << 2) | (code[b] & 3)).astype(np.uint8)
        assert np.array_equal(got[:n], exp), n
        assert (got[n:] == 0xEE).all(), n
        assert L.hcx_pack_read_1b(q.ctypes.data, b.ctypes.data, n, None) == 1, n   # check only
        bN = b.copy()   # refused: an 'N', a quality below 33 or from 97 on
        bN[n // 2] = ord("N")
        assert L.hcx_pack_read_1b(q.ctypes.data, bN.ctypes.data, n, got.ctypes.data) == 0
        for bad in (32, 97, 127, 0):
            q2 = q.copy()
            q2[n - 1] = bad
            assert L.hcx_pack_read_1b(q2.ctypes.data, b.ctypes.data, n, None) == 0, (n, bad)
        h = rng.choice(nonN, n)
        got = np.full((n + 3) // 4 + 8, 0xEE, np.uint8)
        assert L.hcx_pack_hap_2b(h.ctypes.data, n, got.ctypes.data) == 1, n
        c = np.zeros((n + 3) // 4 * 4, np.uint8)
        c[:n] = code[h] & 3
        exp = (c[0::4] | (c[1::4] << 2) | (c[2::4] << 4) | (c[3::4] << 6)).astype(np.uint8)
        assert np.array_equal(got[:(n + 3) // 4], exp), n
        assert (got[(n + 3) // 4:] == 0xEE).all(), n
        h[n - 1] = ord("N")
        assert L.hcx_pack_hap_2b(h.ctypes.data, n, got.ctypes.data) == 0, n


def test_init_rejects_unknown_flags(built):
    """hc_phmm_init flags: HC_PHMM_FLAG_F64 (initNative's use_double) and
    HC_PHMM_FLAG_KEEP_MODE; any other bit is refused before a device is
    touched, and so is an unknown mode of the per-call *_ex entry points."""
    L = hcphmm.lib()
    assert L.hc_phmm_init(4, 0) == hcphmm.EINVAL
    assert b"flags" in L.hc_phmm_last_error()
    assert L.hc_phmm_init_devices(0x80, None, 0) == hcphmm.EINVAL
    L.hc_phmm_cross_ex.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                   ctypes.c_void_p, ctypes.c_uint32]
    assert L.hc_phmm_cross_ex(None, 1, None, 1, None, 2) == hcphmm.EINVAL
    assert b"mode" in L.hc_phmm_last_error()


def test_stale_binary_is_refused(built, monkeypatch):
    """A library whose compiled-in source hashes differ from the tree's is
    refused (bench.py, smoke() and the GPU tests call check_build_id), and the
    content check that ensure_built uses to decide on a rebuild sees it."""
    real = hcphmm.tree_hashes()
    monkeypatch.setattr(hcphmm, "tree_hashes", lambda: {"kernel": "0" * 16, "lib": real["lib"]})
    with pytest.raises(hcphmm.PairHMMError) as e:
        hcphmm.check_build_id()
    assert "stale" in str(e.value)
    assert hcphmm._stale_by_content()
    monkeypatch.setattr(hcphmm, "tree_hashes", lambda: real)
    assert not hcphmm._stale_by_content()
    assert hcphmm.check_build_id()["kernel"] == real["kernel"]
