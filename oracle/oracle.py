"""ctypes loader for the PairHMM oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module. It loads

* ``oracle/liboracle.so``  — our C restatement (pairhmm_oracle.c), and
* ``oracle/_ref/libref_pairhmm.so`` — the reference's AVX kernel compiled from
  /root/reference by oracle/Makefile (optional: absent when never built).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_pairhmm.so")

_u8p = C.POINTER(C.c_uint8)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_f32p = C.POINTER(C.c_float)
_f64p = C.POINTER(C.c_double)


def build(ref: bool = True) -> None:
    """Compile the oracle (and the reference driver when sources exist)."""
    targets = ["oracle"] + (["ref"] if ref else [])
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def _ptr(a, t):
    if a is None:
        return None
    return a.ctypes.data_as(t)


class _Lib:
    def __init__(self, path: str, prefix: str):
        self.path = path
        self.lib = C.CDLL(path)
        p = prefix
        self._f32 = getattr(self.lib, f"{p}_full_prob_f32")
        self._f64 = getattr(self.lib, f"{p}_full_prob_f64")
        self._pairs = getattr(self.lib, f"{p}_pairs")
        self._luts = getattr(self.lib, f"{p}_get_luts")
        self._sizes = getattr(self.lib, f"{p}_lut_sizes")
        args = [C.c_int, C.c_int] + [_u8p] * 6
        self._f32.argtypes = args
        self._f32.restype = C.c_float
        self._f64.argtypes = args
        self._f64.restype = C.c_double
        self._pairs.argtypes = [C.c_long, _i64p, _i32p, _i64p, _i32p] + [_u8p] * 6 + [
            _f32p, _f64p, _u8p, _f64p, C.c_int]
        self._pairs.restype = C.c_long
        self._luts.argtypes = [_f32p, _f64p, _f32p, _f64p, _f32p, _f64p]
        self._sizes.argtypes = [_i32p, _i32p, _i32p]

    def full_prob(self, rs: bytes, q: bytes, i: bytes, d: bytes, c: bytes, hap: bytes, f64=False):
        R, H = len(rs), len(hap)
        bufs = [np.frombuffer(x, dtype=np.uint8).copy() for x in (rs, q, i, d, c, hap)]
        fn = self._f64 if f64 else self._f32
        return fn(R, H, *[_ptr(b, _u8p) for b in bufs])

    def pairs(self, batch, nthreads: int = 1):
        """batch: dict from workloads (read_off, R, hap_off, H, rs, q, ins, dels, gcp, hap)."""
        n = len(batch["R"])
        raw32 = np.zeros(n, np.float32)
        raw64 = np.zeros(n, np.float64)
        resc = np.zeros(n, np.uint8)
        L = np.zeros(n, np.float64)
        b = batch
        nres = self._pairs(
            n, _ptr(b["read_off"], _i64p), _ptr(b["R"], _i32p), _ptr(b["hap_off"], _i64p),
            _ptr(b["H"], _i32p), _ptr(b["rs"], _u8p), _ptr(b["q"], _u8p), _ptr(b["ins"], _u8p),
            _ptr(b["dels"], _u8p), _ptr(b["gcp"], _u8p), _ptr(b["hap"], _u8p),
            _ptr(raw32, _f32p), _ptr(raw64, _f64p), _ptr(resc, _u8p), _ptr(L, _f64p), nthreads)
        return dict(raw_f32=raw32, raw_f64=raw64, rescued=resc, loglik=L, n_rescued=int(nres))

    def luts(self):
        n = [C.c_int32(), C.c_int32(), C.c_int32()]
        self._sizes(*[C.byref(x) for x in n])
        np_, nm, nj = (x.value for x in n)
        out = dict(ph2pr_f=np.zeros(np_, np.float32), ph2pr_d=np.zeros(np_, np.float64),
                   mm_f=np.zeros(nm, np.float32), mm_d=np.zeros(nm, np.float64),
                   jac_f=np.zeros(nj, np.float32), jac_d=np.zeros(nj, np.float64))
        self._luts(_ptr(out["ph2pr_f"], _f32p), _ptr(out["ph2pr_d"], _f64p),
                   _ptr(out["mm_f"], _f32p), _ptr(out["mm_d"], _f64p),
                   _ptr(out["jac_f"], _f32p), _ptr(out["jac_d"], _f64p))
        return out


class Oracle(_Lib):
    """Our C restatement (kind "port")."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build(ref=False)
        super().__init__(path, "hco")
        self.lib.hco_finish.argtypes = [C.c_float, C.c_double]
        self.lib.hco_finish.restype = C.c_double
        self.lib.hco_normalize.argtypes = [C.c_int, C.c_int, _i32p, _f64p, _u8p]
        self.lib.hco_normalize.restype = C.c_int

    def finish(self, f: float, d: float) -> float:
        return self.lib.hco_finish(f, d)

    def normalize(self, L: np.ndarray, read_len: np.ndarray):
        L = np.ascontiguousarray(L, dtype=np.float64).copy()
        nr, nh = L.shape
        keep = np.zeros(nr, np.uint8)
        rl = np.ascontiguousarray(read_len, dtype=np.int32)
        self.lib.hco_normalize(nr, nh, _ptr(rl, _i32p), _ptr(L, _f64p), _ptr(keep, _u8p))
        return L, keep.astype(bool)


class Reference(_Lib):
    """The reference's own AVX kernel (kind "reference"); raises if not built."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        super().__init__(path, "ref")


def reference_available() -> bool:
    return os.path.exists(REF_SO)


# --------------------------------------------------------------------------
# Smith-Waterman: oracle/sw_oracle.c (kind "port", in
# liboracle.so) and the reference aligner (oracle/_ref/libref_sw.so).
REF_SW_SO = os.path.join(HERE, "_ref", "libref_sw.so")
SW_CIGAR_STRIDE = 4096


class _SWLib:
    def __init__(self, fn, nthreads_arg: bool):
        self._fn = fn
        self._nt = nthreads_arg
        args = [C.c_long, _i64p, _i32p, _u8p, _i64p, _i32p, _u8p] + [C.c_int] * 6 + [_i32p, C.c_char_p, C.c_int]
        fn.argtypes = args + ([C.c_int] if nthreads_arg else [])
        fn.restype = C.c_int

    def batch(self, b, params=(200, -150, -260, -11), overhang=9, shortcut=True, nthreads=1,
              stride=SW_CIGAR_STRIDE):
        """IntelSWAligner::align over a flat batch (sw_workloads layout).
        Returns (offsets int32[n], cigars list[str])."""
        n = len(b["ref_len"])
        off = np.zeros(n, np.int32)
        cig = C.create_string_buffer(max(1, n * stride))
        refs = b["refs"] if len(b["refs"]) else np.zeros(1, np.uint8)
        alts = b["alts"] if len(b["alts"]) else np.zeros(1, np.uint8)
        extra = [nthreads] if self._nt else []
        rc = self._fn(n, _ptr(b["ref_off"], _i64p), _ptr(b["ref_len"], _i32p), _ptr(refs, _u8p),
                      _ptr(b["alt_off"], _i64p), _ptr(b["alt_len"], _i32p), _ptr(alts, _u8p),
                      *params, overhang, int(bool(shortcut)), _ptr(off, _i32p), cig, stride, *extra)
        if rc != 0:
            raise RuntimeError("CIGAR buffer too small")
        raw = cig.raw
        cigars = [raw[k * stride:(k + 1) * stride].split(b"\0", 1)[0].decode() for k in range(n)]
        return off, cigars


class SWOracle(_SWLib):
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build(ref=False)
        self.lib = C.CDLL(path)
        super().__init__(self.lib.hco_sw_batch, True)


class SWReference(_SWLib):
    def __init__(self, path: str = REF_SW_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = C.CDLL(path)
        super().__init__(self.lib.ref_sw_align_batch, False)


def sw_reference_available() -> bool:
    return os.path.exists(REF_SW_SO)


# --------------------------------------------------------------------------
# Genotyper numeric core: oracle/gt_oracle.c (in
# liboracle.so) and the reference's MathUtils (oracle/_ref/libref_math.so).
REF_MATH_SO = os.path.join(HERE, "_ref", "libref_math.so")


class GTOracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build(ref=False)
        self.lib = C.CDLL(path)
        self.lib.hco_approx_log10_sum_log10.argtypes = [C.c_double, C.c_double]
        self.lib.hco_approx_log10_sum_log10.restype = C.c_double
        self.lib.hco_gt_site.argtypes = [_f64p, C.c_int, _i32p, C.c_int, _i32p, C.c_int, _f64p, _i32p, _i32p]

    def approx(self, a: float, b: float) -> float:
        return self.lib.hco_approx_log10_sum_log10(a, b)

    def site(self, L, keep, hap_allele, n_alleles):
        L = np.ascontiguousarray(L, np.float64)
        keep = np.ascontiguousarray(keep, np.int32)
        amap = np.ascontiguousarray(hap_allele, np.int32)
        gl = np.zeros(n_alleles * (n_alleles + 1) // 2, np.float64)
        gi, gq = C.c_int32(), C.c_int32()
        self.lib.hco_gt_site(_ptr(L, _f64p), L.shape[1], _ptr(keep, _i32p), len(keep), _ptr(amap, _i32p),
                             n_alleles, _ptr(gl, _f64p), C.byref(gi), C.byref(gq))
        return gl, gi.value, gq.value


class MathReference:
    """The reference's MathUtils::approximate_log10_sum_log10, compiled in place."""

    def __init__(self, path: str = REF_MATH_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = C.CDLL(path)
        self.lib.ref_approx_log10_sum_log10.argtypes = [C.c_double, C.c_double]
        self.lib.ref_approx_log10_sum_log10.restype = C.c_double

    def approx(self, a: float, b: float) -> float:
        return self.lib.ref_approx_log10_sum_log10(a, b)
