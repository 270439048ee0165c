"""Python mirror of the MI355X Smith-Waterman aligner (include/hc_sw.h).

Mirrors ``hc::IntelSWAligner`` (reference src/haplotypecaller/smithwaterman/
intel_smithwaterman.hpp:9-59): ``SWAligner.align(ref, alt, params)`` returns
``(offset, cigar)`` with the reference's semantics (all-match shortcut, then
the SOFTCLIP aligner), and ``align_many`` aligns every haplotype of a region —
or of many regions — against its window in one device pass (the loop of
assembler/graph_wrapper.hpp:232-240). The reference throws
``std::invalid_argument`` on empty sequences; so does this mirror (ValueError).

There is no CPU path: the library must be built and a gfx950 device present,
otherwise every call raises SWError.
"""
from __future__ import annotations

import ctypes as C
import re

import numpy as np

import hcphmm
import sw_workloads as SW

OK, EINVAL, ENODEV, EHIP, ENOMEM, ERANGE = 0, -1, -2, -3, -4, -5
HEADER = hcphmm.HEADER.replace("hc_pairhmm.h", "hc_sw.h")
MAX_LEN1, MAX_LEN2 = 1023, 1024
SOFTCLIP, INDEL, LEADING_INDEL, IGNORE = SW.SOFTCLIP, SW.INDEL, SW.LEADING_INDEL, SW.IGNORE

_u8p = C.POINTER(C.c_uint8)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)


class SWError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hc_sw error {code}: {msg}")
        self.code = code


class Params(C.Structure):
    """hc_sw_params == IntelSWAligner::SWParameters (intel_smithwaterman.hpp:12-18)."""
    _fields_ = [("match", C.c_int32), ("mismatch", C.c_int32), ("open", C.c_int32), ("extend", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("n_pairs", C.c_int64), ("n_shortcut", C.c_int64), ("cells", C.c_int64),
                ("dp_ms", C.c_double), ("trace_ms", C.c_double), ("run_ms", C.c_double),
                ("n_runs", C.c_int64)]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    L = hcphmm.lib()   # raises when the library was never built
    flat = [C.c_int64, _i64p, _i32p, _u8p, _i64p, _i32p, _u8p, Params, C.c_int32, C.c_int32]
    L.hc_sw_init.argtypes = [C.c_int]
    L.hc_sw_align_flat.argtypes = flat + [_i32p, C.c_char_p, C.c_int32]
    L.hc_sw_batch_create.argtypes = flat + [C.POINTER(C.c_void_p)]
    L.hc_sw_batch_run.argtypes = [C.c_void_p, C.c_void_p]
    L.hc_sw_batch_results.argtypes = [C.c_void_p, _i32p, C.c_char_p, C.c_int32, _i32p]
    L.hc_sw_batch_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
    L.hc_sw_batch_destroy.argtypes = [C.c_void_p]
    _lib = L
    return L


def declared_symbols(header: str = HEADER):
    txt = open(header).read()
    return sorted(set(re.findall(r"^\s*int\s+(hc_sw_\w+)\s*\(", txt, re.M)))


def _check(rc: int):
    if rc != OK:
        msg = lib().hc_phmm_last_error()
        raise SWError(rc, msg.decode() if msg else "")


def _p(a, t):
    return a.ctypes.data_as(t)


def init(device: int = -1):
    """Select the device (-1: the one the engine already runs on, else current)."""
    _check(lib().hc_sw_init(device))


def _pools(b):
    refs = b["refs"] if len(b["refs"]) else np.zeros(1, np.uint8)
    alts = b["alts"] if len(b["alts"]) else np.zeros(1, np.uint8)
    return refs, alts


def _args(b, params, overhang, shortcut):
    refs, alts = _pools(b)
    for k in ("ref_off", "alt_off"):
        assert b[k].dtype == np.int64
    for k in ("ref_len", "alt_len"):
        assert b[k].dtype == np.int32
    return (len(b["ref_len"]), _p(b["ref_off"], _i64p), _p(b["ref_len"], _i32p), _p(refs, _u8p),
            _p(b["alt_off"], _i64p), _p(b["alt_len"], _i32p), _p(alts, _u8p), Params(*params),
            int(overhang), int(bool(shortcut)))


def _decode(buf, n, stride):
    raw = buf.raw
    return [raw[k * stride:(k + 1) * stride].split(b"\0", 1)[0].decode() for k in range(n)]


def _worst_stride(b):
    return int(max(16, 4 * (int(b["ref_len"].max(initial=0)) + int(b["alt_len"].max(initial=0))) + 8))


def align_flat(b, params=SW.NEW_SW_PARAMETERS, overhang=SOFTCLIP, shortcut=True, stride=None):
    """hc_sw_align_flat over a flat batch (sw_workloads layout): (offsets, cigars).
    CIGARs go into `stride`-byte slots (default 512; retried at the worst case
    when one does not fit)."""
    n = len(b["ref_len"])
    for st in ([stride] if stride else [min(512, _worst_stride(b)), _worst_stride(b)]):
        off = np.zeros(max(n, 1), np.int32)
        buf = C.create_string_buffer(max(1, n * st))
        rc = lib().hc_sw_align_flat(*_args(b, params, overhang, shortcut), _p(off, _i32p), buf, st)
        if rc != ERANGE or stride:
            break
    _check(rc)
    return off[:n], _decode(buf, n, st)


class Batch:
    """Plan / execute split (hc_sw_batch_*): inputs stay resident on the device."""

    def __init__(self, b, params=SW.NEW_SW_PARAMETERS, overhang=SOFTCLIP, shortcut=True):
        self.n = len(b["ref_len"])
        self.worst = _worst_stride(b)
        h = C.c_void_p()
        _check(lib().hc_sw_batch_create(*_args(b, params, overhang, shortcut), C.byref(h)))
        self.h = h

    def run(self, stream=None):
        _check(lib().hc_sw_batch_run(self.h, C.c_void_p(stream) if stream else None))

    def results(self, scores=False):
        for stride in (min(512, self.worst), self.worst):
            off = np.zeros(max(self.n, 1), np.int32)
            sc = np.zeros(max(self.n, 1), np.int32)
            buf = C.create_string_buffer(max(1, self.n * stride))
            rc = lib().hc_sw_batch_results(self.h, _p(off, _i32p), buf, stride, _p(sc, _i32p) if scores else None)
            if rc != ERANGE:
                break
        _check(rc)
        out = (off[:self.n], _decode(buf, self.n, stride))
        return out + (sc[:self.n],) if scores else out

    def stats(self):
        st = Stats()
        _check(lib().hc_sw_batch_stats(self.h, C.byref(st)))
        return {k: getattr(st, k) for k, _ in Stats._fields_}

    def close(self):
        if self.h:
            lib().hc_sw_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SWAligner:
    """hc::IntelSWAligner (intel_smithwaterman.hpp:9-59) on the MI355X."""

    ORIGINAL_DEFAULT = SW.ORIGINAL_DEFAULT
    STANDARD_NGS = SW.STANDARD_NGS
    NEW_SW_PARAMETERS = SW.NEW_SW_PARAMETERS
    ALIGNMENT_TO_BEST_HAPLOTYPE_SW_PARAMETERS = SW.ALIGNMENT_TO_BEST_HAPLOTYPE
    MINIMAL_MISMATCH_TO_TOLERANCE = 2

    def align(self, ref: bytes, alt: bytes, params=SW.NEW_SW_PARAMETERS):
        """(offset, cigar) of alt against ref; ValueError on empty input (:33-34)."""
        return self.align_many(ref, [alt], params)[0]

    def align_many(self, ref: bytes, alts, params=SW.NEW_SW_PARAMETERS):
        """Every alt against one ref window in one device pass."""
        if not ref or any(not a for a in alts):
            raise ValueError("Non-null sequences are required for the SW aligner")
        if not alts:
            return []
        b = SW.from_pairs([(ref, a) for a in alts])
        off, cig = align_flat(b, params, SOFTCLIP, True)
        return [(int(o), c) for o, c in zip(off, cig)]
