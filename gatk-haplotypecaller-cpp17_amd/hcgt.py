"""Python mirror of the MI355X genotyper numeric core (include/hc_gt.h).

``genotype_sites(mats, sites)`` is the per-site arithmetic of
Genetyper::assign_genotype_likelihoods (reference genotyper/genotyper.hpp:369-399:
marginalize -> calculate_genotype_likelihoods -> get_genotype_quality_and_max_
genotype_index) for many sites in one device pass. Sites are dicts
{m: matrix index, keep: int32[], hap_allele: int32[], n_alleles} over the
read-major likelihood matrices ``mats`` (gt_workloads layout). Returns a list of
(genotype_likelihoods float64[], genotype_index, genotype_quality).
No CPU path: raises GTError without the library or a gfx950 device.
"""
from __future__ import annotations

import ctypes as C
import re

import numpy as np

import hcphmm

HEADER = hcphmm.HEADER.replace("hc_pairhmm.h", "hc_gt.h")
_f64p = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int32)


class GTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hc_gt error {code}: {msg}")
        self.code = code


class Site(C.Structure):
    _fields_ = [("L", _f64p), ("n_reads", C.c_int32), ("n_haps", C.c_int32), ("keep", _i32p),
                ("n_keep", C.c_int32), ("hap_allele", _i32p), ("n_alleles", C.c_int32),
                ("genotype_likelihoods", _f64p), ("genotype_index", _i32p), ("genotype_quality", _i32p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = hcphmm.lib()
        L.hc_gt_genotype_sites.argtypes = [C.POINTER(Site), C.c_int32]
        _lib = L
    return _lib


def declared_symbols(header: str = HEADER):
    return sorted(set(re.findall(r"^\s*int\s+(hc_gt_\w+)\s*\(", open(header).read(), re.M)))


class Prepared:
    """The C structs of a call, built once (the bench times run() alone)."""

    def __init__(self, mats, sites):
        self.mats = [np.ascontiguousarray(m, np.float64) for m in mats]
        self.n = len(sites)
        self.arr = (Site * max(self.n, 1))()
        self.keep_alive, self.outs = [], []
        for k, s in enumerate(sites):
            m = self.mats[s["m"]]
            keep = np.ascontiguousarray(s["keep"], np.int32)
            amap = np.ascontiguousarray(s["hap_allele"], np.int32)
            A = int(s["n_alleles"])
            gl = np.zeros(A * (A + 1) // 2, np.float64)
            gi = np.zeros(1, np.int32)
            gq = np.zeros(1, np.int32)
            self.keep_alive += [keep, amap]
            self.outs.append((gl, gi, gq))
            self.arr[k] = Site(m.ctypes.data_as(_f64p), m.shape[0], m.shape[1],
                               keep.ctypes.data_as(_i32p) if len(keep) else None, len(keep),
                               amap.ctypes.data_as(_i32p), A, gl.ctypes.data_as(_f64p),
                               gi.ctypes.data_as(_i32p), gq.ctypes.data_as(_i32p))

    def run(self):
        rc = lib().hc_gt_genotype_sites(self.arr, self.n)
        if rc != 0:
            msg = lib().hc_phmm_last_error()
            raise GTError(rc, msg.decode() if msg else "")

    def results(self):
        return [(gl.copy(), int(gi[0]), int(gq[0])) for gl, gi, gq in self.outs]


def genotype_sites(mats, sites):
    p = Prepared(mats, sites)
    p.run()
    return p.results()
