"""Python mirror of the MI355X PairHMM engine's C ABI (include/hc_pairhmm.h).

Thin ctypes binding over the in-tree ``libhcpairhmm.so``; the compute always
runs through that library's HIP kernels. There is no Python or CPU fallback:
if the library is missing, or no gfx950 device is usable, calls raise
``PairHMMError``.

Names follow the reference's PairHMM interface
(src/haplotypecaller/pairhmm/intel_pairhmm.hpp):

* :func:`compute_likelihoods` — IntelPairHMM::compute_likelihoods (:48-56):
  reads x haps log10 likelihoods, normalised, poorly modelled reads removed.
* :func:`cross` — computeLikelihoodsNative (:115-152) without normalisation.
* :func:`pairs` — the same per-pair computation over independent pairs.
* :class:`Batch` — plan (pack + upload) once, run the device pass many times.
* :func:`submit_pairs` / :func:`submit_regions` + :meth:`Job.collect` — the
  asynchronous calls: host planning of the next batch overlaps the device pass.
* :func:`init_devices` — one process, several device slots (each call is
  split by cells over them).
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# HC_PHMM_LIB: load another build of the library (A/B experiments only). The
# binding refuses it unless HC_PHMM_AB=1 says the caller means it (an A/B run
# is reported as such by check_build_id; a product run never loads it).
LIB_PATH = os.environ.get("HC_PHMM_LIB") or os.path.join(HERE, "libhcpairhmm.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "hc_pairhmm.h")

OK, EINVAL, ENODEV, EHIP, ENOMEM = 0, -1, -2, -3, -4

_u8p = C.POINTER(C.c_uint8)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_f32p = C.POINTER(C.c_float)
_f64p = C.POINTER(C.c_double)


class PairHMMError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hc_phmm error {code}: {msg}")
        self.code = code


class Read(C.Structure):
    """hc_phmm_read == shacc_pairhmm::Read (shacc_pairhmm.h:12-19)."""
    _fields_ = [("length", C.c_int32), ("bases", C.c_char_p), ("q", C.c_char_p),
                ("i", C.c_char_p), ("d", C.c_char_p), ("c", C.c_char_p)]


class Hap(C.Structure):
    """hc_phmm_hap == shacc_pairhmm::Haplotype (shacc_pairhmm.h:21-24)."""
    _fields_ = [("length", C.c_int32), ("bases", C.c_char_p)]


class Region(C.Structure):
    """hc_phmm_region: one active region's reads x haps cross product."""
    _fields_ = [("reads", C.POINTER(Read)), ("n_reads", C.c_int32), ("haps", C.POINTER(Hap)),
                ("n_haps", C.c_int32), ("out", C.POINTER(C.c_double))]


class Stats(C.Structure):
    _fields_ = [("n_pairs", C.c_int64), ("cells", C.c_int64), ("n_rescued", C.c_int64),
                ("kernel_ms_f32", C.c_double), ("kernel_ms_f64", C.c_double),
                ("run_ms", C.c_double), ("n_launch_waves", C.c_int64), ("n_runs", C.c_int64),
                ("n_lane_pairs", C.c_int64), ("n_seg_waves", C.c_int64), ("n_devices", C.c_int64),
                ("pack_ms", C.c_double), ("upload_bytes", C.c_int64)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "-j8"], check=True)


def ensure_built() -> dict:
    """Build the library if it is missing, or rebuild it if its build id does
    not match the tree's sources (make decides by timestamps, which a copied
    tree may not keep: a binary stale by content is rebuilt with -B); returns
    the verified build id."""
    if _lib is None:
        if not os.path.exists(LIB_PATH) or _stale_by_content():
            build()
        if _stale_by_content():
            subprocess.run(["make", "-s", "-B", "-C", HERE, "-j8"], check=True)
    return check_build_id()


def _stale_by_content() -> bool:
    """Build id of the binary on disk (read from its bytes, without loading it)
    against the tree's hashes."""
    data = open(LIB_PATH, "rb").read()
    t = tree_hashes()
    return f"kernel={t['kernel']} lib={t['lib']}".encode() not in data


_lib = None


def lib():
    """Load libhcpairhmm.so (raises if it was never built)."""
    global _lib
    if _lib is not None:
        return _lib
    if os.environ.get("HC_PHMM_LIB") and os.environ.get("HC_PHMM_AB") != "1":
        raise PairHMMError(EINVAL, f"HC_PHMM_LIB={LIB_PATH} names an A/B build: set HC_PHMM_AB=1 to load it "
                                   "(its build id is then reported, not checked against the tree)")
    if not os.path.exists(LIB_PATH):
        raise PairHMMError(ENODEV, f"{LIB_PATH} missing: run `make -C {HERE}` (no fallback path exists)")
    L = C.CDLL(LIB_PATH)
    L.hc_phmm_init.argtypes = [C.c_uint32, C.c_int]
    L.hc_phmm_init_devices.argtypes = [C.c_uint32, _i32p, C.c_int32]
    L.hc_phmm_submit_pairs.argtypes = [C.c_int64, _i64p, _i32p, _i64p, _i32p] + [_u8p] * 6 + \
        [_f64p, _f32p, _f64p, _u8p, C.POINTER(C.c_void_p)]
    L.hc_phmm_submit_regions.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]
    L.hc_phmm_job_ready.argtypes = [C.c_void_p]
    L.hc_phmm_collect.argtypes = [C.c_void_p]
    L.hc_phmm_last_error.restype = C.c_char_p
    if hasattr(L, "hc_phmm_build_id"):   # (absent from pre-round-4 builds loaded for A/B)
        L.hc_phmm_build_id.restype = C.c_char_p
    flat = [C.c_int64, _i64p, _i32p, _i64p, _i32p] + [_u8p] * 6
    L.hc_phmm_pairs_flat.argtypes = flat + [_f64p, _f32p, _f64p, _u8p]
    L.hc_phmm_cross.argtypes = [C.POINTER(Read), C.c_int32, C.POINTER(Hap), C.c_int32, _f64p]
    L.hc_phmm_cross_ex.argtypes = [C.POINTER(Read), C.c_int32, C.POINTER(Hap), C.c_int32, _f64p, C.c_uint32]
    L.hc_phmm_cross_regions.argtypes = [C.POINTER(Region), C.c_int32]
    L.hc_phmm_compute_likelihoods.argtypes = [C.POINTER(Read), C.c_int32, C.POINTER(Hap), C.c_int32,
                                              _f64p, _u8p, _i32p]
    L.hc_phmm_compute_likelihoods_ex.argtypes = [C.POINTER(Read), C.c_int32, C.POINTER(Hap), C.c_int32,
                                                 _f64p, _u8p, _i32p, C.c_uint32]
    L.hc_phmm_batch_create.argtypes = flat + [C.POINTER(C.c_void_p)]
    L.hc_phmm_batch_run.argtypes = [C.c_void_p, C.c_void_p]
    L.hc_phmm_batch_results.argtypes = [C.c_void_p, _f64p, _f32p, _f64p, _u8p]
    L.hc_phmm_batch_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
    L.hc_phmm_batch_device_results.argtypes = [C.c_void_p] + [C.POINTER(C.c_void_p)] * 3
    L.hc_phmm_batch_bind_outputs.argtypes = [C.c_void_p] * 4
    L.hc_phmm_batch_destroy.argtypes = [C.c_void_p]
    L.hc_phmm_get_luts.argtypes = [_f32p, _f64p, _f32p, _f64p]
    L.hcx_test_plan_timeout.argtypes = [C.c_int]   # test hook (tests only)
    L.hcx_flat_nibble_parts.argtypes = [C.c_int]   # test hook (tests only)
    L.hcx_flat_nibble_parts.restype = C.c_int
    _lib = L
    return L


def build_id() -> dict:
    """The loaded library's build id (hc_phmm_build_id): {"kernel": hash of the
    device kernel sources, "lib": hash of every library source and flag,
    "git": HEAD at build time}."""
    txt = lib().hc_phmm_build_id().decode()
    return dict(kv.split("=", 1) for kv in txt.split())


def tree_hashes() -> dict:
    """The same two hashes of the source tree this module sits in
    (tools/kernel_src_hash.py)."""
    import importlib.util
    path = os.path.join(os.path.dirname(HERE), "tools", "kernel_src_hash.py")
    spec = importlib.util.spec_from_file_location("_hc_kernel_src_hash", path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return {"kernel": m.kernel_src_hash(), "lib": m.lib_src_hash()}


def check_build_id() -> dict:
    """Refuse a stale binary: the loaded library's source hashes must equal the
    tree's. Returns the build id (with the tree's hashes) on success. An A/B
    build loaded through HC_PHMM_LIB is reported, not checked."""
    if os.environ.get("HC_PHMM_LIB"):
        try:
            bid = build_id()
        except AttributeError:
            bid = {}
        return dict(bid, ab_lib=LIB_PATH, tree_kernel=tree_hashes()["kernel"], tree_lib=tree_hashes()["lib"])
    tree = tree_hashes()
    bid = build_id()
    if bid.get("kernel") != tree["kernel"] or bid.get("lib") != tree["lib"]:
        raise PairHMMError(ENODEV, f"{LIB_PATH} is stale: built from kernel={bid.get('kernel')} "
                                   f"lib={bid.get('lib')}, tree has kernel={tree['kernel']} lib={tree['lib']} "
                                   f"(rebuild: make -C {HERE})")
    return dict(bid, tree_kernel=tree["kernel"], tree_lib=tree["lib"])


def declared_symbols(header: str = HEADER):
    """Every function the C header declares (for the export test)."""
    txt = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(hc_phmm_\w+)\s*\(", txt, re.M)))


def _check(rc: int):
    if rc != OK:
        msg = lib().hc_phmm_last_error()
        raise PairHMMError(rc, msg.decode() if msg else "")


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


FLAG_F64 = 1         # HC_PHMM_FLAG_F64: initNative(use_double = true), every pair in fp64 only
FLAG_KEEP_MODE = 2   # HC_PHMM_FLAG_KEEP_MODE: hc_phmm_init selects the device, the default mode stays


def init(device: int = -1, use_double: bool = False) -> None:
    """Select the device (-1: current / whatever the engine already runs on).
    use_double: initNative(use_double) (intel_pairhmm.hpp:71,81,135) — every
    pair computed in fp64 only (process-wide until the next init)."""
    _check(lib().hc_phmm_init(FLAG_F64 if use_double else 0, device))


def init_devices(devices=None, use_double: bool = False) -> None:
    """Configure device slots (HIP ordinals; None = every visible device). An
    ordinal may repeat: two streams on one GPU."""
    fl = FLAG_F64 if use_double else 0
    if devices is None:
        _check(lib().hc_phmm_init_devices(fl, None, 0))
        return
    arr = np.ascontiguousarray(devices, np.int32)
    _check(lib().hc_phmm_init_devices(fl, _p(arr, _i32p), len(arr)))


def device_count() -> int:
    return int(lib().hc_phmm_device_count())


def shutdown() -> None:
    _check(lib().hc_phmm_shutdown())


def get_luts():
    out = dict(ph2pr_f=np.zeros(128, np.float32), ph2pr_d=np.zeros(128, np.float64),
               mm_f=np.zeros(32640, np.float32), mm_d=np.zeros(32640, np.float64))
    _check(lib().hc_phmm_get_luts(_p(out["ph2pr_f"], _f32p), _p(out["ph2pr_d"], _f64p),
                                  _p(out["mm_f"], _f32p), _p(out["mm_d"], _f64p)))
    return out


def _flat_args(b):
    arrs = dict(read_off=np.ascontiguousarray(b["read_off"], np.int64),
                R=np.ascontiguousarray(b["R"], np.int32),
                hap_off=np.ascontiguousarray(b["hap_off"], np.int64),
                H=np.ascontiguousarray(b["H"], np.int32))
    for k in ("rs", "q", "ins", "dels", "gcp", "hap"):
        arrs[k] = np.ascontiguousarray(b[k], np.uint8)
    args = [len(arrs["R"]), _p(arrs["read_off"], _i64p), _p(arrs["R"], _i32p),
            _p(arrs["hap_off"], _i64p), _p(arrs["H"], _i32p)] + \
           [_p(arrs[k], _u8p) for k in ("rs", "q", "ins", "dels", "gcp", "hap")]
    return args, arrs


def result_arrays(n: int):
    """Output arrays of a flat call of n pairs (reusable across calls, as a C++
    caller reuses its result buffers)."""
    return dict(loglik=np.zeros(n, np.float64), raw_f32=np.zeros(n, np.float32),
                raw_f64=np.zeros(n, np.float64), rescued=np.zeros(n, np.uint8))


def pairs(b, out=None):
    """Independent pairs (flat batch dict, see workloads.py) -> dict of results
    (written into `out` from :func:`result_arrays` when given)."""
    args, keep = _flat_args(b)
    n = len(keep["R"])
    if out is None:
        out = result_arrays(n)
    _check(lib().hc_phmm_pairs_flat(*args, _p(out["loglik"], _f64p), _p(out["raw_f32"], _f32p),
                                    _p(out["raw_f64"], _f64p), _p(out["rescued"], _u8p)))
    return out


def _structs(reads, haps):
    """reads: list of (bases, q, i, d, c) bytes; haps: list of bytes."""
    keep = []
    ra = (Read * max(len(reads), 1))()
    for k, r in enumerate(reads):
        bases, q, i, d, c = r
        keep.extend(r)
        ra[k] = Read(len(bases), bases, q, i, d, c)
    ha = (Hap * max(len(haps), 1))()
    for k, h in enumerate(haps):
        keep.append(h)
        ha[k] = Hap(len(h), h)
    return ra, ha, keep


def cross(reads, haps, use_double=None):
    """All reads x all haps -> (n_reads, n_haps) log10 likelihoods (unnormalised).
    use_double: None = the process default (init); True / False = this call's
    mode (hc_phmm_cross_ex)."""
    ra, ha, _keep = _structs(reads, haps)
    out = np.zeros((len(reads), len(haps)), np.float64)
    if use_double is None:
        _check(lib().hc_phmm_cross(ra, len(reads), ha, len(haps), _p(out, _f64p)))
    else:
        _check(lib().hc_phmm_cross_ex(ra, len(reads), ha, len(haps), _p(out, _f64p),
                                      FLAG_F64 if use_double else 0))
    return out


class CrossCall:
    """hc_phmm_cross on one fixed region with its argument structs built once,
    as a C++ caller holds them (IntelPairHMM::compute_likelihoods' inputs,
    intel_pairhmm.hpp:48-56): calling it times the library, not ctypes."""

    def __init__(self, reads, haps):
        self.ra, self.ha, self._keep = _structs(reads, haps)
        self.nr, self.nh = len(reads), len(haps)
        self.out = np.zeros((self.nr, self.nh), np.float64)
        self._outp = _p(self.out, _f64p)

    def __call__(self):
        _check(lib().hc_phmm_cross(self.ra, self.nr, self.ha, self.nh, self._outp))
        return self.out


class RegionsCall:
    """hc_phmm_cross_regions / hc_phmm_submit_regions on fixed regions with the
    argument structs built once (as a C++ caller holds them)."""

    def __init__(self, regions):
        self.arr, self.outs, self._keep = _region_array(regions)
        self.n = len(regions)

    def __call__(self):
        _check(lib().hc_phmm_cross_regions(self.arr, self.n))
        return self.outs

    def submit(self) -> "Job":
        h = C.c_void_p()
        _check(lib().hc_phmm_submit_regions(self.arr, self.n, C.byref(h)))
        return Job(h, self.outs, None)


def _region_array(regions):
    keep, outs = [], []
    arr = (Region * max(len(regions), 1))()
    for k, (reads, haps) in enumerate(regions):
        ra, ha, kk = _structs(reads, haps)
        out = np.zeros((len(reads), len(haps)), np.float64)
        keep.extend([ra, ha, kk])
        outs.append(out)
        arr[k] = Region(ra, len(reads), ha, len(haps), _p(out, _f64p))
    return arr, outs, keep


def cross_regions(regions):
    """Many regions in one device pass: regions = [(reads, haps), ...] as for
    :func:`cross`; returns one (n_reads, n_haps) array per region."""
    arr, outs, _keep = _region_array(regions)
    _check(lib().hc_phmm_cross_regions(arr, len(regions)))
    return outs


class Job:
    """An asynchronous call in flight (hc_phmm_job): :meth:`collect` waits for
    the device and returns the results; the inputs may be dropped already."""

    def __init__(self, handle, result, keep):
        self._h, self._result, self._keep = handle, result, keep

    def ready(self) -> bool:
        rc = lib().hc_phmm_job_ready(self._h)
        if rc < 0:
            _check(rc)
        return rc == 1

    def collect(self):
        h, self._h = self._h, None
        if h is None:
            raise PairHMMError(EINVAL, "job already collected")
        _check(lib().hc_phmm_collect(h))
        self._keep = None
        return self._result

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().hc_phmm_collect(self._h)
            except Exception:
                pass


def submit_pairs(b, out=None) -> Job:
    """Asynchronous :func:`pairs`: returns a :class:`Job` whose collect()
    gives the same dict."""
    args, _arrs = _flat_args(b)
    n = len(_arrs["R"])
    if out is None:
        out = result_arrays(n)
    h = C.c_void_p()
    _check(lib().hc_phmm_submit_pairs(*args, _p(out["loglik"], _f64p), _p(out["raw_f32"], _f32p),
                                      _p(out["raw_f64"], _f64p), _p(out["rescued"], _u8p), C.byref(h)))
    return Job(h, out, None)


def submit_regions(regions) -> Job:
    """Asynchronous :func:`cross_regions`."""
    arr, outs, keep = _region_array(regions)
    h = C.c_void_p()
    _check(lib().hc_phmm_submit_regions(arr, len(regions), C.byref(h)))
    return Job(h, outs, None)


def compute_likelihoods(haps, reads, use_double=None):
    """IntelPairHMM::compute_likelihoods(haplotypes, reads): returns (L, kept_reads)
    where L has one row per surviving read (intel_pairhmm.hpp:48-56, 24-46).
    use_double as in :func:`cross` (the reference's per-instance mode)."""
    ra, ha, _keep = _structs(reads, haps)
    out = np.zeros((len(reads), len(haps)), np.float64)
    keep = np.zeros(max(len(reads), 1), np.uint8)
    nk = C.c_int32(0)
    if use_double is None:
        _check(lib().hc_phmm_compute_likelihoods(ra, len(reads), ha, len(haps), _p(out, _f64p),
                                                 _p(keep, _u8p), C.byref(nk)))
    else:
        _check(lib().hc_phmm_compute_likelihoods_ex(ra, len(reads), ha, len(haps), _p(out, _f64p),
                                                    _p(keep, _u8p), C.byref(nk), FLAG_F64 if use_double else 0))
    mask = keep[:len(reads)].astype(bool)
    return out[mask], [r for r, k in zip(reads, mask) if k]


class Batch:
    """Prepared, device-resident batch: create (pack + H2D) once, run many times."""

    def __init__(self, b):
        args, self._arrs = _flat_args(b)
        self.n = len(self._arrs["R"])
        h = C.c_void_p()
        _check(lib().hc_phmm_batch_create(*args, C.byref(h)))
        self._h = h

    def run(self, stream=None):
        """Enqueue the device pass (asynchronous). stream: a hipStream_t handle as
        int (e.g. torch.cuda.Stream().cuda_stream), or None for the library's own
        stream. The legacy null stream (0, torch's default stream) cannot be
        named through the C ABI, where NULL means the library stream: run under a
        created stream to order the pass with other work."""
        if stream is not None and int(stream) == 0:
            raise ValueError("stream 0 (the null stream) is not selectable; pass a created stream or None")
        _check(lib().hc_phmm_batch_run(self._h, C.c_void_p(stream) if stream else None))

    def results(self):
        n = self.n
        out = dict(loglik=np.zeros(n, np.float64), raw_f32=np.zeros(n, np.float32),
                   raw_f64=np.zeros(n, np.float64), rescued=np.zeros(n, np.uint8))
        _check(lib().hc_phmm_batch_results(self._h, _p(out["loglik"], _f64p), _p(out["raw_f32"], _f32p),
                                           _p(out["raw_f64"], _f64p), _p(out["rescued"], _u8p)))
        return out

    def stats(self) -> Stats:
        st = Stats()
        _check(lib().hc_phmm_batch_stats(self._h, C.byref(st)))
        return st

    def device_results(self):
        p = [C.c_void_p() for _ in range(3)]
        _check(lib().hc_phmm_batch_device_results(self._h, *[C.byref(x) for x in p]))
        return tuple(x.value for x in p)

    def bind_outputs(self, raw_f32=None, raw_f64=None, rescued=None):
        """Write later runs' results into caller-owned device buffers (int pointers,
        e.g. torch_tensor.data_ptr())."""
        _check(lib().hc_phmm_batch_bind_outputs(self._h, raw_f32, raw_f64, rescued))

    def close(self):
        if getattr(self, "_h", None):
            lib().hc_phmm_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
