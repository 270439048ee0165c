"""CPU: the host planner's output, checked without a GPU. The library plans a
batch in dry-run mode (hcx_plan_* with a modelled device, no HIP calls) and
hands back the plan (hcx_dump_*): pair descriptors, slot order, and the
column-segmented waves the fp32 kernel would run. Both planners — the
structured cross-product one (regions) and the general one (flat pairs, and
regions with HC_PHMM_GRID_PLAN=0) — must give a plan the kernel can run
exactly: every pair in exactly one slot, every wave's pairs fitting its 64
lanes at its block width (phmm_seg_kernel's lane -> group map), the wave's
row bounds and step count covering its pairs (run_seg's SegSteps)."""
import ctypes as C

import numpy as np
import pytest

import hcphmm
import workloads as W

WIDTHS = set(range(8, 65, 2))   # HC_SEG_WIDTHS (seg_common.hpp)


@pytest.fixture(scope="module")
def L():
    lib = hcphmm.lib()
    lib.hcx_plan_regions.restype = C.c_double
    lib.hcx_plan_regions.argtypes = [C.c_void_p, C.c_int32, C.c_int, C.c_int]
    lib.hcx_plan_pairs.restype = C.c_double
    lib.hcx_dump_sizes.argtypes = [C.c_void_p]
    lib.hcx_dump_plan.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    return lib


def dump(L):
    sz = np.zeros(5, np.int64)
    L.hcx_dump_sizes(sz.ctypes.data)
    n_pairs, n_order, n_seg, n_waves, grid = (int(x) for x in sz)
    pairs = np.zeros((max(n_pairs, 1), 4), np.int32)
    order = np.zeros(max(n_order, 1), np.int32)
    waves = np.zeros((max(n_waves, 1), 6), np.int32)
    L.hcx_dump_plan(pairs.ctypes.data, order.ctypes.data, waves.ctypes.data)
    return pairs[:n_pairs], order[:n_order], n_seg, waves[:n_waves], grid


def check_plan(pairs, order, n_seg, waves, R, H):
    n = len(R)
    assert len(pairs) == n
    assert np.array_equal(pairs[:, 1], R) and np.array_equal(pairs[:, 3], H)
    seg = order[:n_seg]
    assert len(np.unique(order)) == len(order) == n          # every pair in exactly one slot
    assert n_seg == n                                         # every hap here is in segmented reach
    w = waves[np.argsort(waves[:, 0], kind="stable")]
    starts = np.concatenate([[0], np.cumsum(w[:, 4])[:-1]])
    assert np.array_equal(w[:, 0], starts) and w[:, 4].sum() == n_seg   # slots partitioned by waves
    for slot0, rmax, rmin, bc, npairs, nsteps in w:
        assert bc in WIDTHS and 1 <= npairs <= 64
        p = seg[slot0:slot0 + npairs]
        nb = -(-H[p] // bc)
        assert nb.sum() <= 64 and nb.max() <= 64
        assert rmax == R[p].max() and rmin == R[p].min()
        assert nsteps == (R[p] + nb - 1).max()


def ragged_region(seed, nr, nh):
    rng = np.random.default_rng(seed)
    reads, haps = W.region(n_reads=nr, n_haps=nh, seed=seed)
    haps = [h[:int(rng.integers(30, len(h) + 1))] for h in haps]
    reads = [tuple(x[:int(rng.integers(20, len(r[0]) + 1))] for x in r) for r in reads]
    return reads, haps


@pytest.mark.parametrize("grid", ["1", "0"])
def test_region_plans_are_exact(L, monkeypatch, grid):
    monkeypatch.setenv("HC_PHMM_GRID_PLAN", grid)
    regions = [ragged_region(700 + k, nr, nh) for k, (nr, nh) in enumerate([(415, 24), (90, 7), (1, 1), (200, 40)])]
    regions.insert(2, ([], []))
    arr, outs, keep = hcphmm._region_array(regions)
    assert L.hcx_plan_regions(arr, len(regions), 256, 1) >= 0
    pairs, order, n_seg, waves, used_grid = dump(L)
    assert used_grid == int(grid)
    R = np.concatenate([np.repeat([len(r[0]) for r in rd], len(hp)) for rd, hp in regions if rd and hp])
    H = np.concatenate([np.tile([len(h) for h in hp], len(rd)) for rd, hp in regions if rd and hp])
    check_plan(pairs, order, n_seg, waves, R, H)


@pytest.mark.parametrize("wl", ["S1", "S2:20000", "S4"])
def test_flat_plans_are_exact(L, wl):
    name, _, n = wl.partition(":")
    b = W.config(name, int(n) if n else None)
    args, keep = hcphmm._flat_args(b)
    L.hcx_plan_pairs(*args, C.c_int(256), C.c_int(1), C.c_int(1))
    pairs, order, n_seg, waves, used_grid = dump(L)
    assert used_grid == 0
    check_plan(pairs, order, n_seg, waves, b["R"].astype(np.int64), b["H"].astype(np.int64))


def test_region_plan_uses_full_waves(L):
    """The structured plan of a uniform region fills its waves: at most one
    partly filled wave per (hap group)."""
    reads, haps = W.region(415, 128)
    arr, outs, keep = hcphmm._region_array([(reads, haps)])
    L.hcx_plan_regions(arr, 1, 256, 1)
    pairs, order, n_seg, waves, used_grid = dump(L)
    assert used_grid == 1
    lanes = [(-(-pairs[order[s0:s0 + np_], 3] // bc)).sum() for s0, _, _, bc, np_, _ in waves]
    groups = len({(bc, -(-int(pairs[order[s0], 3]) // bc)) for s0, _, _, bc, _, _ in waves})
    assert sum(1 for x in lanes if x + 7 < 64) <= groups


@pytest.mark.parametrize("policy", ["1", "0"])
def test_region_plan_policy_keeps_two_waves_per_simd(L, monkeypatch, policy):
    """planner.cpp grid_policy: a 415 x 32 region's per-hap choice (10 lanes of
    42 columns, 6 pairs per wave) gives 2 214 waves — a third wave on 190 of
    the 1 024 SIMDs; the pass model takes 9 lanes of 48 columns everywhere
    instead (7 pairs per wave, 1 898 waves). HC_PHMM_GRID_POLICY=0 keeps the
    per-hap choice. Either plan must stay exact."""
    monkeypatch.setenv("HC_PHMM_GRID_POLICY", policy)
    reads, haps = W.region(415, 32)
    arr, outs, keep = hcphmm._region_array([(reads, haps)])
    L.hcx_plan_regions(arr, 1, 256, 1)
    pairs, order, n_seg, waves, used_grid = dump(L)
    assert used_grid == 1
    R = np.repeat([len(r[0]) for r in reads], len(haps))
    H = np.tile([len(h) for h in haps], len(reads))
    check_plan(pairs, order, n_seg, waves, R, H)
    if policy == "1":
        assert len(waves) <= 2 * 1024 and set(waves[:, 3]) <= {46, 48}
    else:
        assert len(waves) > 2 * 1024


def test_one_round_plan_is_exact(L):
    """configs[4] (S4: 2 000 waves of unequal length, all resident at once on
    1 024 SIMDs): every pair is in exactly one wave slot, every wave's shape
    covers its pairs (the snake dispatch order that used to be opt-in here
    measured no faster and was removed)."""
    b = W.config("S4")
    args, keep = hcphmm._flat_args(b)
    L.hcx_plan_pairs(*args, C.c_int(256), C.c_int(1), C.c_int(1))
    pairs, order, n_seg, waves, used_grid = dump(L)
    check_plan(pairs, order, n_seg, waves, b["R"].astype(np.int64), b["H"].astype(np.int64))
    assert 1024 < len(waves) <= 3 * 1024


@pytest.mark.parametrize("stage_ps,growth", [(0.0, 1.0), (0.12, 1.3), (0.24, 1.0), (0.2, 1.2), (1.0, 0.8)])
def test_flat_part_growth(L, monkeypatch, stage_ps, growth):
    """A flat call's pipelined parts on one device (api.cpp flat_part_weights):
    growth = device / host staging time per cell, clamped to [0.8, 1.3], none
    before the first measurement, and a part at most 2x (at least 1/2) the
    first; the parts tile the call in order and their cells follow the
    growth within one pair's cells."""
    monkeypatch.delenv("HC_PHMM_PART_GROWTH_PCT", raising=False)
    L.hcx_flat_cuts.restype = C.c_int
    L.hcx_flat_cuts.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_double, C.c_void_p]
    rng = np.random.default_rng(5)
    cells = (rng.integers(50, 251, 200_000) * rng.integers(100, 501, 200_000)).astype(np.int64)
    np_ = 6
    cuts = np.zeros(np_ + 1, np.int64)
    g = L.hcx_flat_cuts(cells.ctypes.data, len(cells), np_, stage_ps, cuts.ctypes.data) / 1000.0
    assert g == pytest.approx(growth, abs=1e-3)
    assert cuts[0] == 0 and cuts[-1] == len(cells) and np.all(np.diff(cuts) > 0)
    pc = np.add.reduceat(cells, cuts[:-1]).astype(float)
    expect = np.clip(growth ** np.arange(np_), 0.5, 2.0)
    expect *= cells.sum() / expect.sum()
    assert np.all(np.abs(pc - expect) <= cells.max()), (pc, expect)


@pytest.mark.parametrize("np_", [40, 4096])
@pytest.mark.parametrize("stage_ps", [0.12, 1.0])
def test_flat_part_growth_many_parts_is_bounded(L, monkeypatch, np_, stage_ps):
    """Many parts (advisor round 5): the growth stops at 2x (or 1/2) the first
    part, so no part is empty, the last part holds a bounded share of the call,
    and 4 096 parts (1.3^4095 would overflow) still tile it in order."""
    monkeypatch.delenv("HC_PHMM_PART_GROWTH_PCT", raising=False)
    L.hcx_flat_cuts.restype = C.c_int
    L.hcx_flat_cuts.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_double, C.c_void_p]
    cells = np.full(np_ * 50, 1000, np.int64)
    cuts = np.zeros(np_ + 1, np.int64)
    L.hcx_flat_cuts(cells.ctypes.data, len(cells), np_, stage_ps, cuts.ctypes.data)
    sizes = np.diff(cuts)
    assert cuts[0] == 0 and cuts[-1] == len(cells) and np.all(sizes > 0)
    assert sizes.max() <= 2 * sizes.min() + 2


def test_flat_part_growth_forced(L, monkeypatch):
    monkeypatch.setenv("HC_PHMM_PART_GROWTH_PCT", "125")
    L.hcx_flat_cuts.restype = C.c_int
    L.hcx_flat_cuts.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_double, C.c_void_p]
    cells = np.full(10_000, 1000, np.int64)
    cuts = np.zeros(5, np.int64)
    assert L.hcx_flat_cuts(cells.ctypes.data, len(cells), 4, 0.0, cuts.ctypes.data) == 1250
    sizes = np.diff(cuts)
    assert np.allclose(sizes[1:] / sizes[:-1], 1.25, atol=0.01)
