"""GPU parity: the HIP engine (through the C ABI) against the reference's golden
vectors and the oracle, bit for bit. Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu

# "diag" = anti-diagonal kernel; "laneN" = lane-per-pair kernel variant N
# with the carry buffer (lane_kernel.hip kVariants: 0 = 64-col blocks 3
# waves/SIMD, 1 = 64-col 2 waves, 2 = 32-col 4 waves);
# "seg" = the default lane path: column-segmented waves (run_seg: a pair over
# ceil(H/BC) lanes, BC per wave) for H <= 1024, one lane per pair above;
# "segall" = every lane pair column-segmented (up to 64 lanes per pair);
# "auto" = the defaults: flat calls planned on the device (flat_plan.cpp),
# prepared batches on the host planner.
KERNELS = ["diag", "lane0", "lane1", "lane2", "seg", "segall", "auto"]


@pytest.fixture(params=KERNELS)
def kernel(request, monkeypatch):
    """Force one fp32 kernel / lane-kernel variant for the test."""
    if request.param == "auto":
        for k in ("HC_PHMM_KERNEL", "HC_PHMM_LANE_SEG", "HC_PHMM_LANE_VARIANT", "HC_PHMM_FLAT_PLAN"):
            monkeypatch.delenv(k, raising=False)
    elif request.param == "diag":
        monkeypatch.setenv("HC_PHMM_KERNEL", "diag")
    elif request.param == "seg":
        monkeypatch.setenv("HC_PHMM_KERNEL", "lane")
        monkeypatch.setenv("HC_PHMM_LANE_SEG", "auto")
    elif request.param == "segall":
        monkeypatch.setenv("HC_PHMM_KERNEL", "lane")
        monkeypatch.setenv("HC_PHMM_LANE_SEG", "all")
    else:
        monkeypatch.setenv("HC_PHMM_KERNEL", "lane")
        monkeypatch.setenv("HC_PHMM_LANE_VARIANT", request.param[4:])
        monkeypatch.setenv("HC_PHMM_LANE_SEG", "off")
    return request.param


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def assert_same(res, ref, what=""):
    """Bit-exact: raw f32, rescue decision, raw f64 of rescued pairs, log10 result."""
    r32 = res["raw_f32"].view(np.uint32) != ref["raw_f32"].view(np.uint32)
    assert not r32.any(), f"{what}: {r32.sum()} raw_f32 mismatches, first {np.nonzero(r32)[0][:10]}"
    assert np.array_equal(res["rescued"], ref["rescued"]), what
    m = ref["rescued"].astype(bool)
    r64 = res["raw_f64"][m].view(np.uint64) != ref["raw_f64"][m].view(np.uint64)
    assert not r64.any(), f"{what}: {r64.sum()} raw_f64 mismatches"
    ll = res["loglik"].view(np.uint64) != ref["loglik"].view(np.uint64)
    assert not ll.any(), f"{what}: {ll.sum()} loglik mismatches"


def test_golden_bit_exact(engine, kernel, golden, golden_batch):
    res = engine.pairs(golden_batch)
    ref = dict(raw_f32=golden["raw_f32"], rescued=golden["rescued"],
               raw_f64=golden["raw_f64_all"], loglik=golden["loglik"])
    names = list(golden["set_names"])
    for k, name in enumerate(names):
        idx = golden["set_id"] == k
        assert_same({x: res[x][idx] for x in res}, {x: ref[x][idx] for x in ref}, f"{kernel}/{name}")


def test_golden_f64_path_on_every_pair(engine, golden, golden_batch):
    """Force the fp64 kernel onto pairs that do not need rescue by re-running the
    underflow set alone (all rescued) and the edge set's rescued pairs."""
    names = list(golden["set_names"])
    idx = np.nonzero(golden["rescued"].astype(bool))[0]
    sub = W.subset(golden_batch, idx)
    res = engine.pairs(sub)
    assert res["rescued"].all()
    assert np.array_equal(bits(res["raw_f64"]), bits(golden["raw_f64_all"][idx]))
    assert "underflow" in names


def test_s1_full_vs_oracle(engine, kernel, oracle_lib):
    b = W.config("S1")
    res = engine.pairs(b)
    ref = oracle_lib.pairs(b, nthreads=16)
    assert_same(res, ref, "S1")


def test_s1w_full_vs_oracle(engine, oracle_lib):
    """The north star's 101 x 250 shape (S1w: configs[1]'s 10k pairs with the
    250-base haps BASELINE.json's north_star names), the whole batch against
    the oracle, flat call and a prepared batch run twice."""
    b = W.config("S1w")
    assert (b["R"] == 101).all() and (b["H"] == 250).all() and len(b["R"]) == 10_000
    ref = oracle_lib.pairs(b, nthreads=16)
    assert_same(engine.pairs(b), ref, "S1w flat")
    bt = engine.Batch(b)
    for k in range(2):
        bt.run()
        assert_same(bt.results(), ref, f"S1w batch run {k}")
    bt.close()


def test_s2_sample_vs_oracle(engine, kernel, oracle_lib):
    b = W.config("S2", 20_000)
    res = engine.pairs(b)
    ref = oracle_lib.pairs(b, nthreads=16)
    assert_same(res, ref, "S2-20k")


def test_s4_sample_vs_oracle(engine, oracle_lib):
    b = W.subset(W.config("S4"), np.arange(200))
    res = engine.pairs(b)
    ref = oracle_lib.pairs(b, nthreads=16)
    assert res["rescued"].sum() > 100
    assert_same(res, ref, "S4-200")


def test_mixed_lengths_share_waves(engine, kernel, oracle_lib):
    """Pairs of very different R/H packed into the same waves (both W classes)."""
    b = W.generate(3000, (1, 1200), (1, 300), 0.05, seed=5)
    res = engine.pairs(b)
    ref = oracle_lib.pairs(b, nthreads=16)
    assert_same(res, ref, "mixed")


def test_batch_rerun_is_deterministic(engine, kernel):
    b = W.config("S2", 50_000)
    bt = engine.Batch(b)
    bt.run()
    r1 = bt.results()
    bt.run()
    r2 = bt.results()
    st = bt.stats()
    assert st.n_pairs == 50_000 and st.cells == W.cells(b)
    assert st.n_rescued == int(r1["rescued"].sum())
    for k in r1:
        assert np.array_equal(bits(r1[k]), bits(r2[k])), k
    assert np.isfinite(r1["loglik"]).all()
    bt.close()


def test_cross_and_compute_likelihoods(engine, kernel, oracle_lib):
    """Region-shaped call: every read against every hap (intel_pairhmm.hpp:48-56)."""
    rng = np.random.default_rng(3)
    haps = []
    base = W.ACGT[rng.integers(0, 4, 400)]
    for k in range(6):
        h = base.copy()
        h[rng.integers(0, 400, 3)] = W.ACGT[rng.integers(0, 4, 3)]
        haps.append(h.tobytes())
    reads = []
    for k in range(40):
        o = int(rng.integers(0, 250))
        rs = np.frombuffer(haps[k % 6], np.uint8)[o:o + 150].copy()
        if k % 9 == 0:
            rs[:] = W.ACGT[rng.integers(0, 4, 150)]          # junk read -> filtered
        q = (rng.integers(10, 41, 150) + 33).astype(np.uint8).tobytes()
        reads.append((rs.tobytes(), q, b"I" * 150, b"I" * 150, b"+" * 150))
    L = engine.cross(reads, haps)
    flat = W.from_pairs([(r[0], r[1], r[2], r[3], r[4], h) for r in reads for h in haps])
    ref = oracle_lib.pairs(flat, nthreads=16)["loglik"].reshape(len(reads), len(haps))
    assert np.array_equal(bits(L), bits(ref))
    Ln, kept = engine.compute_likelihoods(haps, reads)
    refn, keep = oracle_lib.normalize(ref, np.full(len(reads), 150, np.int32))
    assert len(kept) == int(keep.sum()) < len(reads)
    assert np.array_equal(bits(Ln), bits(refn[keep]))


def test_edge_contract(engine, oracle_lib):
    empty = engine.cross([], [b"ACGT"])
    assert empty.shape == (0, 1)
    with pytest.raises(engine.PairHMMError) as e:
        engine.cross([(b"", b"", b"", b"", b"")], [b"ACGT"])
    assert e.value.code == engine.EINVAL
    # Haps past the anti-diagonal kernel's LDS ring (the reference has no hap
    # length limit: its stripe carries are VLAs, avx-pairhmm-template.h:224)
    # run with the ring in HBM.
    reads = [(b"A", b"I", b"I", b"I", b"+"), (b"ACGTN" * 30, b"5" * 150, b"I" * 150, b"I" * 150, b"+" * 150)]
    haps = [b"A" * 9000, (b"ACGT" * 3000)[:12000]]
    got = engine.cross(reads, haps)
    flat = W.from_pairs([(r[0], r[1], r[2], r[3], r[4], h) for r in reads for h in haps])
    ref = oracle_lib.pairs(flat, nthreads=16)["loglik"].reshape(2, 2)
    assert np.array_equal(bits(got), bits(ref))
    with pytest.raises(engine.PairHMMError) as e:
        engine.cross([(b"A", b"I", b"I", b"I", b"+")], [b"A" * 262145])
    assert e.value.code == engine.EINVAL


def test_s2_full_size_properties(engine):
    """BASELINE configs[2] at full size (1M pairs, lane kernel): every result finite,
    rescue rate tiny, rerun bit-identical, and a 2 000-pair sample equal to the
    oracle bit for bit."""
    import oracle
    b = W.config("S2")
    bt = engine.Batch(b)
    bt.run()
    r1 = bt.results()
    bt.run()
    r2 = bt.results()
    assert np.array_equal(bits(r1["loglik"]), bits(r2["loglik"]))
    assert np.isfinite(r1["loglik"]).all()
    assert r1["rescued"].sum() < 200
    idx = np.random.default_rng(0).choice(len(b["R"]), 2000, replace=False)
    ref = oracle.Oracle().pairs(W.subset(b, idx), nthreads=16)
    assert_same({k: r1[k][idx] for k in r1}, ref, "S2-full-sample")
    bt.close()


def test_cross_regions_matches_per_region_calls(engine):
    """Cross-region batching returns exactly what one call per region returns."""
    regions = [W.region(n_reads=int(nr), n_haps=int(nh), seed=100 + k)
               for k, (nr, nh) in enumerate([(50, 2), (120, 8), (0, 3), (415, 32), (7, 1)])]
    together = engine.cross_regions(regions)
    for (reads, haps), got in zip(regions, together):
        if not reads:
            assert got.shape == (0, len(haps))
            continue
        alone = engine.cross(reads, haps)
        assert np.array_equal(bits(got), bits(alone))


def test_auto_segmentation_on_a_shard(engine, oracle_lib, monkeypatch):
    """A 125k-pair S2 shard (one rank's share of configs[3] at 8 GPUs): the
    engine column-segments every pair (ceil(H/BC) lanes per pair). Same
    arithmetic in the same order as one lane per pair with the carry buffer,
    so the whole shard is bit-identical to the unsegmented run, and a sample
    equals the oracle."""
    b = W.config("S2", 125_000)
    bt = engine.Batch(b)
    bt.run()
    seg = bt.results()
    st = bt.stats()
    bt.close()
    assert st.n_lane_pairs == 125_000 and st.n_seg_waves > 0
    monkeypatch.setenv("HC_PHMM_LANE_SEG", "off")
    bt = engine.Batch(b)
    bt.run()
    one = bt.results()
    assert bt.stats().n_seg_waves == 0
    bt.close()
    for k in seg:
        assert np.array_equal(bits(seg[k]), bits(one[k])), k
    idx = np.random.default_rng(1).choice(125_000, 3000, replace=False)
    assert_same({k: seg[k][idx] for k in seg}, oracle_lib.pairs(W.subset(b, idx), nthreads=16), "shard")


@pytest.mark.parametrize("gaps", ["eq", "cg", "per_base"])
@pytest.mark.parametrize("seg", ["auto", "all"])
def test_seg_widths_and_gap_modes(engine, oracle_lib, monkeypatch, gaps, seg):
    """Column-segmented waves over every compiled block width (H 10..1100 puts
    pairs on BC 16..64 and 1..18 lanes) and the three cell paths: equal
    constant gap qualities (the reference's 'I'/'I'/'+', EQ path: M*mx shared
    with the next column's M*my), constant but unequal (CG path) and per-base
    gap qualities (generic path). Bit-exact against the oracle."""
    monkeypatch.setenv("HC_PHMM_KERNEL", "lane")
    monkeypatch.setenv("HC_PHMM_LANE_SEG", seg)
    b = W.generate(6000, (10, 1100), (5, 250), 0.02, seed=11)
    rng = np.random.default_rng(5)
    n = len(b["ins"])
    if gaps == "cg":
        b["ins"][:] = 40 + 33
        b["dels"][:] = 25 + 33
        b["gcp"][:] = 12 + 33
    elif gaps == "per_base":
        b["ins"][:] = rng.integers(33 + 5, 33 + 60, n, dtype=np.uint8)
        b["dels"][:] = rng.integers(33 + 5, 33 + 60, n, dtype=np.uint8)
        b["gcp"][:] = rng.integers(33 + 5, 33 + 30, n, dtype=np.uint8)
    bt = engine.Batch(b)
    bt.run()
    res = bt.results()
    st = bt.stats()
    bt.close()
    assert st.n_seg_waves > 0
    assert_same(res, oracle_lib.pairs(b, nthreads=16), f"seg={seg}/{gaps}")


@pytest.mark.parametrize("gaps", ["eq", "per_base"])
@pytest.mark.parametrize("cap", [8, 10, 12, 14])
def test_narrow_seg_widths(engine, oracle_lib, monkeypatch, gaps, cap):
    """The narrow block widths small batches use (BC 8-14: up to 64 lanes per
    pair, R + 63 steps) forced through the width cap, bit-exact against the
    oracle on both cell paths."""
    monkeypatch.setenv("HC_PHMM_SEG_CAP", str(cap))
    b = W.generate(3000, (10, 900), (5, 250), 0.02, seed=12 + cap)
    if gaps == "per_base":
        rng = np.random.default_rng(cap)
        n = len(b["ins"])
        b["ins"][:] = rng.integers(33 + 5, 33 + 60, n, dtype=np.uint8)
        b["dels"][:] = rng.integers(33 + 5, 33 + 60, n, dtype=np.uint8)
        b["gcp"][:] = rng.integers(33 + 5, 33 + 30, n, dtype=np.uint8)
    assert_same(engine.pairs(b), oracle_lib.pairs(b, nthreads=16), f"cap={cap}/{gaps}")


def test_repeated_runs_reuse_rescue_counters(engine, oracle_lib):
    """A prepared batch run many times: the fp32 pass appends to one of two
    rescue counters by run parity and the rescue pass zeroes the other for the
    next run (no memset per run); every run gives the same bits and count."""
    b = W.generate(300, (1000, 1400), (150, 250), 0.08, seed=3)
    ref = oracle_lib.pairs(b, nthreads=16)
    bt = engine.Batch(b)
    for _ in range(5):
        bt.run()
        assert_same(bt.results(), ref, "repeat")
        assert bt.stats().n_rescued == int(ref["rescued"].sum()) > 0
    bt.close()


@pytest.mark.parametrize("in_wave", ["on", "off"])
@pytest.mark.parametrize("shape", ["short_list", "mid_list", "long_list", "wide_haps"])
def test_fp64_rescue_tiers(engine, oracle_lib, monkeypatch, shape, in_wave):
    """The fp64 rescue pass is planned on the device: block width 8 / 16 / 32
    by rescue-list size (a short list is latency-bound), pairs binned into
    2^k-lane classes, haps too wide for 64 blocks of 32 on the anti-diagonal
    fp64 kernel. High substitution rates force most pairs into rescue. With
    in_wave on, fp32 waves holding one or two rescued pairs (H <= 512)
    recompute them themselves (short_list is mostly that path)."""
    monkeypatch.setenv("HC_PHMM_RESCUE_IN_WAVE", "0" if in_wave == "off" else "1")
    n, h, r = {"short_list": (40, (300, 900), (100, 250)),
               "mid_list": (1500, (600, 1100), (150, 250)),
               "long_list": (4500, (1000, 1200), (150, 250)),
               "wide_haps": (60, (1800, 3000), (150, 250))}[shape]
    b = W.generate(n, h, r, 0.08, seed=17)
    ref = oracle_lib.pairs(b, nthreads=16)
    assert ref["rescued"].sum() > n // 2
    res = engine.pairs(b)
    assert_same(res, ref, shape)


def test_fp64_rescue_s4_20k(engine, oracle_lib):
    """configs[4] at the 20 000 pairs SURVEY §8(d) also names: a rescue list
    long enough to fill the chip many times over (dynamic longest-first wave
    fetch, widest classes). A rerun gives the same bits and a sample equals
    the oracle."""
    b = W.config("S4", 20_000)
    bt = engine.Batch(b)
    bt.run()
    res = bt.results()
    bt.run()
    again = bt.results()
    bt.close()
    for k in res:
        assert np.array_equal(bits(res[k]), bits(again[k])), k
    m = res["rescued"].astype(bool)
    assert m.sum() > 15_000
    idx = np.random.default_rng(31).choice(20_000, 300, replace=False)
    assert_same({k: res[k][idx] for k in res}, oracle_lib.pairs(W.subset(b, idx), nthreads=16), "S4-20k")


def test_in_wave_rescue_on_s2_shard(engine, oracle_lib):
    """S2's rare rescues (a 125k-pair shard: about two) are recomputed inside
    the fp32 pass by the waves that flag them: every rescued pair, plus a
    sample, equals the oracle; the in-wave cap forces the rest to the list."""
    b = W.config("S2", 125_000)
    res = engine.pairs(b)
    resc = np.flatnonzero(res["rescued"])
    assert len(resc) > 0
    idx = np.union1d(resc, np.random.default_rng(3).choice(125_000, 500, replace=False))
    assert_same({k: res[k][idx] for k in res}, oracle_lib.pairs(W.subset(b, idx), nthreads=16), "S2 in-wave")


def test_in_wave_rescue_cap(engine, oracle_lib, monkeypatch):
    """With the per-run cap at 1 only the first flagged pair is recomputed in
    its wave; the others go through the rescue list. Same bits either way,
    and the rescue count is exact."""
    monkeypatch.setenv("HC_PHMM_RESCUE_IN_WAVE_MAX", "1")
    b = W.generate(200, (200, 700), (100, 250), 0.08, seed=23)
    ref = oracle_lib.pairs(b, nthreads=16)
    bt = engine.Batch(b)
    bt.run()
    assert_same(bt.results(), ref, "cap 1")
    assert bt.stats().n_rescued == int(ref["rescued"].sum()) > 2
    bt.close()


@pytest.mark.parametrize("n", [1, 37, 125_000])
def test_flat_device_planner_matches_host_planner(engine, oracle_lib, monkeypatch, n):
    """Flat calls are planned on the device (pack, cost model, counting sort,
    waves: flat_plan.cpp + pack_kernels.hip flat_*); the host planner
    (HC_PHMM_FLAT_PLAN=0) must give the same bits, and a sample the oracle's."""
    b = W.config("S2", n)
    dev = engine.pairs(b)
    monkeypatch.setenv("HC_PHMM_FLAT_PLAN", "0")
    host = engine.pairs(b)
    for k in dev:
        assert np.array_equal(bits(dev[k]), bits(host[k])), k
    idx = np.random.default_rng(9).choice(n, min(n, 2000), replace=False)
    assert_same({k: dev[k][idx] for k in dev}, oracle_lib.pairs(W.subset(b, idx), nthreads=16), f"flat n={n}")


def test_flat_device_planner_ragged_and_long(engine, oracle_lib):
    """Device planning over a ragged mix: reads 1-600, haps 1-4096 (every
    width and lane count, coarsened R bins), per-base gap qualities on a third
    of the reads; and a batch with a hap past 4096 that the host planner takes."""
    b = W.generate(4000, (1, 4096), (1, 600), 0.03, seed=77)
    rng = np.random.default_rng(8)
    rows = np.repeat(np.arange(4000) % 3 == 1, b["R"])
    m = int(rows.sum())
    b["ins"][rows] = rng.integers(33 + 5, 33 + 60, m, dtype=np.uint8)
    b["dels"][rows] = rng.integers(33 + 5, 33 + 60, m, dtype=np.uint8)
    b["gcp"][rows] = rng.integers(33 + 5, 33 + 30, m, dtype=np.uint8)
    assert_same(engine.pairs(b), oracle_lib.pairs(b, nthreads=16), "ragged")
    c = W.generate(300, (3000, 6000), (50, 200), 0.02, seed=78)
    assert_same(engine.pairs(c), oracle_lib.pairs(c, nthreads=16), "long haps")


def test_use_double_every_golden_pair(engine, golden, golden_batch):
    """initNative(use_double = true) (intel_pairhmm.hpp:71,81,135-140) through
    hc_phmm_init(HC_PHMM_FLAG_F64): result_float = 0 for every pair, so every
    pair's fp64 sum must equal the reference's double kernel on that pair
    (golden raw_f64_all, computed for every pair) bit for bit, and the
    likelihood is glibc log10(raw_f64) - log10(2^1020) — on the flat device
    planner, the host planner and a prepared batch."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.log10.restype = ctypes.c_double
    libm.log10.argtypes = [ctypes.c_double]
    l10 = libm.log10(2.0 ** 1020)
    exp64 = golden["raw_f64_all"]
    exp_ll = np.array([libm.log10(float(x)) - l10 for x in exp64])
    engine.init(0, use_double=True)
    try:
        runs = {"flat": engine.pairs(golden_batch)}
        import os
        os.environ["HC_PHMM_FLAT_PLAN"] = "0"
        try:
            runs["host"] = engine.pairs(golden_batch)
        finally:
            del os.environ["HC_PHMM_FLAT_PLAN"]
        bt = engine.Batch(golden_batch)
        bt.run()
        runs["batch"] = bt.results()
        bt.close()
    finally:
        engine.init(0, use_double=False)
    for name, res in runs.items():
        assert (res["raw_f32"] == 0).all(), name
        assert res["rescued"].all(), name
        d = res["raw_f64"].view(np.uint64) != exp64.view(np.uint64)
        assert not d.any(), f"{name}: {d.sum()} raw_f64 mismatches, first {np.nonzero(d)[0][:10]}"
        ll = res["loglik"].view(np.uint64) != exp_ll.view(np.uint64)
        assert not ll.any(), f"{name}: {ll.sum()} loglik mismatches"
    # and the default mode is back: the fp32 pass decides again
    res = engine.pairs(golden_batch)
    assert np.array_equal(res["rescued"], golden["rescued"])


@pytest.mark.parametrize("variant", ["prio32", "prio64-off", "records"])
def test_schedule_variants_are_bit_identical(engine, golden, golden_batch, variant, monkeypatch):
    """How waves are scheduled never changes a result: the issue-priority
    switches and per-slot records give the default's bits on a 125k-pair S2
    shard (more waves than wave slots) run twice (the counters it zeroes for
    the next run), and on the golden set."""
    env = {"prio32": ("HC_PHMM_PRIO", "1"), "prio64-off": ("HC_PHMM_PRIO64", "0"),
           "records": ("HC_PHMM_REC_MIN_PAIRS", "0")}[variant]
    b = W.config("S2", 125_000)
    ref = engine.pairs(b)
    bt_ref = engine.Batch(b)
    bt_ref.run()
    rb = bt_ref.results()
    bt_ref.close()
    monkeypatch.setenv(*env)
    bt = engine.Batch(b)
    for _ in range(2):   # the second run checks the counters the first one left
        bt.run()
        got = bt.results()
        for k in ("raw_f32", "raw_f64", "rescued", "loglik"):
            assert np.array_equal(bits(got[k]), bits(rb[k])), f"{variant}: {k}"
    bt.close()
    assert_same(engine.pairs(b), ref, f"{variant} flat")
    res = engine.pairs(golden_batch)
    assert_same(res, dict(raw_f32=golden["raw_f32"], rescued=golden["rescued"],
                          raw_f64=golden["raw_f64_all"], loglik=golden["loglik"]), f"{variant} golden")


@pytest.mark.parametrize("solo", ["on", "off"])
def test_small_part_rescues_in_its_waves(engine, oracle_lib, monkeypatch, solo):
    """A small part of seg waves whose haps all fit one wave's fp64 reach
    (H <= 512) launches no fp64 pass: each wave rescues every pair it flagged
    (run.cpp `solo`, HC_PHMM_SOLO_MAX_PAIRS). A rescue-heavy batch (most pairs,
    many per wave) against the oracle, flat and through one prepared batch run
    three times (the seg kernel zeroes the other run parity's counters in
    place of the fp64 launch); off: the same batch through the list."""
    if solo == "off":
        monkeypatch.setenv("HC_PHMM_SOLO_MAX_PAIRS", "0")
    b = W.generate(3000, (100, 500), (60, 200), 0.08, seed=23)
    ref = oracle_lib.pairs(b, nthreads=16)
    n_resc = int(ref["rescued"].sum())
    assert n_resc > 1000
    assert_same(engine.pairs(b), ref, f"solo {solo} flat")
    bt = engine.Batch(b)
    for k in range(3):
        bt.run()
        got = bt.results()
        assert_same(got, ref, f"solo {solo} run {k}")
        assert (got["raw_f64"][~ref["rescued"].astype(bool)] == 0).all()
    assert bt.stats().n_rescued == n_resc
    bt.close()


@pytest.mark.parametrize("mode", ["list", "records"])
def test_rescue_heavy_part(engine, oracle_lib, monkeypatch, mode):
    """Rescues a seg wave defers (past the in-wave limits) go to the fp64
    launch's list. A batch above the solo size with most pairs rescued (H
    100-900), three runs through one prepared batch (the counters go by run
    parity), against the oracle; with per-slot records (the in-wave rescues
    write their pair's raw f64 into the record) and without."""
    if mode == "records":
        monkeypatch.setenv("HC_PHMM_REC_MIN_PAIRS", "0")
    b = W.generate(40000, (100, 900), (60, 200), 0.08, seed=29)
    ref = oracle_lib.pairs(b, nthreads=16)
    n_resc = int(ref["rescued"].sum())
    assert n_resc > 15000
    bt = engine.Batch(b)
    for k in range(3):
        bt.run()
        got = bt.results()
        assert_same(got, ref, f"{mode} run {k}")
        assert (got["raw_f64"][~ref["rescued"].astype(bool)] == 0).all()
    assert bt.stats().n_rescued == n_resc
    bt.close()
    assert_same(engine.pairs(b), ref, f"{mode} flat")


@pytest.mark.parametrize("mode", ["auto", "lane"])
def test_seg_records_and_gather_with_mixed_kernels(engine, oracle_lib, monkeypatch, mode):
    """The fp32 seg waves write per-slot records that the fp64 launch gathers
    into the per-pair outputs (slot_of); pairs of the one-lane and anti-
    diagonal kernels write theirs in place (slot_of = -1). A batch of haps up
    to 6 000 bases (some rescued) split between the seg waves and the anti-
    diagonal kernel (auto: haps past 64 x 64 columns) or the one-lane kernel
    (lane: past the seg reach), against the oracle, with outputs bound to
    caller buffers and run twice."""
    import torch
    if mode == "lane":
        monkeypatch.setenv("HC_PHMM_KERNEL", "lane")
        monkeypatch.setenv("HC_PHMM_LANE_SEG", "auto")
    monkeypatch.setenv("HC_PHMM_REC_MIN_PAIRS", "0")   # records at any size (default: large parts only)
    b = W.generate(600, (100, 6000), (60, 250), 0.03, seed=91)
    ref = oracle_lib.pairs(b, nthreads=16)
    bt = engine.Batch(b)
    n = len(b["R"])
    out32 = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
    out64 = torch.full((n,), float("nan"), dtype=torch.float64, device="cuda")
    outfl = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    bt.bind_outputs(out32.data_ptr(), out64.data_ptr(), outfl.data_ptr())
    for _ in range(2):
        bt.run()
        torch.cuda.synchronize()
        got = dict(raw_f32=out32.cpu().numpy(), raw_f64=out64.cpu().numpy(), rescued=outfl.cpu().numpy())
        r32 = got["raw_f32"].view(np.uint32) != ref["raw_f32"].view(np.uint32)
        assert not r32.any(), f"{r32.sum()} raw_f32 mismatches"
        assert np.array_equal(got["rescued"], ref["rescued"])
        m = ref["rescued"].astype(bool)
        assert np.array_equal(bits(got["raw_f64"][m]), bits(ref["raw_f64"][m]))
        assert (got["raw_f64"][~m] == 0).all()
    st = bt.stats()
    assert 0 < st.n_seg_waves   # seg waves ran ...
    assert st.n_lane_pairs < st.n_pairs if mode == "auto" else st.n_launch_waves > st.n_seg_waves   # ... and another kernel
    bt.close()


@pytest.mark.parametrize("plan", ["static", "dynamic"])
def test_rescue_plan_timeout_is_an_error(engine, oracle_lib, monkeypatch, plan):
    """A fp64 workgroup that gives up waiting for the device-made rescue plan
    (lane_kernel.hip phmm_seg64_kernel, bounded wait) sets the part's device
    error word, and the call fails with HC_PHMM_EHIP instead of returning
    results (verdict round 4). The test-only entry point hcx_test_plan_timeout
    (no environment variable: the release library never reads one for it)
    makes every non-planner workgroup time out at once: a static plan (S4-200:
    fewer waves than two per SIMD) and a dynamic one (thousands of long
    rescued pairs), through a flat call and a prepared batch; the batch then
    runs correctly once the hook is off (the error word is cleared when
    reported)."""
    import hcphmm
    if plan == "static":
        b = W.subset(W.config("S4"), np.arange(200))
    else:
        b = W.generate(4000, (1000, 1500), (150, 250), 0.08, seed=71)
    ref = oracle_lib.pairs(b, nthreads=16)
    assert ref["rescued"].sum() > (3000 if plan == "dynamic" else 100)
    bt = engine.Batch(b)
    L = hcphmm.lib()
    monkeypatch.setenv("HC_PHMM_TEST_PLAN_TIMEOUT", "1")   # (ignored: no release path reads it)
    assert_same(engine.pairs(b), ref, f"{plan}: env var ignored")
    L.hcx_test_plan_timeout(1)
    try:
        with pytest.raises(hcphmm.PairHMMError) as e:
            engine.pairs(b)
        assert e.value.code == hcphmm.EHIP and "rescue plan" in str(e.value)
        bt.run()
        with pytest.raises(hcphmm.PairHMMError) as e:
            bt.results()
        assert e.value.code == hcphmm.EHIP
    finally:
        L.hcx_test_plan_timeout(0)
    bt.run()
    assert_same(bt.results(), ref, f"{plan}: after the hook")
    bt.close()
    assert_same(engine.pairs(b), ref, f"{plan}: flat after the hook")


def test_mode_is_per_call_and_fixed_at_submit(engine, golden, golden_batch):
    """initNative's use_double is per IntelPairHMM instance in the reference
    (intel_pairhmm.hpp:58,81): hc_phmm_cross_ex / compute_likelihoods_ex take
    the mode per call whatever the process default is, and a batch keeps the
    mode it was created with when the default changes later (advisor round 4)."""
    # a small region of S1-shaped reads x haps: the fp32 / fp64 modes differ
    b = W.config("S1", 64)
    reads = [(bytes(b["rs"][o:o + r]), bytes(b["q"][o:o + r]), bytes(b["ins"][o:o + r]),
              bytes(b["dels"][o:o + r]), bytes(b["gcp"][o:o + r])) for o, r in zip(b["read_off"][:8], b["R"][:8])]
    haps = [bytes(b["hap"][o:o + h]) for o, h in zip(b["hap_off"][:4], b["H"][:4])]
    f32 = engine.cross(reads, haps)
    bt = engine.Batch(golden_batch)   # created in fp32 mode
    engine.init(0, use_double=True)
    try:
        assert np.array_equal(bits(engine.cross(reads, haps, use_double=False)), bits(f32))
        f64 = engine.cross(reads, haps)   # process default: fp64 only
        assert not np.array_equal(bits(f64), bits(f32))
        bt.run()
        got = bt.results()
        assert np.array_equal(got["rescued"], golden["rescued"])   # still the fp32 pass deciding
        assert np.array_equal(bits(got["raw_f32"]), bits(golden["raw_f32"]))
    finally:
        engine.init(0, use_double=False)
        bt.close()
    assert np.array_equal(bits(engine.cross(reads, haps, use_double=True)), bits(f64))
    L, kept = engine.compute_likelihoods(haps, reads, use_double=True)
    assert L.shape[1] == len(haps) and len(kept) == L.shape[0]


@pytest.mark.parametrize("shape", ["S4", "S4-300", "many-per-wave", "short-haps", "big-narrow"])
def test_rescue_shapes(engine, oracle_lib, shape):
    """Rescue-heavy parts through the default schedule (the fp64 launch after
    the fp32 pass, or the solo path for small parts of short haps):
    configs[4] (S4, 2 000 pairs, 93 % rescued) and a subset; 8 000 pairs of
    520-700 bases four to a wave, most rescued; short haps (the solo path); a
    60k-pair part of 300-500-base haps (more waves than slots). Flat call and
    a prepared batch run three times (the counters go by run parity), against
    the oracle; the rescued count is the oracle's. (These were the fused
    pass's cases; that opt-in schedule measured slower and was removed,
    DESIGN.md §16.1.)"""
    b = {"S4": lambda: W.config("S4"),
         "S4-300": lambda: W.subset(W.config("S4"), np.arange(300)),
         "many-per-wave": lambda: W.generate(8000, (520, 700), (60, 200), 0.08, seed=41),
         "short-haps": lambda: W.generate(3000, (100, 500), (60, 200), 0.08, seed=23),
         "big-narrow": lambda: W.generate(60000, (300, 500), (60, 200), 0.035, seed=43)}[shape]()
    ref = oracle_lib.pairs(b, nthreads=16)
    n_resc = int(ref["rescued"].sum())
    assert n_resc > (500 if shape == "big-narrow" else len(b["R"]) // 3)
    assert_same(engine.pairs(b), ref, f"{shape} flat")
    bt = engine.Batch(b)
    for k in range(3):
        bt.run()
        got = bt.results()
        assert_same(got, ref, f"{shape} run {k}")
        assert (got["raw_f64"][~ref["rescued"].astype(bool)] == 0).all()
    st = bt.stats()
    assert st.n_rescued == n_resc
    bt.close()


@pytest.mark.parametrize("case", ["long-haps", "mixed-reads", "short-reads", "long-haps-chained",
                                  "mixed-reads-chained", "short-reads-chained", "long-haps-chain2"])
def test_fp64_long_haps_many_waves(engine, oracle_lib, monkeypatch, case):
    """An fp64 pass of many waves over long haps: 4 000 pairs of 1 025-2 048-
    base haps, most rescued, so the plan sorts thousands of 64-lane waves and
    dispatches them greedily from the wave counter (more than two waves per
    SIMD) — against the oracle, flat and through a prepared batch run twice.
    mixed-reads: some reads with an 'N' base, some with insertion != deletion
    gap qualities and a hap with an 'N'; short-reads: R 40-639 (a chain's
    windows of last rows overlap). -chained: every 64-lane pair chained
    (HC_PHMM_CHAIN_TAIL=0; by default only passes past two rounds of single
    waves chain), up to 4 pairs a wave through the same lanes (lane_kernel.hip
    chain_run; a chain holding a non-EQ read or other gap constants runs its
    pairs one by one); -chain2: chains of 2."""
    if case.endswith("-chained") or case.endswith("-chain2"):
        monkeypatch.setenv("HC_PHMM_CHAIN_TAIL", "0")
    if case.endswith("-chain2"):
        monkeypatch.setenv("HC_PHMM_CHAIN", "2")
    case = case.replace("-chained", "").replace("-chain2", "")
    r_range = (40, 639) if case == "short-reads" else (150, 250)
    b = W.generate(4000, (1025, 2048), r_range, 0.08, seed=97)
    if case == "mixed-reads":
        rs, dels, hap = b["rs"].copy(), b["dels"].copy(), b["hap"].copy()
        ro = b["read_off"]
        for p in range(0, 4000, 37):
            rs[ro[p] + 5] = ord("N")
        for p in range(3, 4000, 53):
            dels[ro[p]:ro[p] + b["R"][p]] = ord("J")   # constant gaps, insertion != deletion
        ins = b["ins"].copy()
        for p in range(5, 4000, 61):   # EQ reads with other gap constants than the rest
            ins[ro[p]:ro[p] + b["R"][p]] = ord("J")
            dels[ro[p]:ro[p] + b["R"][p]] = ord("J")
        hap[b["hap_off"][11] + 100] = ord("N")
        b = dict(b, rs=rs, ins=ins, dels=dels, hap=hap)
    ref = oracle_lib.pairs(b, nthreads=16)
    assert ref["rescued"].sum() > 3000
    assert_same(engine.pairs(b), ref, f"{case} flat")
    bt = engine.Batch(b)
    for k in range(2):
        bt.run()
        assert_same(bt.results(), ref, f"{case} run {k}")
    bt.close()
