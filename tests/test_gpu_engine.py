"""GPU: the engine around the kernels — several device slots in one process,
parts and chunks, the asynchronous submit / collect calls, cross-region
batching — bit for bit against the oracle and the golden vectors. On the
1-GPU box a device list [0, 0] gives two slots (two streams, two workspaces)
on one GPU, which exercises every sharding path the 8-GPU node uses."""
import numpy as np
import pytest

import workloads as W
from test_gpu_parity import assert_same, bits

pytestmark = pytest.mark.gpu


@pytest.fixture
def two_slots(engine):
    """The engine on device slots [0, 0]; restored to [0] afterwards."""
    engine.shutdown()
    engine.init_devices([0, 0])
    try:
        yield engine
    finally:
        engine.shutdown()
        engine.init(0)


@pytest.fixture
def many_parts(monkeypatch):
    """Split even small calls into several parts (shards x chunks)."""
    monkeypatch.setenv("HC_PHMM_SHARD_MIN_CELLS", "0")
    monkeypatch.setenv("HC_PHMM_CHUNK_CELLS", "20000000")


def golden_ref(golden):
    return dict(raw_f32=golden["raw_f32"], rescued=golden["rescued"],
                raw_f64=golden["raw_f64_all"], loglik=golden["loglik"])


def test_init_rejects_a_different_device(two_slots):
    assert two_slots.device_count() == 2
    with pytest.raises(two_slots.PairHMMError) as e:
        two_slots.init(0)        # engine runs on [0, 0]: naming [0] is a different selection
    assert e.value.code == two_slots.EINVAL
    two_slots.init(-1)           # -1: whatever the engine runs on
    two_slots.init_devices([0, 0])


def test_two_slots_golden(two_slots, golden, golden_batch, many_parts):
    res = two_slots.pairs(golden_batch)
    assert_same(res, golden_ref(golden), "golden on [0,0]")


def test_two_slots_s2_shard_vs_oracle(two_slots, oracle_lib):
    """A 125k-pair S2 shard (one rank's share of configs[3] at 8 GPUs) split over
    two device slots by cells: a 3 000-pair sample equals the oracle, and the
    whole shard equals the single-slot run."""
    b = W.config("S2", 125_000)
    res = two_slots.pairs(b)
    idx = np.random.default_rng(2).choice(125_000, 3000, replace=False)
    assert_same({k: res[k][idx] for k in res}, oracle_lib.pairs(W.subset(b, idx), nthreads=16), "S2-125k [0,0]")
    bt = two_slots.Batch(b)
    st0 = bt.stats()
    assert st0.n_devices == 2 and st0.pack_ms > 0 and st0.upload_bytes > 0
    bt.run()
    r2 = bt.results()
    st = bt.stats()
    bt.close()
    assert st.n_pairs == 125_000 and st.cells == W.cells(b) and st.n_runs == 1
    for k in res:
        assert np.array_equal(bits(res[k]), bits(r2[k])), k


def test_parts_and_chunks_are_exact(engine, oracle_lib, many_parts):
    """One call cut into many contiguous parts (chunks on one slot) gives the
    same bits as the oracle."""
    b = W.generate(4000, (50, 900), (20, 250), 0.03, seed=21)
    assert_same(engine.pairs(b), oracle_lib.pairs(b, nthreads=16), "chunked")


def test_async_jobs_collected_out_of_order(engine, oracle_lib):
    batches = [W.generate(1500 + 500 * k, (100, 600), (50, 250), 0.02, seed=30 + k) for k in range(4)]
    jobs = [engine.submit_pairs(b) for b in batches]
    for k in (2, 0, 3, 1):
        assert_same(jobs[k].collect(), oracle_lib.pairs(batches[k], nthreads=16), f"job {k}")
    with pytest.raises(engine.PairHMMError):
        jobs[0].collect()


def test_shutdown_refused_while_work_is_live(engine, oracle_lib):
    """hc_phmm_shutdown refuses (error, engine intact) while a submitted job
    or a prepared batch still holds device memory; after collect / close it
    succeeds, and the engine comes back with init (advisor round 2)."""
    b = W.generate(800, (100, 400), (50, 200), 0.02, seed=43)
    ref = oracle_lib.pairs(b, nthreads=16)
    job = engine.submit_pairs(b)
    with pytest.raises(engine.PairHMMError):
        engine.shutdown()
    assert_same(job.collect(), ref, "job after refused shutdown")
    bt = engine.Batch(b)
    with pytest.raises(engine.PairHMMError):
        engine.shutdown()
    bt.run()
    assert_same(bt.results(), ref, "batch after refused shutdown")
    bt.close()
    engine.shutdown()
    engine.init(0)
    assert_same(engine.pairs(b), ref, "after re-init")


def test_async_jobs_overlap_inputs_released(engine, oracle_lib):
    """Inputs may be dropped as soon as submit returns (they are staged)."""
    b = W.generate(2000, (100, 500), (50, 250), 0.01, seed=41)
    ref = oracle_lib.pairs(b, nthreads=16)
    cp = {k: v.copy() for k, v in b.items()}
    job = engine.submit_pairs(cp)
    for v in cp.values():
        v[...] = 0
    del cp
    assert_same(job.collect(), ref, "released inputs")


def _regions_ref(oracle_lib, regions):
    out = []
    for reads, haps in regions:
        if not reads or not haps:
            out.append(np.zeros((len(reads), len(haps))))
            continue
        flat = W.region_flat(reads, haps)
        out.append(oracle_lib.pairs(flat, nthreads=16)["loglik"].reshape(len(reads), len(haps)))
    return out


@pytest.mark.parametrize("split", ["one_part", "many_parts"])
def test_cross_regions_vs_oracle(engine, oracle_lib, monkeypatch, split):
    """Cross-region batching against the oracle: regions of
    different shapes, empty ones, and (many_parts) regions cut into read
    ranges over several parts."""
    if split == "many_parts":
        monkeypatch.setenv("HC_PHMM_SHARD_MIN_CELLS", "0")
        monkeypatch.setenv("HC_PHMM_CHUNK_CELLS", "30000000")
    regions = [W.region(n_reads=int(nr), n_haps=int(nh), seed=200 + k)
               for k, (nr, nh) in enumerate([(50, 2), (120, 8), (0, 3), (415, 32), (7, 1), (300, 5)])]
    got = engine.cross_regions(regions)
    for k, (g, e) in enumerate(zip(got, _regions_ref(oracle_lib, regions))):
        assert g.shape == e.shape
        assert np.array_equal(bits(g), bits(e)), f"region {k}"


@pytest.mark.parametrize("early", ["1", "0"])
def test_early_finish(engine, oracle_lib, monkeypatch, early):
    """A job part's unflagged pairs finished on the host while its fp64 launch
    runs (run.cpp run_part, api.cpp collect; HC_PHMM_EARLY_FINISH): a region
    with hundreds of rescues, a flat call of long haps (most pairs rescued) and
    one with none rescued, against the oracle, every output field."""
    monkeypatch.setenv("HC_PHMM_EARLY_FINISH", early)
    monkeypatch.setenv("HC_PHMM_RESCUE_IN_WAVE_MAX", "4")   # most rescues to the fp64 launch
    reads, haps = W.region(n_reads=415, n_haps=24, seed=211)
    flat = W.region_flat(reads, haps)
    ref = oracle_lib.pairs(flat, nthreads=16)
    assert ref["rescued"].sum() > 50
    got = engine.cross(reads, haps)
    assert np.array_equal(bits(got), bits(ref["loglik"].reshape(len(reads), len(haps))))
    for b in (W.subset(W.config("S4"), np.arange(400)), W.generate(3000, (100, 300), (60, 150), 0.0, seed=7)):
        ref = oracle_lib.pairs(b, nthreads=16)
        assert_same(engine.pairs(b), ref, f"early={early}")


@pytest.mark.parametrize("order", ["tail", "one_round", "tail_blocks"])
def test_flat_dispatch_order_vs_oracle(engine, oracle_lib, monkeypatch, order):
    """The device-planned flat part's dispatch order (pack_kernels.hip
    flat_tail_kernel: coalesced passes, block-scanned bucket cursors, stable
    bulk compaction): a tail of shortest waves after the bulk (one round of
    tail at ~6 000 waves), a one-round plan (1 024 < waves <= 3 072), and the
    tail with flat_prep_kernel on a bounded grid (several pairs per wave);
    every pair against the oracle."""
    if order == "one_round":
        b = W.generate(9000, (100, 500), (40, 250), 0.01, seed=61)
    else:
        monkeypatch.setenv("HC_PHMM_TAIL_ROUNDS", "1")
        if order == "tail_blocks":
            monkeypatch.setenv("HC_PHMM_PREP_BLOCKS", "64")
        b = W.generate(30000, (100, 600), (40, 250), 0.01, seed=62)
    assert_same(engine.pairs(b), oracle_lib.pairs(b, nthreads=16), order)


def test_submit_regions_two_slots(two_slots, oracle_lib):
    regions = [W.region(n_reads=200, n_haps=int(nh), seed=300 + k) for k, nh in enumerate([4, 16, 2, 8])]
    ref = _regions_ref(oracle_lib, regions)
    jobs = [two_slots.submit_regions(regions[:2]), two_slots.submit_regions(regions[2:])]
    got = jobs[1].collect() + jobs[0].collect()
    for g, e in zip(got, ref[2:] + ref[:2]):
        assert np.array_equal(bits(g), bits(e))


def test_per_base_gap_reads_take_the_full_upload(engine, oracle_lib):
    """Reads whose gap qualities vary are uploaded with their i/d/c planes; mixed
    with constant-gap reads in one batch."""
    b = W.generate(3000, (80, 400), (30, 200), 0.02, seed=9)
    rng = np.random.default_rng(4)
    rows = np.repeat(np.arange(3000) % 3 == 0, b["R"])
    n = int(rows.sum())
    b["ins"][rows] = rng.integers(33 + 5, 33 + 60, n, dtype=np.uint8)
    b["gcp"][rows] = rng.integers(33 + 5, 33 + 30, n, dtype=np.uint8)
    assert_same(engine.pairs(b), oracle_lib.pairs(b, nthreads=16), "mixed gaps")


def _ragged_region(seed, n_reads, n_haps, long_hap=False, vary_gaps=False):
    """A region with reads of lengths 20-150 and haps of lengths 30-415 (the
    structured planner sorts reads by R and groups haps by block width)."""
    rng = np.random.default_rng(seed)
    reads, haps = W.region(n_reads=n_reads, n_haps=n_haps, seed=seed)
    haps = [h[:int(rng.integers(30, len(h) + 1))] for h in haps]
    if long_hap:   # longer than 64 blocks of 64 columns: one-lane kernel, general planner
        haps[0] = rng.choice(np.frombuffer(b"ACGT", np.uint8), 4200).tobytes()
    out = []
    for b, q, i, d, c in reads:
        n = int(rng.integers(20, len(b) + 1))
        if vary_gaps and rng.random() < 0.3:
            i = bytes(rng.integers(33 + 5, 33 + 60, len(i), dtype=np.uint8))
        out.append((b[:n], q[:n], i[:n], d[:n], c[:n]))
    return out, haps


@pytest.mark.parametrize("grid", ["1", "0"])
def test_region_planner_ragged_vs_oracle(engine, oracle_lib, monkeypatch, grid):
    """hc_phmm_cross_regions through the structured cross-product planner
    (HC_PHMM_GRID_PLAN=1, the default) and the general one (0): ragged reads
    and haps, reads with varying gap qualities, a region whose hap needs the
    one-lane kernel (general planner for that call), empty regions."""
    monkeypatch.setenv("HC_PHMM_GRID_PLAN", grid)
    regions = [_ragged_region(500 + k, nr, nh, vary_gaps=k % 2 == 1)
               for k, (nr, nh) in enumerate([(415, 24), (90, 7), (1, 1), (200, 40)])]
    regions.insert(2, ([], []))
    for batch in (regions, [_ragged_region(600, 60, 5, long_hap=True)] + regions[:2]):
        got = engine.cross_regions(batch)
        for k, (g, e) in enumerate(zip(got, _regions_ref(oracle_lib, batch))):
            assert g.shape == e.shape
            assert np.array_equal(bits(g), bits(e)), f"grid={grid} region {k}"


def test_submit_unwinds_on_exception(engine, oracle_lib, many_parts):
    """A part whose planning throws (bad_alloc injected by a test hook) makes
    the submit fail with HC_PHMM_ENOMEM and free the parts it had already
    enqueued, so nothing stays live: shutdown then succeeds and the engine
    works again after init (advisor round 3: submit leaked the job and its
    parts, and shutdown was refused for the rest of the process)."""
    import ctypes as C
    L = engine.lib()
    L.hcx_inject_plan_throw.argtypes = [C.c_int]
    L.hcx_inject_plan_throw.restype = None
    b = W.generate(3000, (100, 500), (50, 250), 0.01, seed=44)
    ref = oracle_lib.pairs(b, nthreads=16)
    L.hcx_inject_plan_throw(2)   # the second part of the call throws
    try:
        with pytest.raises(engine.PairHMMError) as e:
            engine.pairs(b)
        assert e.value.code == engine.ENOMEM
    finally:
        L.hcx_inject_plan_throw(0)
    engine.shutdown()            # refused if any part had leaked
    engine.init(0)
    assert_same(engine.pairs(b), ref, "after unwinding")


@pytest.mark.parametrize("case", ["read_n_unsampled", "hap_n_unsampled", "low_qual", "n_and_gaps", "many_n"])
def test_flat_compact_fallbacks(engine, oracle_lib, case):
    """The flat call's compact record fields (one byte per read base, 2-bit
    hap codes) cannot hold an 'N' or a quality below 33: a part whose sample
    shows one starts with the nibble fields; one the sample misses (a single
    'N' read, 'N' hap or low quality between the sampled pairs) is refused in
    pass 2 and planned again with the nibble fields, and one that also has a
    read with varying gap qualities is planned again scanning every read
    (flat_plan.cpp plan_flat_device). Every case against the oracle."""
    b = W.config("S2", 20000)
    rs, q, hap = b["rs"].copy(), b["q"].copy(), b["hap"].copy()
    ro, ho = b["read_off"], b["hap_off"]
    if case in ("read_n_unsampled", "n_and_gaps"):
        rs[ro[7] + 3] = ord("N")        # pair 7: not on the 1-in-19 sample
    if case == "hap_n_unsampled":
        hap[ho[13] + 5] = ord("N")
    if case == "low_qual":
        q[ro[11] + 2] = 32 + 128        # (& 127) = 32: below the compact quality base
    if case == "many_n":
        rng = np.random.default_rng(3)
        for p in rng.choice(len(b["R"]), 300, replace=False):
            rs[ro[p] + rng.integers(0, b["R"][p])] = ord("N")
    b = dict(b, rs=rs, q=q, hap=hap)
    if case == "n_and_gaps":
        ins = b["ins"].copy()
        ins[ro[29] + 1] = ord("J")      # pair 29's gap qualities vary
        b = dict(b, ins=ins)
    L = engine.lib()
    L.hcx_flat_nibble_parts(0)   # (an earlier refusal would make this call skip the compact attempt)
    assert_same(engine.pairs(b), oracle_lib.pairs(b, nthreads=16), case)
    refused = case != "many_n"   # the sample sees one of 300 'N' reads; the others slip past it
    assert (L.hcx_flat_nibble_parts(-1) > 0) == refused, case
    L.hcx_flat_nibble_parts(0)


def test_flat_rare_n_after_refusal(engine, oracle_lib):
    """Rare 'N's the part samples miss: the first call's refusal makes the
    device's next parts start with the nibble records (Device::nibble_parts,
    DESIGN.md §16.7): two calls, both against the oracle, the second planned
    without the compact attempt; with the counter run out, a third call tries
    the compact records again (and is refused again)."""
    b = W.config("S2", 20000)
    rs = b["rs"].copy()
    ro = b["read_off"]
    for p in (7, 4007, 12345):   # off every 1-in-19 sample
        rs[ro[p] + 2] = ord("N")
    b = dict(b, rs=rs)
    ref = oracle_lib.pairs(b, nthreads=16)
    L = engine.lib()
    L.hcx_flat_nibble_parts(0)
    assert_same(engine.pairs(b), ref, "first call (refused, planned again)")
    left = L.hcx_flat_nibble_parts(-1)
    assert 0 < left <= 64
    assert_same(engine.pairs(b), ref, "second call (nibble records from the start)")
    assert L.hcx_flat_nibble_parts(-1) < left
    L.hcx_flat_nibble_parts(0)
    assert_same(engine.pairs(b), ref, "third call (compact attempt again)")
    assert L.hcx_flat_nibble_parts(-1) > 0
    L.hcx_flat_nibble_parts(0)
