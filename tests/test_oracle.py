"""CPU: the oracle (our C restatement) against the reference's golden vectors.

tests/golden/pairhmm_golden.npz was produced by the reference's own AVX kernel
(oracle/_ref, built from /root/reference; tests/golden/make_golden.py). These
tests pin the restatement bit for bit; the GPU parity tests then compare the
HIP engine with both.
"""
import numpy as np
import pytest

import workloads as W


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def test_luts_match_reference(oracle_lib, golden):
    L = oracle_lib.luts()
    for k in ("ph2pr_f", "ph2pr_d", "mm_f", "mm_d"):
        assert np.array_equal(bits(L[k]), bits(golden[k])), k
    import hashlib
    sha = hashlib.sha256(L["jac_f"].tobytes() + L["jac_d"].tobytes()).hexdigest()
    assert sha == str(golden["jac_sha256"])


def test_pairs_bit_exact_all_sets(oracle_lib, golden, golden_batch):
    res = oracle_lib.pairs(golden_batch, nthreads=4)
    assert np.array_equal(bits(res["raw_f32"]), bits(golden["raw_f32"]))
    assert np.array_equal(res["rescued"], golden["rescued"])
    resc = golden["rescued"].astype(bool)
    assert np.array_equal(bits(res["raw_f64"][resc]), bits(golden["raw_f64_all"][resc]))
    assert np.array_equal(bits(res["loglik"]), bits(golden["loglik"]))


@pytest.mark.parametrize("setname", ["edge", "random", "underflow"])
def test_f64_kernel_every_pair(oracle_lib, golden, golden_batch, setname):
    names = list(golden["set_names"])
    idx = np.nonzero(golden["set_id"] == names.index(setname))[0][::3]
    b = golden_batch
    for p in idx:
        ro, R, ho, H = b["read_off"][p], b["R"][p], b["hap_off"][p], b["H"][p]
        args = [b[k][ro:ro + R].tobytes() for k in ("rs", "q", "ins", "dels", "gcp")]
        d = oracle_lib.full_prob(*args, b["hap"][ho:ho + H].tobytes(), f64=True)
        assert np.float64(d).tobytes() == golden["raw_f64_all"][p].tobytes(), p


def test_golden_covers_the_hazards(golden):
    """The fixture exercises rescue, FTZ -> -inf, N bases and per-base gap quals."""
    assert golden["rescued"].sum() > 100
    assert np.isneginf(golden["loglik"]).sum() > 10
    assert (golden["rs"] == ord("N")).any() and (golden["hap"] == ord("N")).any()
    assert len(np.unique(golden["ins"])) > 50
    assert golden["R"].min() == 1 and golden["H"].min() == 1 and golden["H"].max() >= 1500


def test_finish_rules(oracle_lib):
    # intel_pairhmm.hpp:137-143: rescue below 1e-28f, float subtraction otherwise
    f = np.float32(2.0 ** 100)
    expect = float(np.float32(np.log10(f)) - np.float32(np.log10(np.float32(2.0 ** 120))))
    assert oracle_lib.finish(f, 0.0) == pytest.approx(expect, abs=8e-6)   # float ulp at 36
    assert oracle_lib.finish(np.float32(1e-29), 2.0 ** 1000) == pytest.approx(
        1000 * np.log10(2.0) - 1020 * np.log10(2.0), abs=1e-9)
    assert np.isneginf(oracle_lib.finish(0.0, 0.0))


def test_normalize_matches_reference_rules(oracle_lib):
    L = np.array([[-1.0, -10.0, -3.0], [-20.0, -25.0, -30.0], [-0.5, -0.5, -9.0]])
    out, keep = oracle_lib.normalize(L, np.array([100, 100, 500], np.int32))
    assert np.allclose(out[0], [-1.0, -5.5, -3.0])
    assert list(keep) == [True, False, True]      # -20 < min(2, ceil(2))*-4 = -8
    assert np.allclose(out[2], [-0.5, -0.5, -5.0])


def test_workload_generator_shapes():
    b = W.config("S1", 100)
    assert (b["R"] == 101).all() and (b["H"] == 150).all()
    assert set(np.unique(b["ins"])) == {73} and set(np.unique(b["gcp"])) == {43}
    b = W.config("S2", 5000)
    assert b["H"].min() >= 100 and b["H"].max() <= 500
    assert (b["R"] >= 50).all() and (b["R"] <= np.minimum(250, b["H"])).all()
    assert W.cells(b) == int((b["R"].astype(np.int64) * b["H"]).sum())
