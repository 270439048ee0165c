"""Genotyper numeric core (§8(f) row 4). CPU: the oracle against the reference's
compiled MathUtils (golden) and its own site pins; the library exports the
symbol and fails loudly without a GPU. GPU (-m gpu): the HIP kernel against the
golden sites and the oracle, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

import gt_workloads as G


def bits(x):
    return np.ascontiguousarray(x, np.float64).view(np.uint64)


def test_approx_sum_matches_reference_mathutils(gt_golden, gt_oracle_lib):
    a, b, out = gt_golden["approx"]
    mine = np.array([gt_oracle_lib.approx(x, y) for x, y in zip(a, b)])
    assert np.array_equal(bits(mine), bits(out))


def test_approx_sum_vs_freshly_built_reference():
    import oracle
    if not os.path.exists(oracle.REF_MATH_SO):
        pytest.skip("oracle/_ref/libref_math.so not built (needs /root/reference)")
    ref, orc = oracle.MathReference(), oracle.GTOracle()
    rng = np.random.default_rng(5)
    for x, y in zip(rng.uniform(-60, 0, 3000), rng.uniform(-60, 0, 3000)):
        assert np.float64(ref.approx(x, y)).view(np.uint64) == np.float64(orc.approx(x, y)).view(np.uint64)


@pytest.mark.parametrize("name", ["std", "inf"])
def test_oracle_sites_pinned(gt_golden, gt_oracle_lib, name):
    mats, sites, exp = gt_golden["sets"][name]
    for s, (gl, gi, gq) in zip(sites, exp):
        r = gt_oracle_lib.site(mats[s["m"]], s["keep"], s["hap_allele"], s["n_alleles"])
        assert np.array_equal(bits(r[0]), bits(gl)) and r[1] == gi and r[2] == gq


def test_gt_symbol_exported_and_no_fallback():
    import hcphmm
    import hcgt
    out = subprocess.run(["nm", "-D", "--defined-only", hcphmm.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert all(f" T {s}" in out for s in hcgt.declared_symbols())
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    mats, sites = G.sites(1, 1)
    with pytest.raises(hcgt.GTError):
        hcgt.genotype_sites(mats, sites)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["std", "inf"])
def test_gpu_sites_golden(gt_golden, name):
    import hcgt
    mats, sites, exp = gt_golden["sets"][name]
    got = hcgt.genotype_sites(mats, sites)
    for (gl, gi, gq), (egl, egi, egq) in zip(got, exp):
        assert np.array_equal(bits(gl), bits(egl)) and gi == egi and gq == egq


@pytest.mark.gpu
def test_gpu_many_regions_vs_oracle(gt_oracle_lib):
    import hcgt
    mats, sites = G.sites(n_regions=64, sites_per_region=12, seed=90, with_inf=True)
    got = hcgt.genotype_sites(mats, sites)
    for s, (gl, gi, gq) in zip(sites, got):
        egl, egi, egq = gt_oracle_lib.site(mats[s["m"]], s["keep"], s["hap_allele"], s["n_alleles"])
        assert np.array_equal(bits(gl), bits(egl)) and gi == egi and gq == egq


@pytest.mark.gpu
def test_gpu_edge_sites(gt_oracle_lib):
    """All -inf rows (NaN quality), exact ties, one kept read, unused alleles."""
    import hcgt
    L = np.full((4, 3), -np.inf)
    L[1] = [-1.0, -1.0, -2.0]
    L[2] = [-3.0, -3.0, -3.0]
    L[3] = [-0.0, 0.0, -7.9999]
    sites = [dict(m=0, keep=np.array([0], np.int32), hap_allele=np.array([0, 1, 1], np.int32), n_alleles=2),
             dict(m=0, keep=np.array([1, 2, 3], np.int32), hap_allele=np.array([0, 1, 2], np.int32), n_alleles=4),
             dict(m=0, keep=np.array([], np.int32), hap_allele=np.array([0, 0, 0], np.int32), n_alleles=7),
             dict(m=0, keep=np.array([3, 1], np.int32), hap_allele=np.array([1, 0, 1], np.int32), n_alleles=2)]
    got = hcgt.genotype_sites([L], sites)
    for s, (gl, gi, gq) in zip(sites, got):
        egl, egi, egq = gt_oracle_lib.site(L, s["keep"], s["hap_allele"], s["n_alleles"])
        assert np.array_equal(bits(gl), bits(egl)) and gi == egi and gq == egq, (s, gl, egl, gi, egi, gq, egq)
