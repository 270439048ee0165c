"""Seeded synthetic genotyping sites.

A site is what Genetyper::assign_genotype_likelihoods hands to the likelihood
arithmetic for one variant start (reference genotyper/genotyper.hpp:369-399):
the region's read-major log10 likelihood matrix L (n_reads x n_haps, after
IntelPairHMM::compute_likelihoods' normalisation: every value within 4.5 of its
read's best), the reads overlapping the allele window (get_read_indices_to_keep,
:234-243), the haplotype -> allele map (get_haplotype_mapper, :224-232) and the
allele count (2..MAX_ALLELE_COUNT = 7). Several sites share a region's L.
"""
from __future__ import annotations

import numpy as np

MAX_ALLELES = 7


def region_matrix(rng, n_reads, n_haps, with_inf=False):
    """log10 likelihoods shaped like normalised PairHMM output."""
    L = -rng.gamma(2.0, 8.0, size=(n_reads, n_haps)) - rng.uniform(0, 3, size=(n_reads, 1))
    best = L.max(axis=1, keepdims=True)
    L = np.maximum(L, best - 4.5)   # intel_pairhmm.hpp:29-33
    # reads that support one hap exactly tie with it
    if n_haps > 1:
        ties = rng.random(n_reads) < 0.2
        L[ties, 1] = L[ties, 0]
    if with_inf:
        L[rng.random(L.shape) < 0.01] = -np.inf
    return np.ascontiguousarray(L, np.float64)


def sites(n_regions=16, sites_per_region=8, reads=(50, 415), haps=(2, 32), seed=61, with_inf=False):
    """Returns (matrices, sites): matrices = list of L arrays; sites = list of
    dicts {m (matrix index), keep int32[], hap_allele int32[], n_alleles}."""
    rng = np.random.default_rng(seed)
    mats, out = [], []
    for _ in range(n_regions):
        nr = int(rng.integers(reads[0], reads[1] + 1))
        nh = int(rng.integers(haps[0], haps[1] + 1))
        mats.append(region_matrix(rng, nr, nh, with_inf))
        for _ in range(sites_per_region):
            A = int(rng.integers(2, min(MAX_ALLELES, nh + 1) + 1)) if nh >= 2 else 2
            keep = np.sort(rng.choice(nr, size=int(rng.integers(1, nr + 1)), replace=False)).astype(np.int32)
            amap = rng.integers(0, A, size=nh).astype(np.int32)
            amap[0] = 0
            out.append(dict(m=len(mats) - 1, keep=keep, hap_allele=amap, n_alleles=A))
    return mats, out


def n_genotypes(a: int) -> int:
    return a * (a + 1) // 2
