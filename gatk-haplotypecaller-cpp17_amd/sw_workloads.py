"""Seeded synthetic haplotype-to-reference alignment batches.

The reference aligns every assembled haplotype of an active region against the
region's reference window (``assembler/graph_wrapper.hpp:232-240``:
``IntelSWAligner::align(ref, h.bases)`` with NEW_SW_PARAMETERS and the SOFTCLIP
overhang strategy, ``smithwaterman/intel_smithwaterman.hpp:23,29-44``). A batch
is a dict of flat numpy arrays in the layout of the flat C-ABI entry point
``hc_sw_align_flat`` (include/hc_sw.h):

    ref_off[int64], ref_len[int32]   seq1 of pair p: refs[ref_off[p] : +ref_len[p]]
    alt_off[int64], alt_len[int32]   seq2 of pair p: alts[alt_off[p] : +alt_len[p]]
    refs, alts                       uint8 byte pools (raw bases)

Pairs of one region share their ref window (same ref_off). Lengths stay within
the reference aligner's limits: seq2 (alt) <= MAX_SEQ_LEN = 1024
(native/smithwaterman_common.h:47) and seq1 (ref) <= 1023 (a 1024-base seq1
writes E[-1], PairWiseSW.h:199, and corrupts the heap).
"""
from __future__ import annotations

import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
MAX_LEN = 1024

# IntelSWAligner parameter sets (intel_smithwaterman.hpp:21-24): match, mismatch, open, extend
ORIGINAL_DEFAULT = (3, -1, -4, -3)
STANDARD_NGS = (25, -50, -110, -6)
NEW_SW_PARAMETERS = (200, -150, -260, -11)
ALIGNMENT_TO_BEST_HAPLOTYPE = (10, -15, -30, -5)
PARAM_SETS = (NEW_SW_PARAMETERS, ORIGINAL_DEFAULT, STANDARD_NGS, ALIGNMENT_TO_BEST_HAPLOTYPE)
# Not a reference parameter set: large scores that drive H down to
# MATRIX_MIN_CUTOFF (-1e8, smithwaterman_common.h:50) so the cutoff binds.
CUTOFF_PARAMS = (1000, -1000000, -20000000, -3000000)

# Overhang strategies (native/smithwaterman_common.h:26-29)
SOFTCLIP, INDEL, LEADING_INDEL, IGNORE = 9, 10, 11, 12
STRATEGIES = (SOFTCLIP, INDEL, LEADING_INDEL, IGNORE)

# name -> (regions, haps per region, (ref_lo, ref_hi), seed)
CONFIGS = {
    # one real-sized active region: 415-base window, DEFAULT_NUM_PATHS = 128 haps
    "W1": (1, 128, (415, 415), 51),
    # a chromosome's worth of regions batched into one device pass
    "W2": (512, 128, (300, 600), 52),
    # long windows at the reference's length limit
    "W3": (64, 64, (900, 1023), 53),
}


def _mutate(rng, ref: np.ndarray, snp: float, indel: float, trim: float) -> np.ndarray:
    x = ref.copy()
    n = len(x)
    sub = rng.random(n) < snp
    x[sub] = ACGT[(np.searchsorted(ACGT, x[sub]) + rng.integers(1, 4, int(sub.sum()))) % 4]
    k = rng.binomial(n, indel)
    for _ in range(int(k)):
        p = int(rng.integers(0, len(x) + 1))
        ln = int(rng.integers(1, 13))
        if rng.random() < 0.5:
            x = np.concatenate([x[:p], ACGT[rng.integers(0, 4, ln)], x[p:]])
        else:
            x = np.concatenate([x[:p], x[p + ln:]])
    if rng.random() < trim:   # assembly paths that start or end inside the window
        a = int(rng.integers(0, 25))
        b = int(rng.integers(0, 25))
        x = x[a:len(x) - b] if len(x) - a - b >= 8 else x
    if len(x) == 0:
        x = ref[:1].copy()
    return x[:MAX_LEN]


def _window(rng, n: int) -> np.ndarray:
    """A reference window: i.i.d. bases with a few tandem repeats (ties in the DP)."""
    w = ACGT[rng.integers(0, 4, n)]
    for _ in range(int(rng.integers(0, 4))):
        unit = ACGT[rng.integers(0, 4, int(rng.integers(1, 5)))]
        rep = np.tile(unit, int(rng.integers(3, 12)))
        p = int(rng.integers(0, max(1, n - len(rep))))
        w[p:p + len(rep)] = rep[:n - p]
    return w


def regions(n_regions, haps_per_region, ref_range, seed=0, snp=0.01, indel=0.004, trim=0.3):
    """n_regions windows of length U[ref_range]; per window, hap 0 is the window
    itself (the reference path of the assembly graph, taken by the all-match
    shortcut) and the rest carry SNPs, 1-12 base indels and trimmed ends."""
    rng = np.random.default_rng(seed)
    lo, hi = ref_range
    refs, alts, ref_off, ref_len, alt_off, alt_len = [], [], [], [], [], []
    ro = ao = 0
    for _ in range(n_regions):
        w = _window(rng, int(rng.integers(lo, hi + 1)))
        refs.append(w)
        for h in range(haps_per_region):
            a = w.copy() if h == 0 else _mutate(rng, w, snp, indel, trim)
            alts.append(a)
            ref_off.append(ro)
            ref_len.append(len(w))
            alt_off.append(ao)
            alt_len.append(len(a))
            ao += len(a)
        ro += len(w)
    return dict(ref_off=np.array(ref_off, np.int64), ref_len=np.array(ref_len, np.int32),
                refs=np.concatenate(refs), alt_off=np.array(alt_off, np.int64),
                alt_len=np.array(alt_len, np.int32), alts=np.concatenate(alts))


def config(name: str, n_regions: int | None = None):
    nr, hp, rr, seed = CONFIGS[name]
    return regions(n_regions or nr, hp, rr, seed)


def from_pairs(pairs):
    """[(ref bytes, alt bytes)] -> flat batch (every pair owns its ref)."""
    refs = [np.frombuffer(r, np.uint8) for r, _ in pairs]
    alts = [np.frombuffer(a, np.uint8) for _, a in pairs]
    rl = np.array([len(r) for r in refs], np.int32)
    al = np.array([len(a) for a in alts], np.int32)
    ro = np.zeros(len(pairs), np.int64)
    ao = np.zeros(len(pairs), np.int64)
    if len(pairs) > 1:
        np.cumsum(rl[:-1], out=ro[1:])
        np.cumsum(al[:-1], out=ao[1:])
    cat = lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.uint8)
    return dict(ref_off=ro, ref_len=rl, refs=cat(refs), alt_off=ao, alt_len=al, alts=cat(alts))


def subset(batch, idx):
    return from_pairs([pair(batch, int(k)) for k in idx])


def pair(batch, k):
    r = batch["refs"][batch["ref_off"][k]:batch["ref_off"][k] + batch["ref_len"][k]].tobytes()
    a = batch["alts"][batch["alt_off"][k]:batch["alt_off"][k] + batch["alt_len"][k]].tobytes()
    return r, a


def cells(batch) -> int:
    return int((batch["ref_len"].astype(np.int64) * batch["alt_len"].astype(np.int64)).sum())


def edge_pairs(seed=11):
    """Edge grid: tiny and maximal lengths, lengths around the 64-row stripe and
    8-cell word boundaries, identical / near-identical pairs (the all-match
    shortcut and just past it), unrelated pairs, homopolymers and tandem
    repeats (score ties -> the reference's tie-break rules), and non-ACGT bytes
    (raw byte equality, no N wildcard: PairWiseSW.h:25-27)."""
    rng = np.random.default_rng(seed)
    out = []
    lens = [1, 2, 3, 7, 8, 9, 31, 63, 64, 65, 66, 127, 128, 129, 200, 415, 1000, 1023, 1024]
    for n1 in lens[:-1]:   # seq1 of 1024 writes E[-1] in the reference (PairWiseSW.h:199)
        for n2 in lens:
            if (n1 > 200 or n2 > 200) and rng.random() < 0.6:
                continue
            r = _window(rng, n1)
            if rng.random() < 0.5 and n2 <= n1:
                o = int(rng.integers(0, n1 - n2 + 1))
                a = _mutate(rng, r[o:o + n2], 0.03, 0.0, 0.0)
            else:
                a = ACGT[rng.integers(0, 4, n2)]
            out.append((r.tobytes(), a[:n2].tobytes()))
    for n in (1, 2, 5, 64, 150, 415, 1023):
        r = ACGT[rng.integers(0, 4, n)]
        out.append((r.tobytes(), r.tobytes()))                     # identical
        for k in (1, 2, 3, 4):                                     # k mismatches
            a = r.copy()
            pos = rng.choice(n, size=min(k, n), replace=False)
            a[pos] = ACGT[(np.searchsorted(ACGT, a[pos]) + 1) % 4]
            out.append((r.tobytes(), a.tobytes()))
    for n in (10, 64, 100, 300):
        out.append((b"A" * n, b"A" * (n // 2)))                    # homopolymer ties
        out.append((b"A" * (n // 2), b"A" * n))
        out.append((b"AC" * (n // 2), b"AC" * (n // 3) + b"G"))    # tandem repeats
        out.append((b"ACGT" * (n // 4), b"CGTA" * (n // 4 + 1)))
        out.append((b"A" * n, b"C" * n))                           # nothing matches
    for _ in range(24):
        n1, n2 = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        pool = np.frombuffer(b"ACGTNacgtn-*", np.uint8)
        out.append((pool[rng.integers(0, len(pool), n1)].tobytes(),
                    pool[rng.integers(0, len(pool), n2)].tobytes()))
    return out


def shortcut_mask(batch):
    """Pairs IntelSWAligner::align answers without the DP (intel_smithwaterman.hpp:47-58)."""
    n = len(batch["ref_len"])
    m = np.zeros(n, bool)
    for k in np.nonzero(batch["ref_len"] == batch["alt_len"])[0]:
        r, a = pair(batch, int(k))
        m[k] = np.count_nonzero(np.frombuffer(r, np.uint8) != np.frombuffer(a, np.uint8)) <= 2
    return m


def dp_cells(batch) -> int:
    """Cells of the pairs that run the DP (the all-match shortcut skips the rest)."""
    keep = ~shortcut_mask(batch)
    return int((batch["ref_len"][keep].astype(np.int64) * batch["alt_len"][keep].astype(np.int64)).sum())
