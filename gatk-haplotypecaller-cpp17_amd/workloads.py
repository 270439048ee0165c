"""Seeded synthetic read x haplotype batches.

A batch is a dict of flat numpy arrays in the layout the flat C-ABI entry
point ``hc_phmm_pairs_flat`` takes (include/hc_pairhmm.h):

    read_off[int64], R[int32]   rows of pair p: rs/q/ins/dels/gcp[read_off[p] : +R[p]]
    hap_off[int64],  H[int32]   hap of pair p:  hap[hap_off[p] : +H[p]]
    rs, q, ins, dels, gcp, hap  uint8 byte pools (raw SAM bytes: bases, Phred+33)

Generator (numpy PCG64, not mt19937_64 — the distribution is what §8(d) fixes):
hap bases i.i.d. uniform ACGT; R ~ U[r_lo, min(r_hi, H)]; read = hap[off : off+R],
off ~ U[0, H-R]; per-base substitution rate e; base quality Phred ~ U[10, 40]
stored as ASCII+33; ins/del GOP = 'I' (73), GCP = '+' (43) per base — exactly
what the reference's SAMRecord supplies (sam.hpp:30-32, 47-49).
"""
from __future__ import annotations

import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
GOP = 73   # 'I'
GCP = 43   # '+'

# name -> (n_pairs, (h_lo, h_hi), (r_lo, r_hi), subst, seed)
CONFIGS = {
    "S1": (10_000, (150, 150), (101, 101), 0.01, 42),
    "S1w": (10_000, (250, 250), (101, 101), 0.01, 42),
    "S2": (1_000_000, (100, 500), (50, 250), 0.01, 43),
    "S4": (2_000, (1000, 2000), (150, 250), 0.08, 44),
}


def generate(n, h_range, r_range, subst=0.01, seed=0, q_range=(10, 40)):
    rng = np.random.default_rng(seed)
    h_lo, h_hi = h_range
    r_lo, r_hi = r_range
    H = rng.integers(h_lo, h_hi + 1, size=n, dtype=np.int64)
    r_top = np.minimum(r_hi, H)
    R = r_lo + np.floor(rng.random(n) * (r_top - r_lo + 1)).astype(np.int64)
    R = np.minimum(R, r_top)
    hap_off = np.zeros(n, np.int64)
    np.cumsum(H[:-1], out=hap_off[1:])
    read_off = np.zeros(n, np.int64)
    np.cumsum(R[:-1], out=read_off[1:])
    tot_h, tot_r = int(H.sum()), int(R.sum())
    hap_codes = rng.integers(0, 4, size=tot_h, dtype=np.uint8)
    start = np.floor(rng.random(n) * (H - R + 1)).astype(np.int64)
    # read base k of pair p = hap[hap_off[p] + start[p] + k]
    idx = np.arange(tot_r, dtype=np.int64)
    idx += np.repeat(hap_off + start - read_off, R)
    rd = hap_codes[idx]
    del idx
    sub = rng.random(tot_r) < subst
    nsub = int(sub.sum())
    rd[sub] = (rd[sub] + rng.integers(1, 4, size=nsub, dtype=np.uint8)) % 4
    q = (rng.integers(q_range[0], q_range[1] + 1, size=tot_r, dtype=np.uint8) + 33).astype(np.uint8)
    return dict(
        read_off=read_off, R=R.astype(np.int32), hap_off=hap_off, H=H.astype(np.int32),
        rs=ACGT[rd], q=q,
        ins=np.full(tot_r, GOP, np.uint8), dels=np.full(tot_r, GOP, np.uint8),
        gcp=np.full(tot_r, GCP, np.uint8), hap=ACGT[hap_codes],
    )


def config(name: str, n: int | None = None):
    n0, hr, rr, e, seed = CONFIGS[name]
    return generate(n or n0, hr, rr, e, seed)


def cells(batch) -> int:
    return int(np.dot(batch["R"].astype(np.int64), batch["H"].astype(np.int64)))


def subset(batch, idx):
    """Re-pack the pairs `idx` of a batch into a new compact batch."""
    idx = np.asarray(idx, dtype=np.int64)
    R = batch["R"][idx].astype(np.int64)
    H = batch["H"][idx].astype(np.int64)
    ro = np.zeros(len(idx), np.int64)
    ho = np.zeros(len(idx), np.int64)
    if len(idx):
        np.cumsum(R[:-1], out=ro[1:])
        np.cumsum(H[:-1], out=ho[1:])
    ridx = (np.arange(int(R.sum()), dtype=np.int64)
            + np.repeat(batch["read_off"][idx] - ro, R))
    hidx = (np.arange(int(H.sum()), dtype=np.int64)
            + np.repeat(batch["hap_off"][idx] - ho, H))
    out = dict(read_off=ro, R=R.astype(np.int32), hap_off=ho, H=H.astype(np.int32))
    for k in ("rs", "q", "ins", "dels", "gcp"):
        out[k] = batch[k][ridx]
    out["hap"] = batch["hap"][hidx]
    return out


def from_pairs(pairs):
    """pairs: list of (read_bases, qual, ins, del, gcp, hap) byte strings."""
    n = len(pairs)
    R = np.array([len(p[0]) for p in pairs], np.int32)
    H = np.array([len(p[5]) for p in pairs], np.int32)
    ro = np.zeros(n, np.int64)
    ho = np.zeros(n, np.int64)
    if n:
        np.cumsum(R[:-1].astype(np.int64), out=ro[1:])
        np.cumsum(H[:-1].astype(np.int64), out=ho[1:])

    def cat(k):
        return np.frombuffer(b"".join(p[k] for p in pairs), dtype=np.uint8).copy()

    return dict(read_off=ro, R=R, hap_off=ho, H=H, rs=cat(0), q=cat(1), ins=cat(2),
                dels=cat(3), gcp=cat(4), hap=cat(5))


def edge_pairs(seed=7, variants=4):
    """SURVEY Appendix B edge grid: R x H sizes x 4 byte-content variants
    (random bytes incl. N / lowercase / IUPAC, quals 0..127, random GOP/GCP)."""
    rng = np.random.default_rng(seed)
    Rs = [1, 2, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 101, 128, 199, 200]
    Hs = [1, 2, 7, 8, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 150, 250, 1000, 1024, 1500]
    alpha = np.frombuffer(b"ACGTNacgtnRYKMSWBDHV.-*", dtype=np.uint8)
    out = []
    for R in Rs:
        for H in Hs:
            for v in range(variants):
                if v == 0:      # clean ACGT, realistic quals, constant gaps
                    hap = ACGT[rng.integers(0, 4, H)]
                    rs = ACGT[rng.integers(0, 4, R)]
                    q = rng.integers(43, 74, R).astype(np.uint8)
                    i = np.full(R, GOP, np.uint8); d = i.copy(); c = np.full(R, GCP, np.uint8)
                elif v == 1:    # N-rich bases
                    hap = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, H)]
                    rs = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, R)]
                    q = rng.integers(33, 127, R).astype(np.uint8)
                    i = np.full(R, GOP, np.uint8); d = i.copy(); c = np.full(R, GCP, np.uint8)
                elif v == 2:    # arbitrary bytes, full quality range, per-base gaps
                    hap = alpha[rng.integers(0, len(alpha), H)]
                    rs = alpha[rng.integers(0, len(alpha), R)]
                    q = rng.integers(0, 256, R).astype(np.uint8)
                    i = rng.integers(0, 256, R).astype(np.uint8)
                    d = rng.integers(0, 256, R).astype(np.uint8)
                    c = rng.integers(0, 256, R).astype(np.uint8)
                else:           # read copied from hap (high likelihood), random gaps
                    hap = ACGT[rng.integers(0, 4, H)]
                    if R <= H:
                        o = int(rng.integers(0, H - R + 1))
                        rs = hap[o:o + R].copy()
                    else:
                        rs = ACGT[rng.integers(0, 4, R)]
                    q = rng.integers(33, 80, R).astype(np.uint8)
                    i = rng.integers(20, 90, R).astype(np.uint8)
                    d = rng.integers(20, 90, R).astype(np.uint8)
                    c = rng.integers(10, 60, R).astype(np.uint8)
                out.append((rs.tobytes(), q.tobytes(), i.tobytes(), d.tobytes(), c.tobytes(), hap.tobytes()))
    return out


def region(n_reads=415, n_haps=32, H=415, R=150, subst=0.01, seed=45):
    """One active-region-shaped cross product (SURVEY §8(d) 'cross-product variant'):
    n_haps haplotypes of length ~H that differ from a common base by a few SNPs
    and small indels, n_reads reads of length R drawn from them with `subst`
    substitutions. Returns (reads, haps) as the C ABI's cross call takes them:
    reads = [(bases, qual, ins_gop, del_gop, gcp)], haps = [bases]."""
    rng = np.random.default_rng(seed)
    base = ACGT[rng.integers(0, 4, H)]
    haps = []
    for h in range(n_haps):
        x = base.copy()
        if h:
            k = rng.integers(1, 4)
            pos = rng.integers(0, H, k)
            x[pos] = ACGT[rng.integers(0, 4, k)]
            if rng.random() < 0.5:
                p = int(rng.integers(10, H - 10))
                if rng.random() < 0.5:
                    x = np.concatenate([x[:p], ACGT[rng.integers(0, 4, int(rng.integers(1, 6)))], x[p:]])
                else:
                    x = np.concatenate([x[:p], x[p + int(rng.integers(1, 6)):]])
        haps.append(x.tobytes())
    reads = []
    for r in range(n_reads):
        src = np.frombuffer(haps[int(rng.integers(0, n_haps))], np.uint8)
        o = int(rng.integers(0, max(1, len(src) - R + 1)))
        rs = src[o:o + R].copy()
        sub = rng.random(len(rs)) < subst
        rs[sub] = ACGT[(np.searchsorted(ACGT, rs[sub]) + rng.integers(1, 4, int(sub.sum()))) % 4]
        q = (rng.integers(10, 41, len(rs)) + 33).astype(np.uint8)
        n = len(rs)
        reads.append((rs.tobytes(), q.tobytes(), bytes([GOP]) * n, bytes([GOP]) * n, bytes([GCP]) * n))
    return reads, haps


def region_flat(reads, haps):
    """Expand a region's cross product into a flat batch (read-major pairs)."""
    return from_pairs([(r[0], r[1], r[2], r[3], r[4], h) for r in reads for h in haps])
