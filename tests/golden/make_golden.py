"""Generate the PairHMM golden fixtures from the REFERENCE kernel.

Run in the build container (needs oracle/_ref/libref_pairhmm.so, built by
`make -C oracle ref` from /root/reference sources):

    python tests/golden/make_golden.py

Writes tests/golden/pairhmm_golden.npz: inputs (flat batch layout of
workloads.py) + the reference's outputs for every pair:
    raw_f32      compute_full_prob_avxs<float>        (bits)
    raw_f64_all  compute_full_prob_avxd<double>       (bits, every pair)
    rescued      raw_f32 < 1e-28f                      (intel_pairhmm.hpp:137)
    loglik       finished log10 likelihood             (intel_pairhmm.hpp:137-143)
and the reference LUTs (ph2pr, matchToMatchProb) plus a SHA-256 of the
Jacobian tables. Sets: SURVEY Appendix-B edge grid (1 596 pairs), a random
mixed set, S1/S4 samples, an underflow set that drives fp64 results into
the denormal / FTZ -> 0 -> -inf region, and haps of 8 193 - 20 000 bases.
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd"))

import oracle  # noqa: E402
import workloads as W  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pairhmm_golden.npz")


def concat(batches):
    out = {k: [] for k in batches[0]}
    ro = ho = 0
    for b in batches:
        out["read_off"].append(b["read_off"] + ro)
        out["hap_off"].append(b["hap_off"] + ho)
        for k in ("R", "H", "rs", "q", "ins", "dels", "gcp", "hap"):
            out[k].append(b[k])
        ro += len(b["rs"])
        ho += len(b["hap"])
    return {k: np.concatenate(v) for k, v in out.items()}


def random_mixed(n, seed):
    """Random pairs: R 10-199, H R..R+299, 1 in 7 reads carrying N bases."""
    rng = np.random.default_rng(seed)
    pairs = []
    for k in range(n):
        R = int(rng.integers(10, 200))
        H = int(rng.integers(R, R + 300))
        hap = W.ACGT[rng.integers(0, 4, H)]
        o = int(rng.integers(0, H - R + 1))
        rs = hap[o:o + R].copy()
        sub = rng.random(R) < 0.03
        rs[sub] = W.ACGT[rng.integers(0, 4, int(sub.sum()))]
        if k % 7 == 0:
            rs[rng.integers(0, R, 3)] = ord("N")
        q = rng.integers(43, 74, R).astype(np.uint8)
        i = np.full(R, W.GOP, np.uint8)
        c = np.full(R, W.GCP, np.uint8)
        pairs.append((rs.tobytes(), q.tobytes(), i.tobytes(), i.tobytes(), c.tobytes(), hap.tobytes()))
    return W.from_pairs(pairs)


def underflow_set(seed):
    out = []
    for e in (0.15, 0.25, 0.35, 0.45):
        out.append(W.generate(12, (1500, 2000), (200, 250), e, seed, q_range=(35, 40)))
        seed += 1
    return concat(out)


def long_haps(seed):
    """Haplotypes past the anti-diagonal kernel's LDS ring (H 8 193, 12 000,
    20 000): reads copied from the hap, random reads (rescued in fp64), one
    base, 8 % substitutions at R 250, and an N-rich read with per-base gap
    qualities."""
    rng = np.random.default_rng(seed)
    pairs = []
    for H in (8193, 12000, 20000):
        hap = W.ACGT[rng.integers(0, 4, H)]
        o = int(rng.integers(0, H - 250))
        kinds = []
        rs = hap[o:o + 150].copy()
        kinds.append((rs, rng.integers(43, 74, 150), np.full(150, W.GOP), np.full(150, W.GOP), np.full(150, W.GCP)))
        rs = W.ACGT[rng.integers(0, 4, 101)]
        kinds.append((rs, rng.integers(60, 74, 101), np.full(101, W.GOP), np.full(101, W.GOP), np.full(101, W.GCP)))
        kinds.append((hap[o:o + 1].copy(), np.array([60]), np.array([W.GOP]), np.array([W.GOP]), np.array([W.GCP])))
        rs = hap[o:o + 250].copy()
        sub = rng.random(250) < 0.08
        rs[sub] = W.ACGT[rng.integers(0, 4, int(sub.sum()))]
        kinds.append((rs, rng.integers(43, 74, 250), np.full(250, W.GOP), np.full(250, W.GOP), np.full(250, W.GCP)))
        rs = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, 64)]
        kinds.append((rs, rng.integers(33, 127, 64), rng.integers(20, 90, 64), rng.integers(20, 90, 64),
                      rng.integers(10, 60, 64)))
        for rs, q, i, d, c in kinds:
            pairs.append(tuple(np.asarray(x, np.uint8).tobytes() for x in (rs, q, i, d, c)) + (hap.tobytes(),))
    return W.from_pairs(pairs)


def main():
    ref = oracle.Reference()
    sets = {
        "edge": W.from_pairs(W.edge_pairs(seed=7)),
        "random": random_mixed(1200, seed=11),
        "s1": W.subset(W.config("S1"), np.arange(300)),
        "s2": W.subset(W.config("S2", 20_000), np.arange(400)),
        "s4": W.subset(W.config("S4"), np.arange(40)),
        "underflow": underflow_set(seed=101),
        "long_haps": long_haps(seed=131),
    }
    names = list(sets)
    batch = concat([sets[k] for k in names])
    set_id = np.concatenate([np.full(len(sets[k]["R"]), i, np.int8) for i, k in enumerate(names)])
    res = ref.pairs(batch, nthreads=os.cpu_count() or 1)
    n = len(batch["R"])
    raw64_all = np.zeros(n, np.float64)
    for p in range(n):
        ro, R, ho, H = batch["read_off"][p], batch["R"][p], batch["hap_off"][p], batch["H"][p]
        raw64_all[p] = ref.full_prob(*(batch[k][ro:ro + R].tobytes() for k in ("rs", "q", "ins", "dels", "gcp")),
                                     batch["hap"][ho:ho + H].tobytes(), f64=True)
    lut = ref.luts()
    jac_sha = hashlib.sha256(lut["jac_f"].tobytes() + lut["jac_d"].tobytes()).hexdigest()
    np.savez_compressed(
        OUT, set_names=np.array(names), set_id=set_id, **batch,
        raw_f32=res["raw_f32"], raw_f64_all=raw64_all, rescued=res["rescued"], loglik=res["loglik"],
        ph2pr_f=lut["ph2pr_f"], ph2pr_d=lut["ph2pr_d"], mm_f=lut["mm_f"], mm_d=lut["mm_d"],
        jac_sha256=np.array(jac_sha))
    ninf = int(np.isneginf(res["loglik"]).sum())
    print(f"wrote {OUT}: {n} pairs, {res['n_rescued']} rescued, {ninf} -inf, "
          f"{os.path.getsize(OUT) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
