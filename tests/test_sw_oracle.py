"""CPU: the Smith-Waterman oracle (oracle/sw_oracle.c) against the reference.

tests/golden/sw_golden.npz holds the reference aligner's own outputs
(oracle/_ref/libref_sw.so compiled from /root/reference by oracle/Makefile;
tests/golden/make_sw_golden.py). These tests pin the restatement on every
offset and CIGAR; the GPU parity tests (test_gpu_sw.py) then compare the HIP
aligner with both.
"""
import numpy as np
import pytest

import sw_workloads as S


def test_sw_golden_cases_cover_every_strategy_and_param_set(sw_golden):
    combos = {(c["params"], c["strategy"]) for c in sw_golden["cases"] if c["set"] == "edge"}
    assert combos >= {(p, s) for p in S.PARAM_SETS for s in S.STRATEGIES}
    assert any(p == S.CUTOFF_PARAMS for p, _ in combos)


def test_sw_oracle_matches_reference_golden(sw_golden, sw_oracle_lib):
    for c in sw_golden["cases"]:
        b = sw_golden["sets"][c["set"]]
        off, cig = sw_oracle_lib.batch(b, c["params"], c["strategy"], shortcut=True, nthreads=4)
        assert np.array_equal(off, c["offset"]), c["name"]
        assert cig == c["cigar"], c["name"]


def test_sw_all_match_shortcut(sw_oracle_lib):
    # intel_smithwaterman.hpp:36-37,47-58: equal lengths, <= 2 mismatches -> (0, "<n>M")
    r = b"ACGTACGTAC" * 10
    a2 = bytearray(r); a2[3] = ord("A"); a2[50] = ord("T")
    a3 = bytearray(a2); a3[90] = ord("G")
    b = S.from_pairs([(r, r), (r, bytes(a2)), (r, bytes(a3)), (r, r[:-1])])
    off, cig = sw_oracle_lib.batch(b)
    assert cig[0] == "100M" and cig[1] == "100M" and off[0] == off[1] == 0
    off_n, cig_n = sw_oracle_lib.batch(b, shortcut=False)
    assert cig[2] == cig_n[2] and cig[3] == cig_n[3]


def test_sw_cigar_consumes_alt(sw_golden):
    # Every CIGAR spans the whole alt (seq2): M + I + S lengths == len(alt).
    import re
    for c in sw_golden["cases"]:
        b = sw_golden["sets"][c["set"]]
        for k, cig in enumerate(c["cigar"]):
            n = sum(int(x) for x, op in re.findall(r"(\d+)([MIDSR])", cig) if op in "MIS")
            if c["strategy"] == S.IGNORE:
                continue   # IGNORE repeats the last op over the overhang (PairWiseSW.h:345-352)
            assert n == b["alt_len"][k], (c["name"], k, cig)


def test_sw_oracle_vs_reference_fresh_pairs():
    import oracle
    if not oracle.sw_reference_available():
        pytest.skip("oracle/_ref/libref_sw.so not built (needs /root/reference)")
    ref, orc = oracle.SWReference(), oracle.SWOracle()
    b = S.regions(3, 64, (100, 700), seed=99, snp=0.03, indel=0.01)
    for p in S.PARAM_SETS[:2]:
        for st in S.STRATEGIES:
            ro, rc = ref.batch(b, p, st)
            oo, oc = orc.batch(b, p, st, nthreads=4)
            assert np.array_equal(ro, oo) and rc == oc, (p, st)
