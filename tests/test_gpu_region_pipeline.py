"""GPU: the region pipeline of HaplotypeCaller::call_region (haplotypecaller.hpp:
83-107) — Smith-Waterman of the candidate haplotypes, PairHMM with the read
filter, the genotyper's per-site arithmetic — composed from the three drop-ins
(hc::MI355XSWAligner, hc::MI355XPairHMM, hc_gt_genotype_sites) in a compiled
C++ program, against the same chain on the reference's own kernels compiled
from its sources (oracle/_ref) plus the oracle's restated filter and genotyper
loops. Offsets, CIGARs, kept reads, likelihood matrices, genotype likelihoods,
genotypes and qualities must all be bit-identical (tests/cpp/region_pipeline.cpp).
VCF parity with the reference binary stays unpinned (Boost and chrM absent)."""
import json
import os
import subprocess

import pytest

import hcphmm

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")


def build(tmp_path):
    exe = tmp_path / "region_pipeline"
    libdir = os.path.dirname(hcphmm.LIB_PATH)
    orc = os.path.join(ROOT, "oracle")
    for lib in ("libref_pairhmm.so", "libref_sw.so", "libref_math.so"):
        if not os.path.exists(os.path.join(REF, lib)):
            pytest.fail(f"oracle/_ref/{lib} missing: build it with `make -C oracle ref` where /root/reference exists")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "region_pipeline.cpp"),
                    "-L", libdir, "-lhcpairhmm", "-L", REF, "-lref_pairhmm", "-lref_sw", "-lref_math",
                    "-L", orc, "-loracle", "-fopenmp",
                    f"-Wl,-rpath,{libdir}:{REF}:{orc}", "-o", str(exe)], check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2])
def test_region_pipeline_matches_reference_chain(tmp_path, seed):
    exe = build(tmp_path)
    out = tmp_path / "summary.json"
    p = subprocess.run([str(exe), "48", str(seed), str(out)], capture_output=True, text=True, timeout=600)
    assert out.exists(), p.stderr[-2000:]
    s = json.loads(out.read_text())
    print(s)
    assert p.returncode == 0, s
    assert s["sites"] > 48 and s["non_ref_genotypes"] > 10 and s["reads_kept"] < s["reads"]
    for k in ("sw_mismatch", "keep_mismatch", "likelihood_mismatch", "gl_mismatch", "gt_gq_mismatch"):
        assert s[k] == 0, (k, s)
