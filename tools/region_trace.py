"""Per-phase host timings (HC_PHMM_TRACE=1) of one active-region call,
hc_phmm_cross on 415 reads x N haps, the shape IntelPairHMM::compute_likelihoods
sees (haplotypecaller.hpp:103). Run on the GPU box:
    HC_PHMM_TRACE=1 python tools/region_trace.py 32
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

nh = int(sys.argv[1]) if len(sys.argv) > 1 else 32
hcphmm.init(0)
reads, haps = W.region(415, nh)
for k in range(4):
    t0 = time.perf_counter()
    hcphmm.cross(reads, haps)
    print(f"call {k}: {(time.perf_counter() - t0) * 1e3:.3f} ms", file=sys.stderr, flush=True)
