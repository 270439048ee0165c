"""Host phases (HC_PHMM_TRACE=1) and timing of the bench's 64-region call: 64
regions of 415 reads x 32 haps through one hc_phmm_cross_regions call (the
cross-region batching of SURVEY.md §8(f) row 2).
    HC_PHMM_TRACE=1 python tools/regions_trace.py [reps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
hcphmm.init(0)
regs = [W.region(415, 32, seed=1000 + k) for k in range(64)]
rc = sum(W.cells(W.region_flat(r, h)) for r, h in regs)
call = hcphmm.RegionsCall(regs)
for k in range(reps):
    t0 = time.perf_counter()
    call()
    dt = time.perf_counter() - t0
    print(f"call {k}: {dt * 1e3:.2f} ms  {rc / dt / 1e9:.0f} GCUPS", file=sys.stderr, flush=True)
