"""End-to-end host-path timings (S2 pairs_flat, 415 x 32 / 128 region cross calls,
64 regions in one call), median of 5, for A/B of two library builds (HC_PHMM_LIB)."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd"))
import hcphmm, workloads as W
hcphmm.init(0)
def med(f, n=5):
    f()
    t = []
    for _ in range(n):
        t0 = time.perf_counter(); f(); t.append(time.perf_counter() - t0)
    return round(float(np.median(t)) * 1e3, 3)
out = {}
b = W.config("S2")
out["s2_pairs_ms"] = med(lambda: hcphmm.pairs(b), 3)
for nh in (32, 128):
    reads, haps = W.region(415, nh)
    call = hcphmm.CrossCall(reads, haps)
    out[f"region_415x{nh}_ms"] = med(call, 10)
regs = [W.region(415, 32, seed=100 + k) for k in range(64)]
rc = hcphmm.RegionsCall(regs)
out["regions64_ms"] = med(rc, 5)
print(json.dumps(out))
