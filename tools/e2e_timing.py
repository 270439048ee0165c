import sys, time, os
sys.path.insert(0, "gatk-haplotypecaller-cpp17_amd")
import hcphmm, workloads as W
hcphmm.init(0)
b = W.config("S2")
for k in range(3):
    t = time.perf_counter(); r = hcphmm.pairs(b); dt = time.perf_counter() - t
    print(f"call {k}: {dt*1e3:.1f} ms  {W.cells(b)/dt/1e9:.1f} GCUPS", flush=True)
