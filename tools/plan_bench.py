"""Host-planning time of the engine without a GPU (hcx_plan_* hooks of
libhcpairhmm.so): S2 (1M pairs) as hc_phmm_pairs_flat plans it, and one
415 x N region as hc_phmm_cross plans it.

    HC_PHMM_TRACE=1 python tools/plan_bench.py [s2|region|all] [reps]
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "all"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
L = hcphmm.lib()
L.hcx_plan_pairs.restype = C.c_double
L.hcx_plan_regions.restype = C.c_double
L.hcx_plan_regions.argtypes = [C.c_void_p, C.c_int32, C.c_int, C.c_int]
if what in ("s2", "all"):
    b = W.config("S2")
    args, keep = hcphmm._flat_args(b)
    ms = L.hcx_plan_pairs(*args, C.c_int(256), C.c_int(1), C.c_int(reps))
    print(f"S2 1M pairs plan: {ms:.2f} ms/call", flush=True)
if what in ("region", "all"):
    for nh in (32, 128):
        reads, haps = W.region(415, nh)
        arr, outs, keep = hcphmm._region_array([(reads, haps)])
        ms = L.hcx_plan_regions(arr, 1, 256, reps * 10)
        print(f"region 415x{nh} plan: {ms:.3f} ms/call", flush=True)
