"""Host passes of a flat call (flat_plan.cpp) without a GPU: pass 1 (lengths,
offsets) and pass 2 (records: qualities, code nibbles, gap check) over S2,
on this machine's cores. usage: python tools/flat_host_bench.py [pairs] [reps]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import numpy as np  # noqa: E402

import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 250_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
b = W.config("S2", n)
args, keep = hcphmm._flat_args(b)
L = hcphmm.lib()
ms = np.zeros(2)
L.hcx_flat_host_passes(*args, C.c_int(reps), ms.ctypes.data_as(C.POINTER(C.c_double)))
rb = 5 * int(b["R"].sum()) + int(b["H"].sum())
print(f"{n} pairs: pass 1 {ms[0]:.3f} ms, pass 2 {ms[1]:.3f} ms "
      f"({rb / ms[1] / 1e6:.1f} GB/s of caller bytes read)")
