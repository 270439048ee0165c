"""fp64 chain waves on a uniform batch (every pair R x H): fp64 kernel time
and the per-wave durations (HC_PHMM_TIMELINE records), so a chain wave's
time per step can be set against a single wave's.

    HC_PHMM_CHAIN=4 HC_PHMM_CHAIN_TAIL=0 python tools/chain_probe.py [R] [H] [n]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

os.environ.setdefault("HC_PHMM_TIMELINE", "1")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 200
H = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
hcphmm.init(0)
L = hcphmm.lib()
L.hcx_timeline64.argtypes = [C.c_void_p, C.c_int]
b = W.generate(n, (H, H), (R, R), 0.08, seed=5)
bt = hcphmm.Batch(b)
for _ in range(5):
    bt.run()
st = bt.stats()
cap = 2 * n + 16
buf = np.zeros(3 * cap, np.uint64)
n64 = L.hcx_timeline64(buf.ctypes.data, cap)
r = buf[:3 * n64].reshape(n64, 3).astype(np.int64)[:n]
r = r[r[:, 1] > 0]
if not len(r):   # (HC_PHMM_TIMELINE=0: the kernel time only, e.g. under rocprofv3 --pmc)
    print(json.dumps(dict(R=R, H=H, pairs=n, kernel_ms_f64=round(st.kernel_ms_f64, 4))), flush=True)
    bt.close()
    sys.exit(0)
d = (r[:, 1] - r[:, 0]) / 100.0
s = (r[:, 0] - r[:, 0].min()) / 100.0
e = (r[:, 1] - r[:, 0].min()) / 100.0
out = dict(R=R, H=H, pairs=n, rescued=int(st.n_rescued), chain=os.environ.get("HC_PHMM_CHAIN"),
           tail=os.environ.get("HC_PHMM_CHAIN_TAIL"), kernel_ms_f64=round(st.kernel_ms_f64, 4), waves=int(len(d)),
           dur_us={str(q): round(float(np.percentile(d, q)), 1) for q in (10, 50, 90, 99)},
           first_round_dur_p50=round(float(np.median(d[s < 5.0])), 1) if (s < 5.0).any() else None,
           later_dur_p50=round(float(np.median(d[s >= 5.0])), 1) if (s >= 5.0).any() else None,
           last_end_us=round(float(e.max()), 1))
# Slow waves (over twice the median): their hardware slots (SIMD, wave id)
# and what else ran on those slots and their SIMD.
hw = r[:, 2] & 0xFFFFFFFF
xcc = (r[:, 2] >> 32) & 0xF
simd = ((xcc * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 64 + ((hw >> 8) & 15) * 4 + ((hw >> 4) & 3)
slot = simd * 16 + (hw & 15)
med = np.median(d)
slow = d > 2 * med
out2 = dict(slow=int(slow.sum()), slow_slots=int(len(np.unique(slot[slow]))), slow_simds=int(len(np.unique(simd[slow]))),
            tasks_per_slot=np.bincount(np.unique(slot, return_inverse=True)[1]).tolist()[:0],
            slots=int(len(np.unique(slot))), simds=int(len(np.unique(simd))))
# for a few slow waves: the other tasks of their SIMD (start, dur, slot)
ex = []
for j in np.where(slow)[0][:3]:
    same = np.where(simd == simd[j])[0]
    ex.append(dict(slow=dict(start=round(s[j], 1), dur=round(d[j], 1), wave_id=int(hw[j] & 15), tg=int((hw[j] >> 16) & 15)),
                   simd_tasks=[(round(s[k], 1), round(d[k], 1), int(hw[k] & 15), int((hw[k] >> 16) & 15)) for k in same[np.argsort(s[same])]]))
out2["examples"] = ex
out.update(out2)
print(json.dumps(out), flush=True)
bt.close()
