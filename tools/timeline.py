"""Per-wave timeline of the segmented fp32 pass (HC_PHMM_TIMELINE=1 build hook):
for a batch, the start / end of every wave (s_memrealtime, 100 MHz) and its
CU / SIMD (HW_ID), after warm-up runs. Prints a summary: pass span, when the
last wave starts, how busy the wave slots are over time (tenths of the span),
the idle slot-time at the end, wave duration spread.
    HC_PHMM_TIMELINE=1 python tools/timeline.py S2:125000 [out.npy]
    HC_PHMM_TIMELINE=1 python tools/timeline.py cross:415:128     (the region call's own plan)
"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

os.environ["HC_PHMM_TIMELINE"] = "1"
name, _, n = sys.argv[1].partition(":")
hcphmm.init(0)
L = hcphmm.lib()
L.hcx_timeline.argtypes = [C.c_void_p, C.c_int]
cap = 4_000_000
buf = np.zeros(3 * cap, np.uint64)
if name == "cross":   # the region call itself (structured plan), cross:NR:NH
    nr, nh = (int(x) for x in n.split(":"))
    call = hcphmm.CrossCall(*W.region(n_reads=nr, n_haps=nh))
    for _ in range(8):
        call()
    st = type("St", (), {"kernel_ms_f32": float("nan")})()
    nw = L.hcx_timeline(buf.ctypes.data, cap)
else:
    if name == "region":   # the same pairs as a flat batch
        nr, nh = (int(x) for x in n.split(":"))
        b = W.region_flat(*W.region(n_reads=nr, n_haps=nh))
    else:
        b = W.config(name, int(n) if n else None)
    bt = hcphmm.Batch(b)
    for _ in range(4):
        bt.run()
    st = bt.stats()
    nw = L.hcx_timeline(buf.ctypes.data, cap)
    bt.close()
rec = buf[:3 * nw].reshape(nw, 3).astype(np.int64)
t0 = rec[:, 0].min()
start = (rec[:, 0] - t0) / 100.0   # us
end = (rec[:, 1] - t0) / 100.0
hw = rec[:, 2]
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
slot_simd = ((se * 2 + sh) * 16 + cu) * 4 + simd
span = end.max()
dur = end - start
order = np.arange(nw)
out = dict(workload=sys.argv[1], waves=int(nw), kernel_ms_f32=round(st.kernel_ms_f32, 4), span_us=round(span, 1),
           last_start_us=round(start.max(), 1), first_end_us=round(end.min(), 1),
           dur_us=dict(p10=round(float(np.percentile(dur, 10)), 1), p50=round(float(np.median(dur)), 1),
                       p90=round(float(np.percentile(dur, 90)), 1), max=round(float(dur.max()), 1)),
           distinct_simds=int(len(np.unique(slot_simd))))
# resident waves over time (tenths of the span)
tt = np.linspace(0, span, 21)[1:-1]
out["resident_waves"] = [int(((start <= t) & (end > t)).sum()) for t in tt]
# per-SIMD busy end: when each SIMD's last wave ends
simd_end = {}
for s_, e_ in zip(slot_simd, end):
    simd_end[s_] = max(simd_end.get(s_, 0), e_)
se_arr = np.array(list(simd_end.values()))
out["simd_last_end_us"] = dict(p10=round(float(np.percentile(se_arr, 10)), 1), p50=round(float(np.median(se_arr)), 1),
                               p90=round(float(np.percentile(se_arr, 90)), 1))
# start delay of the first waves (dispatch ramp)
out["start_us_first_3072"] = dict(p50=round(float(np.median(np.sort(start)[:3072])), 2),
                                  max=round(float(np.sort(start)[min(3071, nw - 1)]), 2))
out["in_order_start_corr"] = round(float(np.corrcoef(order, start)[0, 1]), 3)
print(json.dumps(out), flush=True)
if len(sys.argv) > 2:
    np.save(sys.argv[2], rec)
