"""Per-wave timelines of both passes of a rescue-heavy batch (configs[4], S4)
— the fp32 seg waves and the fp64 rescue waves (HC_PHMM_TIMELINE=1 records:
start / end of s_memrealtime at 100 MHz, HW_ID, the fp64 wave's first pair) —
after warm-up runs of a prepared batch. Names the critical path: the fp32
wave that ends last and the fp64 wave that ends last, with their pairs'
(R, H), the gap between the passes, and per-SIMD sums of wave time.

    python tools/timeline_rescue.py [S4[:pairs]] [out.json]
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
name, _, n = (sys.argv[1] if len(sys.argv) > 1 else "S4").partition(":")
hcphmm.init(0)
L = hcphmm.lib()
for f in (L.hcx_timeline, L.hcx_timeline64):
    f.argtypes = [C.c_void_p, C.c_int]
b = W.config(name, int(n) if n else None)
bt = hcphmm.Batch(b)
for _ in range(6):
    bt.run()
st = bt.stats()
cap = 2 * len(b["R"]) + 16
buf = np.zeros(3 * cap, np.uint64)
n32 = L.hcx_timeline(buf.ctypes.data, cap)
r32 = buf[:3 * n32].reshape(n32, 3).astype(np.int64).copy()
n64 = L.hcx_timeline64(buf.ctypes.data, cap)
r64 = buf[:3 * n64].reshape(n64, 3).astype(np.int64).copy()
plan = r64[len(b["R"])] if n64 > len(b["R"]) else None   # {planner start, plan published, list length}
# the planner's phase stamps: counted, table, scattered, costs, prefix, planned
phases = r64[len(b["R"]) + 1:len(b["R"]) + 3].reshape(-1) if n64 >= len(b["R"]) + 3 else None
r64 = r64[:len(b["R"])]
r64 = r64[r64[:, 1] > 0]
bt.close()


def simd_of(word):
    """SIMD of a record's HW_ID (low word) and XCC_ID (bits 32-35): 8 XCDs x 128."""
    hw = word & 0xFFFFFFFF
    xcc = (word >> 32) & 0xF
    return ((xcc * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 64 + ((hw >> 8) & 15) * 4 + ((hw >> 4) & 3)


t0 = r32[:, 0].min()
out = dict(workload=sys.argv[1] if len(sys.argv) > 1 else "S4", pairs=len(b["R"]), fp32_waves=int(n32),
           fp64_waves=int(len(r64)), kernel_ms_f32=round(st.kernel_ms_f32, 4), kernel_ms_f64=round(st.kernel_ms_f64, 4),
           device_pass_ms=round(st.run_ms, 4))
e32 = (r32[:, 1] - t0) / 100.0
s32 = (r32[:, 0] - t0) / 100.0
out["fp32"] = dict(first_start_us=round(s32.min(), 1), last_start_us=round(s32.max(), 1),
                   last_end_us=round(e32.max(), 1), end_p50_us=round(float(np.median(e32)), 1),
                   dur_p50_us=round(float(np.median(e32 - s32)), 1), dur_max_us=round(float((e32 - s32).max()), 1))
if len(r64):
    s64 = (r64[:, 0] - t0) / 100.0
    e64 = (r64[:, 1] - t0) / 100.0
    pid = (r64[:, 2] >> 40).astype(np.int64)
    k = int(np.argmax(e64))
    d64 = e64 - s64
    kd = int(np.argmax(d64))
    if plan is not None and plan[1] > 0:
        out["fp64_plan"] = dict(start_us=round((plan[0] - t0) / 100.0, 1), published_us=round((plan[1] - t0) / 100.0, 1),
                                plan_us=round((plan[1] - plan[0]) / 100.0, 1), listed=int(plan[2]),
                                launch_gap_us=round((plan[0] - t0) / 100.0 - e32.max(), 1))
        if phases is not None:
            names = ["count", "table", "scatter", "costs", "prefix", "order"]
            prev = plan[0]
            ph = {}
            for nm, v in zip(names, phases):
                if v > 0:
                    ph[nm] = round((int(v) - int(prev)) / 100.0, 1)
                    prev = v
            ph["publish"] = round((int(plan[1]) - int(prev)) / 100.0, 1)
            out["fp64_plan"]["phase_us"] = ph
    out["fp64"] = dict(first_start_us=round(s64.min(), 1), last_start_us=round(s64.max(), 1),
                       last_end_us=round(e64.max(), 1), gap_after_fp32_us=round(s64.min() - e32.max(), 1),
                       dur_p10_us=round(float(np.percentile(d64, 10)), 1),
                       dur_p50_us=round(float(np.median(d64)), 1), dur_max_us=round(float(d64.max()), 1),
                       critical=dict(pair=int(pid[k]), R=int(b["R"][pid[k]]), H=int(b["H"][pid[k]]),
                                     start_us=round(s64[k], 1), dur_us=round(d64[k], 1)),
                       longest=dict(pair=int(pid[kd]), R=int(b["R"][pid[kd]]), H=int(b["H"][pid[kd]]),
                                    dur_us=round(d64[kd], 1)))
    out["fp64"]["dur_pct_us"] = {str(q): round(float(np.percentile(d64, q)), 1) for q in (75, 90, 95, 99)}
    top = np.argsort(-d64)[:12]
    out["fp64"]["longest_waves"] = [dict(pair=int(pid[j]), R=int(b["R"][pid[j]]), H=int(b["H"][pid[j]]),
                                         start_us=round(s64[j], 1), dur_us=round(d64[j], 1)) for j in top]
    sim = simd_of(r64[:, 2])
    busy = {}
    cnt = {}
    for s_, d_ in zip(sim, d64):
        busy[s_] = busy.get(s_, 0.0) + d_
        cnt[s_] = cnt.get(s_, 0) + 1
    ends = {}
    for s_, e_ in zip(sim, e64):
        ends[s_] = max(ends.get(s_, 0.0), e_)
    ea = np.array(list(ends.values()))
    out["fp64"]["simds"] = len(ends)
    out["fp64"]["waves_per_simd"] = {str(c): int(v) for c, v in zip(*np.unique(list(cnt.values()), return_counts=True))}
    out["fp64"]["simd_last_end_us"] = dict(p10=round(float(np.percentile(ea, 10)), 1),
                                           p50=round(float(np.median(ea)), 1), max=round(float(ea.max()), 1))
    # duration of a wave by its SIMD's company: alone vs sharing
    solo = np.array([cnt[s_] == 1 for s_ in sim])
    if solo.any() and (~solo).any():
        out["fp64"]["dur_us_alone_p50"] = round(float(np.median(d64[solo])), 1)
        out["fp64"]["dur_us_shared_p50"] = round(float(np.median(d64[~solo])), 1)
print(json.dumps(out), flush=True)
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
