#!/usr/bin/env python3
"""One config's committed profile (profiles/r03_pmc_<name>.json) from a
rocprofv3 kernel trace and --pmc passes of the same command:

    python tools/profile_summary.py OUT.json --trace DIR --skip W --cells N \
        [--kernel SUBSTR] NAME=DIR ...

--skip W drops each kernel's first W launches (warm-up) from the timing
average, so the committed average is the warm launches' — the ones bench.py
times with HIP events. PMC means are per dispatch over every launch (each
launch does the same work). (With --calls: per call, the sum over a call's launches.) HBM bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE
(KB) x 1024 (MI355X_MICROARCH.md, gfx950: FETCH_SIZE counts 128-B requests at
64 B). The kernel source hash (tools/kernel_src_hash.py) ties the file to the
device code it measured."""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_src_hash import kernel_src_hash  # noqa: E402

VALU_PEAK = 78.6e12


def short(k):
    return k.replace("hcphmm::(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def main():
    a = sys.argv[1:]
    out = a.pop(0)
    opts, passes = {}, []
    while a:
        x = a.pop(0)
        if x.startswith("--"):
            opts[x[2:]] = a.pop(0)
        else:
            passes.append(x.split("=", 1))
    skip = int(opts.get("skip", "0"))
    # --calls C: the traced program made C calls of which the first `skip` were
    # warm-up, each with the same number of launches of every kernel (a call
    # may cut its pairs into parts); figures are then per call.
    calls = int(opts.get("calls", "0"))
    cells = int(opts["cells"])
    launches = defaultdict(list)
    for f in glob.glob(os.path.join(opts["trace"], "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            launches[short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    kern = {}
    for k, v in launches.items():
        v.sort()
        d = [(e - s) / 1e6 for s, e in v]
        per = len(d) // calls if calls and len(d) % calls == 0 else 1
        warm = d[skip * per:] if len(d) > skip * per else d
        kern[k] = dict(launches=len(d), launches_per_unit=per, warm_launches=len(warm),
                       avg_ms_warm=round(sum(warm) / len(warm) * per, 4),
                       min_ms=round(min(d), 4), max_ms=round(max(d), 4), avg_ms_all=round(sum(d) / len(d), 4))
    for name, d in passes:
        vals = defaultdict(lambda: defaultdict(list))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                try:
                    vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
                except (KeyError, ValueError):
                    pass
        for k, cs in vals.items():
            per = kern.get(k, {}).get("launches_per_unit", 1)
            for c, v in cs.items():
                kern.setdefault(k, {})[c] = round(sum(v) / len(v) * per, 3)
    # dominant_kernel: the engine kernel with the longest warm time per unit;
    # fp32_kernel: the fp32 column-segmented pass (the bench roofline's kernel);
    # fp64_kernel: the fp64 rescue pass, priced per rescued cell (--rescued-cells).
    ours = {k: v for k, v in kern.items() if "phmm" in k or "rescue" in k or "kernel" in k}
    timed = {k: v for k, v in ours.items() if "avg_ms_warm" in v}
    dk = max(timed, key=lambda k: timed[k]["avg_ms_warm"]) if timed else None
    f32 = opts.get("kernel", "phmm_seg_")
    fk = next((k for k in timed if f32 in k and "seg64" not in k), None)
    f64k = next((k for k in timed if "phmm_seg64_kernel" in k), None)
    s = dict(kernel_src_hash=kernel_src_hash(), cells=cells, dominant_kernel=dk, fp32_kernel=fk, fp64_kernel=f64k,
             skip=skip, unit="call" if calls else "launch",
             passes={n: d for n, d in passes}, kernels=kern)
    if fk:
        e = kern[fk]
        s["frac_from_warm_avg"] = round(12 * cells / (e["avg_ms_warm"] * 1e-3) / VALU_PEAK, 4)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            s["hbm_bytes_per_launch"] = int((2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024)
            s["hbm_bytes_per_cell"] = round(s["hbm_bytes_per_launch"] / cells, 5)
            s["write_bytes_per_launch"] = int(e["WRITE_SIZE"] * 1024)
        if "SQ_INSTS_VALU" in e:
            s["valu_lane_instr_per_cell"] = round(e["SQ_INSTS_VALU"] * 64 / cells, 3)
        if "SQ_LDS_BANK_CONFLICT" in e:
            s["lds_bank_conflict_cycles_per_launch"] = int(e["SQ_LDS_BANK_CONFLICT"])
    rc = int(opts.get("rescued-cells", "0"))
    if f64k and rc > 0:
        e = kern[f64k]
        s["rescued_cells"] = rc
        s["fp64_frac_from_warm_avg"] = round(12 * rc / (e["avg_ms_warm"] * 1e-3) / 39.3e12, 4)
        if "SQ_INSTS_VALU" in e:
            s["fp64_valu_lane_instr_per_rescued_cell"] = round(e["SQ_INSTS_VALU"] * 64 / rc, 3)
        if "SQ_WAVE_CYCLES" in e and "SQ_BUSY_CYCLES" in e and e["SQ_BUSY_CYCLES"] > 0:
            s["fp64_mean_resident_waves_per_busy_cycle"] = round(e["SQ_WAVE_CYCLES"] / e["SQ_BUSY_CYCLES"], 2)
    json.dump(s, open(out, "w"), indent=1)
    s["dominant"] = kern.get(dk)
    print(json.dumps({k: s[k] for k in s if k not in ("kernels", "passes")}))


if __name__ == "__main__":
    main()
