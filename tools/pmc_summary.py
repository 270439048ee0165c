#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output into a per-kernel JSON (profiles/).

    python tools/pmc_summary.py OUT.json NAME=DIR [NAME=DIR ...] [--cells N]

Each DIR is one rocprofv3 `--pmc ... --output-format csv -d DIR` pass (one
counter group per pass, as MI355X_MICROARCH.md prescribes: FETCH_SIZE and
WRITE_SIZE never share a pass). For every kernel the mean counter value per
dispatch is reported. HBM bytes per launch follow the guide's gfx950 rule:
FETCH_SIZE (KB) is multiplied by 2 (it tallies 128-B requests at 64 B) and
WRITE_SIZE (KB) taken as is; both x 1024.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read_pass(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "?")
                c = row.get("Counter_Name", "?")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                vals[k][c].append(v)
    return vals


def main():
    out = sys.argv[1]
    cells = None
    passes = []
    for a in sys.argv[2:]:
        if a.startswith("--cells="):
            cells = int(a.split("=", 1)[1])
        elif "=" in a:
            passes.append(a.split("=", 1))
    kern = defaultdict(dict)
    for name, d in passes:
        for k, cs in read_pass(d).items():
            for c, v in cs.items():
                kern[k][c] = dict(mean=sum(v) / len(v), n=len(v))
    summary = {"passes": {n: d for n, d in passes}, "kernels": {}}
    dominant = None
    for k, cs in kern.items():
        ent = {c: round(v["mean"], 3) for c, v in cs.items()}
        fetch = cs.get("FETCH_SIZE", {}).get("mean")
        write = cs.get("WRITE_SIZE", {}).get("mean")
        if fetch is not None and write is not None:
            ent["hbm_bytes_per_launch"] = int((2 * fetch + write) * 1024)
            ent["hbm_bytes_note"] = "2*FETCH_SIZE + WRITE_SIZE (KB) x 1024, gfx950 correction"
        summary["kernels"][k] = ent
    # Dominant fp32 PairHMM kernel: column-segmented > one-lane > anti-diagonal.
    def rank(k):
        for r, tag in enumerate(("phmm_seg_kernel", "phmm_lane_kernel", "phmm_diag_kernel<float")):
            if tag in k:
                return r
        return None
    for k in kern:
        if rank(k) is not None and (dominant is None or rank(k) < rank(dominant)):
            dominant = k
    if dominant:
        summary["dominant_kernel"] = dominant
        summary["hbm_bytes_per_launch"] = summary["kernels"][dominant].get("hbm_bytes_per_launch")
        if cells:
            summary["cells"] = cells
            k = summary["kernels"][dominant]
            if "SQ_INSTS_VALU" in k:
                summary["valu_lane_instr_per_cell"] = round(k["SQ_INSTS_VALU"] * 64 / cells, 3)
        if cells and summary["hbm_bytes_per_launch"]:
            summary["hbm_bytes_per_cell"] = summary["hbm_bytes_per_launch"] / cells
    with open(out, "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
