"""Planner / kernel-variant sweep on the GPU box: one process, several
device-resident batches under different HC_PHMM_* settings, each timed over
10 device passes (HIP events) and checked bit for bit against the first
setting of its workload (all settings must give the same bits).

    python tools/sweep.py S1 S1w S2 --env HC_PHMM_SEG_CAP=8,12,16 > out.jsonl

Each output line: workload, pairs, settings, kernel_ms_f32, kernel_ms_f64,
run_ms, frac_f32 (12 * cells / fp32 kernel time / 78.6 T), identical."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd"))

import numpy as np  # noqa: E402

import hcphmm  # noqa: E402
import workloads as W  # noqa: E402


def bits(r):
    return {k: np.ascontiguousarray(v).view(np.uint8) for k, v in r.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="+", help="NAME or NAME:pairs")
    ap.add_argument("--env", action="append", default=[], help="VAR=v1,v2,... (one run per value; '-' = unset)")
    ap.add_argument("--runs", type=int, default=10)
    a = ap.parse_args()
    settings = [{}]
    for spec in a.env:
        var, vals = spec.split("=", 1)
        settings = [dict(s, **{var: v}) for s in settings for v in vals.split(",")]
    hcphmm.init(0)
    for wl in a.workloads:
        name, _, n = wl.partition(":")
        if name == "region":   # region:NREADS:NHAPS, one cross product as flat pairs
            nr, nh = (int(x) for x in n.split(":"))
            b = W.region_flat(*W.region(n_reads=nr, n_haps=nh))
        else:
            b = W.config(name, int(n) if n else None)
        cells = W.cells(b)
        ref = None
        for st in settings:
            for k, v in st.items():
                if v == "-":
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            bt = hcphmm.Batch(b)
            for _ in range(2):
                bt.run()
            bt.stats()
            for _ in range(a.runs):
                bt.run()
            s = bt.stats()
            r = bits(bt.results())
            bt.close()
            same = None
            if ref is None:
                ref = r
            else:
                same = all(np.array_equal(r[k], ref[k]) for k in ref)
            print(json.dumps(dict(workload=name, pairs=len(b["R"]), settings=st,
                                  kernel_ms_f32=round(s.kernel_ms_f32, 4), kernel_ms_f64=round(s.kernel_ms_f64, 4),
                                  run_ms=round(s.run_ms, 4), waves=int(s.n_launch_waves),
                                  frac_f32=round(12 * cells / (s.kernel_ms_f32 * 1e-3) / 78.6e12, 4),
                                  rescued=int(s.n_rescued), identical=same)), flush=True)
        for k in {k for s in settings for k in s}:
            os.environ.pop(k, None)


if __name__ == "__main__":
    main()
