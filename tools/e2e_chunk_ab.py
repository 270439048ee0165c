"""S2 through hc_phmm_pairs_flat (host buffers in, log10 out), one 415 x 128
region call and 64 regions of 415 x 32 in one call, under several
HC_PHMM_CHUNK_CELLS values (cells per pipelined part), alternating settings
over rounds in one process; median per setting.
    python tools/e2e_chunk_ab.py 1.2e10,6e9,4e9"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

vals = sys.argv[1].split(",")
hcphmm.init(0)
b = W.config("S2")
cells = W.cells(b)
out = hcphmm.result_arrays(len(b["R"]))
reads, haps = W.region(415, 128)
rcall = hcphmm.CrossCall(reads, haps)
regs = hcphmm.RegionsCall([W.region(415, 32, seed=100 + k) for k in range(64)])
ref = None
times = {v: [] for v in vals}
rt = {v: [] for v in vals}
mt = {v: [] for v in vals}
for rnd in range(3):
    for v in vals:
        os.environ["HC_PHMM_CHUNK_CELLS"] = str(int(float(v)))
        hcphmm.pairs(b, out)
        if ref is None:
            ref = out["loglik"].copy()
        assert (out["loglik"].view("u8") == ref.view("u8")).all(), v
        for _ in range(3):
            t0 = time.perf_counter()
            hcphmm.pairs(b, out)
            times[v].append(time.perf_counter() - t0)
        for _ in range(10):
            t0 = time.perf_counter()
            rcall()
            rt[v].append(time.perf_counter() - t0)
        regs()
        for _ in range(3):
            t0 = time.perf_counter()
            regs()
            mt[v].append(time.perf_counter() - t0)
for v in vals:
    m = statistics.median(times[v])
    print(json.dumps({"chunk_cells": v, "s2_ms": round(m * 1e3, 2), "s2_gcups": round(cells / m / 1e9, 1),
                      "region_415x128_ms": round(statistics.median(rt[v]) * 1e3, 3),
                      "regions64_ms": round(statistics.median(mt[v]) * 1e3, 2)}), flush=True)
