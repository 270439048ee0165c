"""S2 through the real call path (hc_phmm_pairs_flat: host buffers in, log10
likelihoods out), a few calls; HC_PHMM_TRACE=1 prints the host phases."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gatk-haplotypecaller-cpp17_amd"))
import numpy as np  # noqa: E402

import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

t0 = time.perf_counter()
hcphmm.init(0)
print(f"init: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
b = W.config(sys.argv[1] if len(sys.argv) > 1 else "S2")
if os.environ.get("N_FRAC"):   # put an 'N' base into this fraction of the reads (real reads carry them)
    frac = float(os.environ["N_FRAC"])
    rng = np.random.default_rng(7)
    rs = b["rs"].copy()
    picks = np.where(rng.random(len(b["R"])) < frac)[0]
    rs[b["read_off"][picks] + (b["R"][picks] // 2)] = ord("N")
    b = dict(b, rs=rs)
    print(f"reads with an N: {len(picks)}", flush=True)
cells = W.cells(b)
if os.environ.get("PRE_BATCH"):   # as bench.py: a resident batch of the same pairs created and run first
    bt = hcphmm.Batch(b)
    for _ in range(3):
        bt.run()
    print(f"resident batch: {bt.stats().run_ms:.2f} ms", flush=True)
out = hcphmm.result_arrays(len(b["R"]))
for v in out.values():
    v.fill(0)
ts = []
for k in range(int(os.environ.get("REPS", "5"))):
    t = time.perf_counter()
    r = hcphmm.pairs(b, out)
    dt = time.perf_counter() - t
    ts.append(dt)
    print(f"call {k}: {dt * 1e3:.1f} ms  {cells / dt / 1e9:.1f} GCUPS", flush=True)
print(f"median of calls 1..: {np.median(ts[1:]) * 1e3:.2f} ms  {cells / np.median(ts[1:]) / 1e9:.1f} GCUPS")
