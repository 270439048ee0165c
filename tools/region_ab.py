"""A/B of the one-region call (hc_phmm_cross, 415 reads x N haps) under
HC_PHMM_* settings, in one process: for each setting, 5 warm-up calls then
the median of 30 timed calls, alternating settings across 3 rounds so that
host-clock drift hits every setting alike.
    python tools/region_ab.py 128 HC_PHMM_MIN_CHUNKS=1,2,3 [VAR=a,b ...]
Several VAR=... arguments form their cross product.
"""
import itertools
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

nh = int(sys.argv[1])
axes = [(a.split("=", 1)[0], a.split("=", 1)[1].split(",")) for a in sys.argv[2:]]
vals = list(itertools.product(*[[(k, v) for v in vs] for k, vs in axes]))
hcphmm.init(0)
reads, haps = W.region(415, nh)
call = hcphmm.CrossCall(reads, haps)
ref = None
times = {v: [] for v in vals}
for rnd in range(3):
    for v in vals:
        for k, x in v:
            os.environ[k] = x
        for _ in range(5):
            out = call().copy()
        if ref is None:
            ref = out
        assert (out.view("u8") == ref.view("u8")).all(), v
        for _ in range(30):
            t0 = time.perf_counter()
            call()
            times[v].append((time.perf_counter() - t0) * 1e3)
for v in vals:
    print(json.dumps({"haps": nh, **dict(v), "median_ms": round(statistics.median(times[v]), 3),
                      "min_ms": round(min(times[v]), 3)}), flush=True)
