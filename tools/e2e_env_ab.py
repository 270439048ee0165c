"""A/B of the S2 end-to-end flat call (hc_phmm_pairs_flat: host buffers in,
log10 likelihoods out) under HC_PHMM_* settings in one process: per setting a
first call, then the median of 5, alternating settings over 3 rounds so host
drift hits each alike; results checked identical across settings.
    python tools/e2e_env_ab.py HC_PHMM_FLAT_COMPACT=0,1 [HC_PHMM_PART_GROWTH_PCT=100,125]
Several VAR=... arguments form their cross product."""
import itertools
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

# "@name:K=V;K=V" arguments name whole settings (compared as they are, no
# cross product); the others are VAR=v1,v2 axes.
presets = [a for a in sys.argv[1:] if a.startswith("@")]
axes = [(a.split("=", 1)[0], a.split("=", 1)[1].split(",")) for a in sys.argv[1:] if not a.startswith("@")]
combos = list(itertools.product(*[[(k, v) for v in vals] for k, vals in axes]))
if presets:
    combos = [(("preset", a[1:].split(":", 1)[0]),) + tuple(tuple(kv.split("=", 1)) for kv in a.split(":", 1)[1].split(";") if kv)
              for a in presets]
all_keys = {k for c in combos for k, _ in c if k != "preset"}
hcphmm.init(0)
b = W.config("S2")
outs = [hcphmm.result_arrays(len(b["R"])) for _ in range(2)]
ref = None
times = {c: [] for c in combos}
for rnd in range(3):
    for c in combos:
        for k in all_keys:   # a setting that leaves a variable out runs with it unset
            os.environ.pop(k, None)
        for k, v in c:
            if k != "preset":
                os.environ[k] = v
        hcphmm.pairs(b, outs[0])
        if ref is None:
            ref = outs[0]["loglik"].copy()
        assert (outs[0]["loglik"].view("u8") == ref.view("u8")).all(), c
        for _ in range(2 if rnd else 1):
            t0 = time.perf_counter()
            hcphmm.pairs(b, outs[1])
            times[c].append((time.perf_counter() - t0) * 1e3)
cells = W.cells(b)
for c in combos:
    m = statistics.median(times[c])
    print(json.dumps(dict(dict(c), median_ms=round(m, 3), min_ms=round(min(times[c]), 3),
                          gcups=round(cells / (m * 1e-3) / 1e9, 1))), flush=True)
