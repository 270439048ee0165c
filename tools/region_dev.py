"""Device time of one region call (hc_phmm_cross, 415 reads x N haps) under
HC_PHMM_* settings: each setting in its own child process with
HC_PHMM_TRACE=1; the medians of the traced device phases (fp32 pass, fp64
pass) and of the call over 20 calls after 5 warm-up calls.
    python tools/region_dev.py 128 HC_PHMM_SEG_Q=-1,0,1 [VAR=...]
"""
import itertools
import json
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time
sys.path.insert(0, os.path.join(%r, "gatk-haplotypecaller-cpp17_amd"))
import hcphmm, workloads as W
hcphmm.init(0)
reads, haps = W.region(415, %d)
call = hcphmm.CrossCall(reads, haps)
for k in range(25):
    t0 = time.perf_counter(); call(); t1 = time.perf_counter()
    print("CALL %%.4f" %% ((t1 - t0) * 1e3), file=sys.stderr, flush=True)
'''
nh = int(sys.argv[1])
specs = [a.split("=", 1) for a in sys.argv[2:]]
grid = list(itertools.product(*[[(k, v) for v in vals.split(",")] for k, vals in specs]))
for combo in grid:
    env = dict(os.environ, HC_PHMM_TRACE="1", **dict(combo))
    p = subprocess.run([sys.executable, "-c", CHILD % (ROOT, nh)], env=env, capture_output=True, text=True,
                       timeout=120)
    if p.returncode:
        sys.stderr.write(p.stderr[-2000:])
        sys.exit(1)
    f32 = [float(x) for x in re.findall(r"fp32 ([0-9.]+) ms", p.stderr)][5:]
    f64 = [float(x) for x in re.findall(r"fp64 ([0-9.]+) ms", p.stderr)][5:]
    call = [float(x) for x in re.findall(r"CALL ([0-9.]+)", p.stderr)][5:]
    print(json.dumps(dict(haps=nh, settings=dict(combo), fp32_ms=statistics.median(f32),
                          fp64_ms=statistics.median(f64), call_ms=statistics.median(call))), flush=True)
