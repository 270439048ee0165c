"""SW DP kernel time of W2 / W3 at warm clocks (0.3 s of back-to-back passes,
then 10 timed), for A/B between library builds (HC_PHMM_LIB)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd")]
import hcsw  # noqa: E402
import sw_workloads as S  # noqa: E402

hcsw.init(0)
out = {}
for name in sys.argv[1:] or ["W2", "W3"]:
    bt = hcsw.Batch(S.config(name))
    t0, k = time.perf_counter(), 0
    while k < 3 or time.perf_counter() - t0 < 0.3:
        bt.run()
        k += 1
        if k % 4 == 0:
            bt.stats()
    bt.stats()
    for _ in range(10):
        bt.run()
    st = bt.stats()
    out[name] = round(st["dp_ms"], 4)
print(json.dumps(out), flush=True)
