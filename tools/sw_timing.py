"""Time the HIP Smith-Waterman pass on W2 (device-resident) and the reference aligner on a sample."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd"), os.path.join(ROOT, "oracle")]
import hcsw, sw_workloads as S
hcsw.init(0)
for name in sys.argv[1:] or ["W2"]:
    b = S.config(name)
    t = time.time(); bt = hcsw.Batch(b); t_create = time.time() - t
    bt.run(); bt.stats()
    for _ in range(5): bt.run()
    st = bt.stats()
    t = time.time(); bt.results(); t_res = time.time() - t
    st.update(name=name, create_s=t_create, results_s=t_res,
              tcups_dp=st["cells"] / (st["dp_ms"] * 1e-3) / 1e12, gcups_run=st["cells"] / (st["run_ms"] * 1e-3) / 1e9)
    print(json.dumps(st), flush=True)
# one region through the synchronous host API (hc_sw_align_flat)
one = S.config("W1")
hcsw.align_flat(one)
t = time.time()
for _ in range(20):
    hcsw.align_flat(one)
print(json.dumps({"region_415x128_call_ms": (time.time() - t) / 20 * 1e3}))
