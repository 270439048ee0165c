"""Debug: which golden pairs differ per kernel setting (fp64 rescue path)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd"))
import hcphmm
g = np.load(os.path.join(ROOT, "tests", "golden", "pairhmm_golden.npz"), allow_pickle=False)
keys = ("read_off", "R", "hap_off", "H", "rs", "q", "ins", "dels", "gcp", "hap")
b = {k: g[k] for k in keys}
hcphmm.init(0)
names = list(g["set_names"])
for setting in [dict(), dict(HC_PHMM_KERNEL="diag"), dict(HC_PHMM_KERNEL="diag", HC_PHMM_RESCUE_ORDER="0"),
                dict(HC_PHMM_RESCUE_IN_WAVE="0")]:
    for k in ("HC_PHMM_KERNEL", "HC_PHMM_RESCUE_ORDER", "HC_PHMM_RESCUE_IN_WAVE"):
        os.environ.pop(k, None)
    os.environ.update(setting)
    bt = hcphmm.Batch(b)
    bt.run()
    r = bt.results()
    st = bt.stats()
    m = g["rescued"].astype(bool)
    bad = m & (r["raw_f64"].view(np.uint64) != g["raw_f64_all"].view(np.uint64))
    print(setting, "rescued", int(m.sum()), int(r["rescued"].sum()), "n_rescued", st.n_rescued,
          "bad f64", int(bad.sum()), "chain", st.rescue_chain)
    for s in range(len(names)):
        idx = np.flatnonzero(bad & (g["set_id"] == s))
        if len(idx):
            print("  ", names[s], len(idx), "of", int((m & (g["set_id"] == s)).sum()),
                  [(int(b["R"][i]), int(b["H"][i]), float(r["raw_f64"][i]), float(g["raw_f64_all"][i])) for i in idx[:4]])
    bt.close()
