import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd")
for p in (PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "pairhmm_golden.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden():
    g = np.load(GOLDEN, allow_pickle=False)
    return {k: g[k] for k in g.files}


@pytest.fixture(scope="session")
def golden_batch(golden):
    keys = ("read_off", "R", "hap_off", "H", "rs", "q", "ins", "dels", "gcp", "hap")
    return {k: golden[k] for k in keys}


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build(ref=False)
    return oracle.Oracle()


@pytest.fixture(scope="session")
def engine():
    """The HIP engine on cuda:0 (gpu tests only)."""
    import hcphmm
    bid = hcphmm.ensure_built()   # refuses a binary not built from this tree
    print(f"[engine] libhcpairhmm build id: {bid}")
    hcphmm.init(0)
    return hcphmm


SW_GOLDEN = os.path.join(ROOT, "tests", "golden", "sw_golden.npz")


@pytest.fixture(scope="session")
def sw_golden():
    """Reference aligner outputs (tests/golden/make_sw_golden.py): per set a flat
    batch, per case (set, params, strategy) offsets and CIGARs."""
    g = np.load(SW_GOLDEN, allow_pickle=False)
    d = {k: g[k] for k in g.files}
    sets = {}
    for k, v in d.items():
        if "__" in k:
            s, f = k.split("__", 1)
            sets.setdefault(s, {})[f] = v
    cases = []
    for c in d["cases"]:
        c = c.decode()
        parts = c.split("_")
        cases.append(dict(name=c, set=parts[0], params=tuple(int(x) for x in parts[1:5]),
                          strategy=int(parts[5]), offset=d[c + "_offset"],
                          cigar=[x.decode() for x in d[c + "_cigar"]]))
    return dict(sets=sets, cases=cases)


@pytest.fixture(scope="session")
def sw_oracle_lib():
    import oracle
    oracle.build(ref=False)
    return oracle.SWOracle()


GT_GOLDEN = os.path.join(ROOT, "tests", "golden", "gt_golden.npz")


@pytest.fixture(scope="session")
def gt_golden():
    """tests/golden/make_gt_golden.py: reference MathUtils outputs + site pins."""
    g = np.load(GT_GOLDEN, allow_pickle=False)
    d = {k: g[k] for k in g.files}
    sets = {}
    for name in ("std", "inf"):
        mats = [d[f"{name}_mat{k}"] for k in range(int(d[f"{name}_n_mats"]))]
        sites, ko, mo, go = [], 0, 0, 0
        exp = []
        for s in range(len(d[f"{name}_site_m"])):
            m = int(d[f"{name}_site_m"][s])
            A = int(d[f"{name}_site_A"][s])
            nk = int(d[f"{name}_keep_n"][s])
            nh = mats[m].shape[1]
            G = A * (A + 1) // 2
            sites.append(dict(m=m, n_alleles=A, keep=d[f"{name}_keep"][ko:ko + nk],
                              hap_allele=d[f"{name}_amap"][mo:mo + nh]))
            exp.append((d[f"{name}_gl"][go:go + G], int(d[f"{name}_gi"][s]), int(d[f"{name}_gq"][s])))
            ko, mo, go = ko + nk, mo + nh, go + G
        sets[name] = (mats, sites, exp)
    return dict(approx=(d["approx_a"], d["approx_b"], d["approx_out"]), sets=sets)


@pytest.fixture(scope="session")
def gt_oracle_lib():
    import oracle
    oracle.build(ref=False)
    return oracle.GTOracle()
