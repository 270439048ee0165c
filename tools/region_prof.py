"""Driver for the region profile (tools/profile_r03.sh region): W warm-up then
C timed hc_phmm_cross calls on one 415 reads x N haps active region (the call
shape of haplotypecaller.hpp:103); prints the call count and the pairs/cells of
one call for tools/profile_summary.py --calls."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import workloads as W  # noqa: E402

nh = int(sys.argv[1]) if len(sys.argv) > 1 else 128
warm, calls = 5, 30
hcphmm.init(0)
reads, haps = W.region(415, nh)
call = hcphmm.CrossCall(reads, haps)
for _ in range(warm + calls):
    call()
print(json.dumps(dict(calls=warm + calls, warm=warm, cells=W.cells(W.region_flat(reads, haps)))))
