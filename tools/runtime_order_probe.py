"""Which order of runtime start-up works in one process: this library's HIP
runtime and torch's. usage: runtime_order_probe.py lib-first|torch-first"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
order = sys.argv[1]
import hcphmm  # noqa: E402
import torch  # noqa: E402

steps = [("lib", lambda: hcphmm.init(0)), ("torch", lambda: torch.full((4,), 1.0, device="cuda").sum().item())]
if order == "torch-first":
    steps.reverse()
for name, f in steps:
    try:
        f()
        print(order, name, "ok", flush=True)
    except Exception as e:  # noqa: BLE001
        print(order, name, "FAILED", type(e).__name__, str(e)[:120], flush=True)
