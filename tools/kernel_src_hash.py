"""Hash of the PairHMM device code's sources and build flags: a committed PMC
summary (profiles/r*_pmc_*.json) describes the kernels only while this hash is
unchanged; bench.py reports PMC traffic only when the hashes agree."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd", "csrc")
FILES = ["lane_kernel.hip", "seg_common.hpp", "kernels.hpp", "kernels.hip", "pack_kernels.hip", "luts.hpp",
         "device_common.hpp"]


def kernel_src_hash() -> str:
    h = hashlib.sha256()
    for f in FILES:
        h.update(f.encode())
        h.update(open(os.path.join(SRC, f), "rb").read())
    mk = open(os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd", "Makefile")).read()
    h.update("".join(ln for ln in mk.splitlines() if ln.startswith("DEV_FLAGS")).encode())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(kernel_src_hash())
