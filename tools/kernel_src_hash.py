"""Hashes of the PairHMM engine's sources and build flags.

kernel_src_hash(): the device kernels only — a committed PMC summary
(profiles/r*_pmc_*.json) describes the kernels while this hash is unchanged;
bench.py reports PMC traffic only when the hashes agree.

lib_src_hash(): every source of libhcpairhmm.so (csrc/, include/, the
Makefile's flag lines, the Jacobian table generator).

    python tools/kernel_src_hash.py                  # kernel hash
    python tools/kernel_src_hash.py --header OUT.h [--extra "FLAGS"]
                                                     # both hashes + git HEAD as C macros

The Makefile compiles that header into the library (hc_phmm_build_id()), so a
run can prove which sources the binary it loaded was built from: bench.py and
__graft_entry__.smoke() compare the library's hashes with the tree's and
refuse a stale binary. The Makefile passes its EXTRA_DEV_FLAGS (A/B builds,
e.g. -DHC_SEG_WPB=4) with --extra: a non-empty value enters both hashes, so
such a build never matches the tree and is loaded only as an A/B build
(hcphmm.py: HC_PHMM_LIB with HC_PHMM_AB=1)."""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd")
SRC = os.path.join(PKG, "csrc")
FILES = ["lane_kernel.hip", "seg_common.hpp", "kernels.hpp", "kernels.hip", "pack_kernels.hip", "luts.hpp",
         "device_common.hpp"]


def _flag_lines(prefixes):
    mk = open(os.path.join(PKG, "Makefile")).read()
    return "".join(ln for ln in mk.splitlines() if ln.startswith(prefixes)).encode()


def kernel_src_hash(extra: str = "") -> str:
    h = hashlib.sha256()
    for f in FILES:
        h.update(f.encode())
        h.update(open(os.path.join(SRC, f), "rb").read())
    h.update(_flag_lines(("DEV_FLAGS",)))
    if extra.strip():
        h.update(b"EXTRA_DEV_FLAGS=" + extra.strip().encode())
    return h.hexdigest()[:16]


def lib_src_hash(extra: str = "") -> str:
    h = hashlib.sha256()
    files = [os.path.join(SRC, f) for f in sorted(os.listdir(SRC))]
    inc = os.path.join(ROOT, "include")
    files += [os.path.join(inc, f) for f in sorted(os.listdir(inc))]
    files.append(os.path.join(ROOT, "tools", "gen_jacobian.py"))
    for p in files:
        if not os.path.isfile(p):
            continue
        h.update(os.path.relpath(p, ROOT).encode())
        h.update(open(p, "rb").read())
    h.update(_flag_lines(("DEV_FLAGS", "HOST_FLAGS")))
    if extra.strip():
        h.update(b"EXTRA_DEV_FLAGS=" + extra.strip().encode())
    return h.hexdigest()[:16]


def git_head() -> str:
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip()
        dirty = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--untracked-files=no"],
                               capture_output=True, text=True, timeout=10).stdout.strip()
        return (head or "unknown") + ("-dirty" if head and dirty else "")
    except (OSError, subprocess.SubprocessError):
        return "unknown"


def write_header(path: str, extra: str = "") -> None:
    txt = (f'#define HC_KERNEL_SRC_HASH "{kernel_src_hash(extra)}"\n'
           f'#define HC_LIB_SRC_HASH "{lib_src_hash(extra)}"\n'
           f'#define HC_GIT_HEAD "{git_head()}"\n')
    try:
        if open(path).read() == txt:
            return   # unchanged: keep the timestamp (no relink)
    except OSError:
        pass
    with open(path, "w") as f:
        f.write(txt)


if __name__ == "__main__":
    if len(sys.argv) in (3, 5) and sys.argv[1] == "--header":
        write_header(sys.argv[2], sys.argv[4] if len(sys.argv) == 5 and sys.argv[3] == "--extra" else "")
    elif len(sys.argv) == 2 and sys.argv[1] == "--lib":
        print(lib_src_hash())
    else:
        print(kernel_src_hash())
