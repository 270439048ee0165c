"""Instruction mix of a kernel's innermost loops from the gfx950 ISA (any
kernel; isa_step_breakdown.py is the PairHMM-specific version): for every
loop whose blocks LLVM annotates with one header ("; in Loop: Header=BBx_y
Depth=d" with no deeper loop inside), the count of VALU (and how many of them
are DPP moves, 64-bit or transcendental: two issue cycles), SALU, LDS, VMEM /
SMEM, s_waitcnt, s_nop (and the wait states they insert) and branch
instructions, plus the loop's blocks.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S \\
        -o sw.s gatk-haplotypecaller-cpp17_amd/csrc/sw_kernels.hip
    python tools/isa_loop_mix.py sw.s KERNEL_SUBSTRING [--json OUT]
"""
import json
import re
import sys
from collections import Counter, defaultdict


def kernel_body(lines, sub):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and sub in l.split(":")[0]:
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit(f"kernel {sub} not found")


def classify(op):
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_memrealtime")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    body = kernel_body(open(path).read().splitlines(), sub)
    blocks = []   # (label, header, depth, instructions)
    cur = None
    for l in body:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*(.*)$", l)
        if m:
            hm = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", m.group(2))
            lbl = m.group(1).lstrip(".L").replace("; %bb.", "bb.")
            if "Loop Header: Depth=" in m.group(2) or "Inner Loop Header: Depth=" in m.group(2):
                dm = re.search(r"Depth=(\d+)", m.group(2))
                hdr, depth = lbl, int(dm.group(1))
            elif hm:
                hdr, depth = hm.group(1), int(hm.group(2))
            else:
                hdr, depth = None, 0
            cur = [lbl, hdr, depth, []]
            blocks.append(cur)
            continue
        if cur is None:
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        cur[3].append(t)
    # The header line of a loop's first block carries "Loop Header" on the
    # next comment line in LLVM's output; fall back to "in Loop" membership.
    loops = defaultdict(list)
    depth = {}
    for lbl, hdr, d, ins in blocks:
        if hdr:
            loops[hdr].append(ins)
            depth[hdr] = max(depth.get(hdr, 0), d)
    parents = set()
    for lbl, hdr, d, ins in blocks:
        pass
    res = []
    for hdr, blist in loops.items():
        c = Counter()
        nops = 0
        for ins in blist:
            for t in ins:
                op = t.split()[0]
                k = classify(op)
                c[k] += 1
                if k == "s_nop":
                    nops += int(t.split()[1], 0) + 1
                if k == "valu":
                    if "_dpp" in op or "row_" in t or "wave_" in t:
                        c["valu_dpp"] += 1
                    if op.endswith(("_f64", "_b64_e32", "_u64", "_i64")) or "_f64_" in op:
                        c["valu_64bit"] += 1
        res.append(dict(loop=hdr, depth=depth[hdr], blocks=len(blist), counts=dict(c), nop_wait_states=nops))
    res.sort(key=lambda e: -sum(v for k, v in e["counts"].items() if k in ("valu", "salu", "lds", "vmem")))
    for e in res:
        print(json.dumps(e))
    if out:
        with open(out, "w") as f:
            for e in res:
                f.write(json.dumps(e) + "\n")


if __name__ == "__main__":
    main()
