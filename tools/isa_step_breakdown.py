"""Per-step instruction breakdown of the column-segmented step loops, from the
gfx950 ISA (verdict round 4, item 4: instructions per step by role).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
        -fgpu-flush-denormals-to-zero -fdenormal-fp-math=preserve-sign \
        -munsafe-fp-atomics -fno-slp-vectorize --cuda-device-only -S \
        -o lane.s gatk-haplotypecaller-cpp17_amd/csrc/lane_kernel.hip
    python tools/isa_step_breakdown.py lane.s KERNEL_SUBSTRING [--json OUT]

LLVM annotates every loop member block with its header ("; in Loop:
Header=BBx_y"), so each step loop is the set of blocks sharing a header. A
plain step hands off 2 values by DPP (Y and the right-edge T; 4 DPP moves in
fp64) and does 11 (EQ path) or 12 (generic) mul/add per cell; a row-sum step
hands off 2 more and adds 2 per cell. The loop's kind, steps and block width
BC are the reading of its DPP and arithmetic counts that gives a compiled
width (8-64, even). Issue slots price each instruction at the rates measured on
gfx950 (tools/ubench/op_rate.hip, profiles/r02_op_rate_ubench.jsonl): 1 for
the full-rate forms, 2 for the half-rate ones (DPP, v_bfe, v_bitop3, v_cmp,
v_lshl_*, v_cndmask on an SGPR mask, f64 arithmetic, any VOP3 with an SGPR
operand)."""
import collections
import json
import re
import sys

FULL = {"v_mul_f32", "v_add_f32", "v_sub_f32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32",
        "v_xor_b32", "v_not_b32", "v_lshrrev_b32", "v_ashrrev_i32", "v_mov_b32", "v_mov_b64"}


def role(op, txt):
    if "_dpp" in op or " wave_shr" in txt or "row_shr" in txt:
        return "handoff (DPP)"
    if op in ("v_mul_f32", "v_add_f32", "v_mul_f64", "v_add_f64"):
        return "cell arithmetic"
    if op in ("v_bfe_i32", "v_bitop3_b32", "v_bitop3_b16", "v_bfi_b32"):
        return "prior select"
    if op.startswith("v_cndmask") or op == "v_and_b32" and ("v" in txt.split(",")[-1] and "0x" not in txt):
        return "hand-off mask"
    if op.startswith("v_cmp") or op.startswith("s_"):
        return "row guard / loop (cmp, scalar)"
    if op.startswith("v_mov"):
        return "register moves"
    if op.startswith("global_") or op.startswith("ds_") or op.startswith("buffer_") or op.startswith("scratch_"):
        return "memory (read word, LDS priors, match row)"
    if op.startswith("v_"):
        return "row word / address arithmetic"
    return "other"


def slots(op, txt):
    if not op.startswith("v_"):
        return 0.0
    sgpr_operand = re.search(r"[ ,]s\[?\d", txt.split(op, 1)[1]) is not None
    if op in FULL and "_dpp" not in op and "_e64" not in txt.split()[0] and not sgpr_operand:
        return 1.0
    if op == "v_cndmask_b32" and txt.split()[0].endswith("_e32"):
        return 1.0
    return 2.0


def main():
    path, kname = sys.argv[1], sys.argv[2]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if re.match(r"^_Z\S*:", ln) and kname in ln)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    loops = collections.defaultdict(list)   # header -> [(op, txt)]
    cur = None
    lab = None   # the last label: its loop-header note may follow on a comment line
    for ln in lines[start:end]:
        m = re.match(r"^\.(LBB\w+):\s*;?\s*(.*)$", ln)
        if m:
            lab, com = m.group(1), m.group(2)
            h = re.search(r"Header=(BB\w+)", com)
            if "Loop Header" in com:
                cur = lab[1:]
            elif h:
                cur = h.group(1)
            else:
                cur = None
            continue
        if lab is not None and re.match(r"^\s+;.*Loop Header", ln):
            # ".LBBx:  ; Parent Loop BBy" then ";  =>  This Inner Loop Header":
            # the label heads an inner loop (a one-block step loop has no
            # other member blocks, so without this it was missed).
            cur = lab[1:]
            continue
        if not ln.lstrip().startswith(";"):
            lab = None
        s = ln.strip()
        if cur is None or not s or s.startswith(";") or s.startswith("."):
            continue
        loops[cur].append((re.sub(r"_e(32|64)$", "", s.split()[0]), s))
    rows = []
    for hdr, ins in loops.items():
        c = collections.Counter(op for op, _ in ins)
        f32 = c["v_mul_f32"] + c["v_add_f32"]
        f64 = c["v_mul_f64"] + c["v_add_f64"]
        dpp = sum(1 for op, t in ins if "_dpp" in op)
        if dpp == 0 or (f32 < 100 and f64 < 100):
            continue
        fp64 = f64 > f32
        arith = f64 if fp64 else f32
        dpp_plain = 4 if fp64 else 2
        guess = None
        for sums, per_cell in ((False, 11), (False, 12), (True, 13), (True, 14)):
            steps = dpp // (dpp_plain * (2 if sums else 1))
            if steps and arith % (steps * per_cell) == 0:
                bc = arith // (steps * per_cell)
                if 8 <= bc <= 64 and bc % 2 == 0:
                    guess = (sums, steps, bc, per_cell == 11 or per_cell == 13)
                    break
        if guess is None:
            continue
        sums, steps, bc, eq = guess
        by_role = collections.Counter()
        by_slot = collections.Counter()
        for op, t in ins:
            r = role(op, t)
            by_role[r] += 1
            by_slot[r] += slots(op, t)
        rows.append(dict(loop=hdr, fp64=fp64, bc=bc, eq=eq, row_sums=sums, steps_per_iteration=steps,
                         arith_per_step=arith / steps,
                         instr_per_step={k: round(v / steps, 2) for k, v in by_role.items()},
                         slots_per_step={k: round(v / steps, 2) for k, v in by_slot.items()},
                         total_instr_per_step=round(len(ins) / steps, 2),
                         valu_instr_per_step=round(sum(n for op, n in c.items() if op.startswith("v_")) / steps, 2),
                         valu_slots_per_step=round(sum(by_slot.values()) / steps, 2)))
    rows.sort(key=lambda r: (r["fp64"], not r["eq"], r["row_sums"], r["bc"]))
    for r in rows:
        print(json.dumps(r))
    if out_json:
        with open(out_json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
