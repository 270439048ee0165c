"""Packing model for configs[1] (S1: 10 000 pairs, R = 101, H = 150) on the
fp32 column-segmented kernel (verdict round 5, item 6): every way to lay the
batch out as seg waves, priced before any GPU time.

A pair of hap length H at block width BC takes nb = ceil(H / BC) consecutive
lanes; a wave holds floor(64 / nb) pairs (or fewer) and runs R + nb - 1 steps
of BC columns per lane. The pass is one round when the waves
fit the resident slots, and then lasts as long as its busiest SIMD: waves are
dealt to the 1 024 SIMDs in order, so a SIMD holds ceil(W / 1024) or
floor(W / 1024) waves. Two prices per layout:

  cell_share    cells / (64 lanes x steps x BC) over the waves: the fraction of
                the lane-column-steps swept that are cells (S1 today: 0.762)
  simd_work     the busiest SIMD's lane-column-steps (waves x steps x BC) plus
                the per-step overhead (12 instructions per step, ~0.86 cell
                equivalents of 14 per cell, isa_step_breakdown), relative to
                today's layout (BC 14, 5 pairs per wave, 2 000 waves)

Layouts: every compiled BC (8-64, even) with the lanes per pair nb and nb + 1
(the planner's two candidates), any pairs-per-wave count up to the lane limit,
at the kernel's occupancy limit of 3 waves per SIMD; plus two packings the
verdict named — pairs of a wave sharing lanes across R (moot here: every S1
read has R = 101) and two pairs streamed through the same lanes one after the
other (one skew for two pairs, half the waves).

    python tools/s1_packing_model.py [out.jsonl]
"""
import json
import math
import sys

N, R, H = 10_000, 101, 150
SIMDS = 1024
OCC = 3
STEP_OVERHEAD = 12 / 14.0   # per-step instructions in cell units (13.8-14 instructions per cell)


def layout(bc, nb, ppw, streamed=1):
    """ppw pairs per wave side by side, each over nb lanes of bc columns;
    `streamed` pairs one after the other on the same lanes."""
    if nb * bc < H or nb * ppw > 64:
        return None
    pairs_per_wave = ppw * streamed
    waves = math.ceil(N / pairs_per_wave)
    if waves > OCC * SIMDS:
        return None
    steps = streamed * R + nb - 1
    per_simd = math.ceil(waves / SIMDS)
    cells = N * R * H
    swept = waves * 64 * steps * bc
    simd_work = per_simd * steps * (bc + STEP_OVERHEAD)
    return dict(bc=bc, nb=nb, pairs_per_wave=ppw, streamed=streamed, waves=waves, steps=steps,
                waves_per_simd_max=per_simd, cell_share=round(cells / swept, 4), simd_work=simd_work)


rows = []
for bc in range(8, 66, 2):
    for nb in (math.ceil(H / bc), math.ceil(H / bc) + 1):
        for ppw in range(1, 64 // nb + 1):
            for streamed in (1, 2):
                e = layout(bc, nb, ppw, streamed)
                if e:
                    rows.append(e)
base = layout(14, 11, 5)
for e in rows:
    e["simd_work_vs_today"] = round(e["simd_work"] / base["simd_work"], 4)
    e.pop("simd_work")
rows.sort(key=lambda e: e["simd_work_vs_today"])
best = rows[0]
share_ok = [e for e in rows if e["cell_share"] > 0.80 and e["waves_per_simd_max"] <= 2]
summary = dict(today=dict(bc=14, nb=11, pairs_per_wave=5, waves=2000, cell_share=base["cell_share"]),
               best_by_simd_work=best,
               best_with_cell_share_above_0_80_at_2_per_simd=min(share_ok, key=lambda e: e["simd_work_vs_today"])
               if share_ok else None,
               layouts_priced=len(rows),
               layouts_10pct_better=sum(1 for e in rows if e["simd_work_vs_today"] <= 0.90))
print(json.dumps(summary))
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        f.write(json.dumps(summary) + "\n")
        for e in rows:
            f.write(json.dumps(e) + "\n")
