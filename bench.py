#!/usr/bin/env python3
"""PairHMM throughput bench (GCUPS) for the MI355X engine.

    python bench.py [--gpus N --steps K --warmup W --workload S2]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Workload (BASELINE.json configs[2] / configs[3]): the seeded synthetic WGS-mix
batch S2 — 1 000 000 independent (read, hap) pairs, H ~ U[100, 500],
R ~ U[50, min(250, H)], 1 % substitutions, Phred U[10, 40] (+33), GOP 'I',
GCP '+' (SURVEY.md §8(d)). One step = the whole device pass of the hot path
over that batch: fp32 anti-diagonal kernel, device-built rescue list, fp64
rescue kernel; with N > 1 the same batch is sharded by cells over the ranks
(strong scaling) and the step ends with the RCCL gather of the per-pair raw
results to rank 0 (configs[3]). Inputs are resident in HBM before timing.

Prints one JSON line (rank 0). `value` = total cells / max-over-ranks wall time
of the K timed steps. `roofline` prices the dominant kernel (fp32 PairHMM) by
its algorithmic work, 12 fp32 mul/add per cell, against the non-FMA fp32 VALU
rate; `cpu_baseline` times the reference's own AVX kernel (oracle/_ref) on the
host cores, same batch.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "gatk-haplotypecaller-cpp17_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

VALU_PEAK_TOPS = 78.6      # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz, one f32 mul/add per lane-cycle
FLOPS_PER_CELL = 12        # computeMXY: 8 mul + 4 add (avx-pairhmm-template.h:183-198)
HBM_PEAK_GBS = 8000.0


def algorithmic_bytes(b):
    """Per pair: read rows 5 B x R + hap H B + 8 B result."""
    return int(5 * b["R"].astype(np.int64).sum() + b["H"].astype(np.int64).sum() + 8 * len(b["R"]))


def cpu_baseline(batch, threads, reps, sample_desc):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    kind = "reference"
    try:
        lib = oracle.Reference()
    except FileNotFoundError:
        lib, kind = oracle.Oracle(), "port"
    import workloads as W
    cells = W.cells(batch)
    best = None
    res = None
    for _ in range(reps):
        t0 = time.perf_counter()
        res = lib.pairs(batch, nthreads=threads)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return dict(value=cells / best / 1e9, unit="GCUPS", cores=threads, kind=kind,
                sample=sample_desc, seconds=round(best, 3)), res


def traffic_from_profiles(workload, cells):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary
    of this workload (profiles/*pmc*<workload>*.json, tools/pmc_summary.py),
    scaled by cells when this launch is a shard of the profiled one; else None."""
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc*{workload}*.json")))
    if not cands:
        return None, None
    try:
        d = json.load(open(cands[-1]))
        per_cell = d.get("hbm_bytes_per_cell")
        t = int(per_cell * cells) if per_cell else d.get("hbm_bytes_per_launch")
        return t, os.path.relpath(cands[-1], ROOT)
    except Exception:
        return None, None


SW_OPS_PER_CELL = 22       # MAIN_CODE int32 vector ops per cell (PairWiseSW.h:4-38)
INT32_VALU_PEAK_TOPS = 78.6   # 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz (wave64 issues over 2 cycles; no packed int32 ops)


def sw_secondary(no_cpu: bool):
    """Smith-Waterman on W2: 512 region windows (300-600
    bp) x 128 haplotypes, NEW_SW_PARAMETERS, SOFTCLIP, all-match shortcut — the
    graph_wrapper.hpp:232-240 loop for 512 regions in one device pass. Device
    pass timed with HIP events; the reference aligner (oracle/_ref, 1 thread,
    as the reference calls it) on the first 16 regions, checked for identical
    offsets and CIGARs."""
    import hcsw
    import sw_workloads as SWW
    hcsw.init(-1)   # the device the PairHMM engine was initialised on
    b = SWW.config("W2")
    bt = hcsw.Batch(b)
    for _ in range(2):
        bt.run()
    bt.stats()
    for _ in range(5):
        bt.run()
    st = bt.stats()
    off, cig = bt.results()
    bt.close()
    cells = st["cells"]
    tcups = cells / (st["dp_ms"] * 1e-3) / 1e12
    ent = dict(workload="W2", pairs=st["n_pairs"], shortcut_pairs=st["n_shortcut"], dp_cells=cells,
               dp_kernel_ms=round(st["dp_ms"], 3), trace_kernel_ms=round(st["trace_ms"], 3),
               device_pass_ms=round(st["run_ms"], 3), gcups=round(cells / (st["run_ms"] * 1e-3) / 1e9, 1),
               roofline=dict(bound="valu-int32", achieved=round(tcups * SW_OPS_PER_CELL, 2),
                             peak=INT32_VALU_PEAK_TOPS, unit="Top/s",
                             frac=round(tcups * SW_OPS_PER_CELL / INT32_VALU_PEAK_TOPS, 4),
                             note=f"{SW_OPS_PER_CELL} int32 ops/cell x DP cells / sw_dp_kernel time"))
    # one region through the host API (the real per-region call shape)
    one = SWW.config("W1")
    hcsw.align_flat(one)
    t0 = time.perf_counter()
    for _ in range(5):
        hcsw.align_flat(one)
    ent["region_415x128_call_ms"] = round((time.perf_counter() - t0) / 5 * 1e3, 3)
    if not no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        kind = "reference"
        try:
            ref = oracle.SWReference()
        except FileNotFoundError:
            ref, kind = oracle.SWOracle(), "port"
        nreg = 16
        idx = np.arange(nreg * 128)
        sub = SWW.subset(b, idx)
        t0 = time.perf_counter()
        r_off, r_cig = ref.batch(sub)
        dt = time.perf_counter() - t0
        same = np.array_equal(r_off, off[idx]) and r_cig == [cig[k] for k in idx]
        ent["cpu_baseline"] = dict(value=round(SWW.dp_cells(sub) / dt / 1e9, 3), unit="GCUPS", cores=1, kind=kind,
                                   sample=f"first {nreg} regions of W2 ({len(idx)} pairs), IntelSWAligner::align "
                                          f"semantics, 1 thread", seconds=round(dt, 3))
        ent["parity_vs_cpu_reference"] = "identical" if same else "MISMATCH"
        t0 = time.perf_counter()
        ref.batch(one)
        ent["region_415x128_cpu_reference_1core_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    return ent


def gt_secondary(no_cpu: bool):
    """Genotyper numeric core: 512 regions (415 reads x
    32 haps, normalised log10 likelihoods) x 16 variant sites, one call of
    hc_gt_genotype_sites with host buffers (the matrices' upload included); the
    oracle (C restatement, 1 thread) on the same sites beside it, compared bit
    for bit."""
    import hcgt
    import gt_workloads as GW
    mats, sites = GW.sites(n_regions=512, sites_per_region=16, reads=(415, 415), haps=(32, 32), seed=63)
    prep = hcgt.Prepared(mats, sites)
    prep.run()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        prep.run()
    dt = (time.perf_counter() - t0) / reps
    got = prep.results()
    ent = dict(regions=len(mats), sites=len(sites), call_ms=round(dt * 1e3, 3),
               note="host matrices in, per-site genotype likelihoods / GT / GQ out; 54 MB of likelihoods uploaded per call")
    if not no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        orc = oracle.GTOracle()
        import ctypes as C
        _f, _i = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        args = []
        for s in sites:   # marshal first: time the C loop, not ctypes
            L = mats[s["m"]]
            A = s["n_alleles"]
            gl = np.zeros(A * (A + 1) // 2)
            gi, gq = C.c_int32(), C.c_int32()
            args.append(((L.ctypes.data_as(_f), L.shape[1], s["keep"].ctypes.data_as(_i), len(s["keep"]),
                          s["hap_allele"].ctypes.data_as(_i), A, gl.ctypes.data_as(_f), C.byref(gi), C.byref(gq)),
                         gl, gi, gq))
        fn = orc.lib.hco_gt_site
        t0 = time.perf_counter()
        for a, *_ in args:
            fn(*a)
        dc = time.perf_counter() - t0
        exp = [(gl, gi.value, gq.value) for _, gl, gi, gq in args]
        same = all(np.array_equal(g[0].view(np.uint64), e[0].view(np.uint64)) and g[1] == e[1] and g[2] == e[2]
                   for g, e in zip(got, exp))
        ent["cpu_baseline"] = dict(value=round(dc * 1e3, 1), unit="ms", cores=1, kind="port",
                                   sample="same sites, oracle/gt_oracle.c (genotyper.hpp is not buildable here)")
        ent["parity_vs_cpu_oracle"] = "bit-exact" if same else "MISMATCH"
    return ent


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="S2", choices=["S1", "S1w", "S2", "S4"])
    ap.add_argument("--pairs", type=int, default=None, help="override pair count")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-reps", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip end-to-end and secondary configs")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--check", type=int, default=0,
                    help="rank 0 re-computes this many random pairs alone and compares them bit for bit "
                         "with the gathered multi-rank results")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    import hcphmm
    import shard
    import workloads as W

    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)   # several ranks per GPU only when rehearsing with gloo
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    gloo = args.dist_backend == "gloo"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if gloo:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    hcphmm.init(gpu)

    batch = W.config(args.workload, args.pairs)
    n_total = len(batch["R"])
    total_cells = W.cells(batch)
    shards = shard.shard_pairs(batch["R"], batch["H"], world)
    mine = shards[rank]
    sub = batch if world == 1 else W.subset(batch, mine)
    my_cells = W.cells(sub)
    nmax = max(len(s) for s in shards)

    bt = hcphmm.Batch(sub)
    raw32 = torch.zeros(nmax, dtype=torch.float32, device=dev)
    raw64 = torch.zeros(nmax, dtype=torch.float64, device=dev)
    flag = torch.zeros(nmax, dtype=torch.uint8, device=dev)
    bt.bind_outputs(raw32.data_ptr(), raw64.data_ptr(), flag.data_ptr())
    gdev = torch.device("cpu") if gloo else dev
    g32 = [torch.empty(nmax, dtype=torch.float32, device=gdev) for _ in range(world)] if (world > 1 and rank == 0) else None
    g64 = [torch.empty(nmax, dtype=torch.float64, device=gdev) for _ in range(world)] if (world > 1 and rank == 0) else None

    # The device pass and the gather run on one created stream: the library
    # enqueues on it (a created stream's handle is non-zero; 0 would select the
    # library's own stream, unordered with torch's), and RCCL / the gloo copy
    # to host then wait for the pass.
    stream = torch.cuda.Stream(device=dev)

    def step():
        with torch.cuda.stream(stream):
            bt.run(stream.cuda_stream)
            if world > 1:
                s32, s64 = (raw32.cpu(), raw64.cpu()) if gloo else (raw32, raw64)
                dist.gather(s32, gather_list=g32, dst=0)   # RCCL gather over xGMI
                dist.gather(s64, gather_list=g64, dst=0)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    bt.stats()   # reset the kernel event log: the averages below cover the timed steps only
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = bt.stats()
    ms_step = elapsed / args.steps * 1e3
    value = total_cells * args.steps / elapsed / 1e9

    # Dominant kernel: fp32 anti-diagonal PairHMM. Algorithmic work 12 ops/cell.
    k_ms = st.kernel_ms_f32
    achieved = FLOPS_PER_CELL * my_cells / (k_ms * 1e-3) / 1e12 if k_ms > 0 else 0.0
    traffic, tsrc = traffic_from_profiles(args.workload, my_cells)
    roofline = dict(bound="valu", achieved=round(achieved, 3), peak=VALU_PEAK_TOPS, unit="TFLOP/s",
                    frac=round(achieved / VALU_PEAK_TOPS, 4), traffic=traffic,
                    kernel=(("phmm_seg_kernel" if st.n_seg_waves > 0 else "phmm_lane_kernel")
                            if st.n_lane_pairs == st.n_pairs else "phmm_diag_kernel<float,16>"),
                    kernel_ms=round(k_ms, 4),
                    flops_per_cell=FLOPS_PER_CELL, cells_per_launch=my_cells,
                    hbm_algorithmic_GBs=round(algorithmic_bytes(sub) / (k_ms * 1e-3) / 1e9, 2) if k_ms > 0 else None,
                    hbm_peak_GBs=HBM_PEAK_GBS, traffic_source=tsrc)

    out = {
        "metric": "PairHMM GCUPS (cell updates/s), fp32 pass + fp64 rescue",
        "value": round(value, 2), "unit": "GCUPS", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "strong" if world > 1 else "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded generator, SURVEY.md §8(d))",
        "config": {"workload": f"{args.workload}: {n_total} independent pairs"
                               + (", H~U[100,500], R~U[50,min(250,H)], 1% subst" if args.workload == "S2" else ""),
                   "pairs": n_total, "cells": total_cells, "parallelism": f"pair-shard x{world}",
                   "rescued_fp64": int(st.n_rescued) if world == 1 else None},
        "roofline": roofline,
        "kernel_ms_f64": round(st.kernel_ms_f64, 4),
        "device_pass_ms": round(st.run_ms, 4),
    }

    cpu_res = None
    if rank == 0 and world == 1 and not args.no_cpu:
        thr = min(args.cpu_threads, os.cpu_count() or 1)
        cb, cpu_res = cpu_baseline(batch, thr, args.cpu_reps,
                                   f"the full {args.workload} batch ({n_total} pairs), {thr} OpenMP threads, "
                                   f"best of {args.cpu_reps}")
        out["cpu_baseline"] = cb
        if not args.no_extra:
            s1 = W.subset(batch, np.arange(min(n_total, 20_000)))
            c1, _ = cpu_baseline(s1, 1, 1, f"first {len(s1['R'])} pairs of {args.workload}, 1 thread")
            out["cpu_baseline_1core"] = c1

    if rank == 0 and world == 1:
        r = bt.results()
        out["config"]["rescued_fp64"] = int(r["rescued"].sum())
        if cpu_res is not None:
            same = all(np.array_equal(np.ascontiguousarray(r[k]).view(np.uint8),
                                      np.ascontiguousarray(cpu_res[k]).view(np.uint8))
                       for k in ("raw_f32", "rescued", "loglik"))
            out["parity_vs_cpu_reference"] = "bit-exact" if same else "MISMATCH"
    if rank == 0 and world == 1 and not args.no_extra:
        # First call grows the library's device/pinned workspace; later calls reuse it.
        t0 = time.perf_counter()
        hcphmm.pairs(batch)
        e2e_first = time.perf_counter() - t0
        e2e_reps = []
        for _ in range(3):
            t0 = time.perf_counter()
            hcphmm.pairs(batch)
            e2e_reps.append(time.perf_counter() - t0)
        e2e = float(np.median(e2e_reps))
        out["end_to_end_gcups"] = round(total_cells / e2e / 1e9, 2)
        out["end_to_end_ms"] = round(e2e * 1e3, 2)
        out["end_to_end_first_call_ms"] = round(e2e_first * 1e3, 2)
        out["end_to_end_note"] = ("host plan + pack + H2D + kernels + D2H + host log10, one call of "
                                  "hc_phmm_pairs_flat on host buffers (median of 3 after a first call "
                                  "that sizes the workspace)")
        sec = {}
        # S1w1M: the north star's 101x250 shape at a size that fills the chip
        # (S1/S1w are 10k-pair, latency-bound passes of < 0.15 ms).
        for name, npairs in (("S1", None), ("S1w", None), ("S1w1M", 1_000_000), ("S4", None)):
            b2 = W.config(name.replace("1M", ""), npairs)
            bb = hcphmm.Batch(b2)
            for _ in range(2):
                bb.run()
            bb.stats()
            for _ in range(5):
                bb.run()
            s2 = bb.stats()
            sec[name] = dict(pairs=len(b2["R"]), cells=W.cells(b2), device_pass_ms=round(s2.run_ms, 4),
                             gcups=round(W.cells(b2) / (s2.run_ms * 1e-3) / 1e9, 2),
                             kernel_ms_f32=round(s2.kernel_ms_f32, 4),
                             frac_f32_kernel=round(12 * W.cells(b2) / (s2.kernel_ms_f32 * 1e-3) / 78.6e12, 4)
                             if s2.kernel_ms_f32 > 0 else None,
                             rescued=int(s2.n_rescued))
            bb.close()
        # One active region, the real call shape of IntelPairHMM::compute_likelihoods:
        # 415 reads x n haps, hap ~415 bp, read 150 bp; host buffers in, doubles out.
        for nh in (32, 128):
            reads, haps = W.region(415, nh)
            hcphmm.cross(reads, haps)
            t0 = time.perf_counter()
            reps = 5
            for _ in range(reps):
                hcphmm.cross(reads, haps)
            dt = (time.perf_counter() - t0) / reps
            flat = W.region_flat(reads, haps)
            ent = dict(reads=len(reads), haps=nh, cells=W.cells(flat), call_ms=round(dt * 1e3, 3),
                       gcups=round(W.cells(flat) / dt / 1e9, 2))
            if not args.no_cpu:
                c1, _ = cpu_baseline(flat, 1, 1, "same region, 1 thread")
                ent["cpu_reference_1core_ms"] = round(c1["seconds"] * 1e3, 1)
            sec[f"region_415x{nh}"] = ent
        # Cross-region batching: 64 such regions (415 x 32) in one call.
        regs = [W.region(415, 32, seed=1000 + k) for k in range(64)]
        hcphmm.cross_regions(regs)
        t0 = time.perf_counter()
        hcphmm.cross_regions(regs)
        dt = time.perf_counter() - t0
        rc = sum(W.cells(W.region_flat(r, h)) for r, h in regs[:1]) * len(regs)
        sec["regions_64x_415x32_one_call"] = dict(regions=len(regs), cells_approx=rc, call_ms=round(dt * 1e3, 2),
                                                   gcups=round(rc / dt / 1e9, 2))
        sec["smith_waterman"] = sw_secondary(args.no_cpu)
        sec["genotyper"] = gt_secondary(args.no_cpu)
        out["secondary"] = sec
    if world > 1:
        out["gather"] = f"dist.gather ({'gloo, rehearsal' if gloo else 'RCCL'}) of raw_f32 + raw_f64 per step"
    if args.check and world > 1 and rank == 0:
        # Reassemble batch order from the last step's gathered shards and compare a
        # random sample with a single-process run of the same pairs.
        full32 = np.zeros(n_total, np.float32)
        full64 = np.zeros(n_total, np.float64)
        for r, sh in enumerate(shards):
            full32[sh] = g32[r][: len(sh)].cpu().numpy()
            full64[sh] = g64[r][: len(sh)].cpu().numpy()
        idx = np.sort(np.random.default_rng(7).choice(n_total, min(args.check, n_total), replace=False))
        ref = hcphmm.pairs(W.subset(batch, idx))
        ok = (np.array_equal(full32[idx].view(np.uint32), ref["raw_f32"].view(np.uint32)) and
              np.array_equal(full64[idx].view(np.uint64), ref["raw_f64"].view(np.uint64)))
        out["multi_rank_check"] = f"{len(idx)} pairs {'bit-exact' if ok else 'MISMATCH'}"
    bt.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
