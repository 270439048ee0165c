// Device-side packing and planning of a batch (the reference's getData /
// precompute_masks work, intel_pairhmm.hpp:154-203 and
// avx-pairhmm-template.h:3-35, done once per read and once per haplotype
// instead of once per pair).
//
//   pack_reads   uploaded read bytes -> one uint32 row word per base
//                (kernels.hpp pack_row). The upload carries 2 bytes per base
//                (base, quality); a read whose gap qualities are constant —
//                every read the reference builds, sam.hpp:30-32,47-49 — sends
//                them once in its descriptor, the others send 3 more planes.
//   hap_tables   hap bytes -> per-hap match table, (ceil(H/32) + 3) rows of 5
//                words: bit (MSB first) per column for read codes 0..4.
//   grid_*       descriptors, slot order and waves of a structured
//                (cross-product) plan from its block and segment tables.
//   flat_*       a flat batch planned on the device: rows, tables, each pair's
//                segmented shape, a counting sort and the waves (flat_plan.cpp).
//
// The packers are byte-streaming kernels, one wave per read / per haplotype
// (coalesced byte loads across the wave; the match words come from ballots).
#include <algorithm>

#include "kernels.hpp"

namespace hcphmm {
namespace {

// ConvertChar (pairhmm_common.h:26-44): A0 C1 T2 G3 N4, every other byte -> 0.
__device__ __forceinline__ uint32_t base_code(uint32_t b)
{
    return b == 'C' ? 1u : b == 'T' ? 2u : b == 'G' ? 3u : b == 'N' ? 4u : 0u;
}

// Row words of one read, lanes over rows (a wave). gw: constant gap qualities
// i | d << 7 | c << 14 (already & 127), or -1 when they vary: then the i, d, c
// planes are at gi, gd, gc.
__device__ __forceinline__ void pack_read(const uint8_t* __restrict__ bases, const uint8_t* __restrict__ quals,
                                          const uint8_t* __restrict__ gi, const uint8_t* __restrict__ gd,
                                          const uint8_t* __restrict__ gc, int len, int gw, uint32_t* __restrict__ rows,
                                          int lane)
{
    for (int k = lane; k < len; k += 64) {
        const uint32_t q = quals[k] & 127u;
        const uint32_t code = base_code(bases[k]) << 28;
        uint32_t w;
        if (gw >= 0) {
            w = q | (uint32_t(gw) << 7) | code;
            if (k == 0) w |= 0x80000000u;   // constant-gap tag on the read's first row
        } else {
            w = q | ((gi[k] & 127u) << 7) | ((gd[k] & 127u) << 14) | ((gc[k] & 127u) << 21) | code;
        }
        rows[k] = w;
    }
}

// One wave per read (grid-stride). rdesc: {row offset, length, constant gap
// qualities or -1, offset of the read's rows in the i/d/c planes when they vary}.
__device__ __forceinline__ void pack_reads(const uint8_t* __restrict__ bases, const uint8_t* __restrict__ quals,
                                           const uint8_t* __restrict__ gaps, long long gap_stride,
                                           const int4* __restrict__ rdesc, int nreads, uint32_t* __restrict__ rows)
{
    const int lane = threadIdx.x & 63;
    for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < nreads; r += gridDim.x * 4) {
        const int4 d = rdesc[r];
        const int off = __builtin_amdgcn_readfirstlane(d.x), len = __builtin_amdgcn_readfirstlane(d.y);
        const int gw = __builtin_amdgcn_readfirstlane(d.z), goff = __builtin_amdgcn_readfirstlane(d.w);
        const uint8_t* g = gaps + goff;
        pack_read(bases + off, quals + off, g, g + gap_stride, g + 2 * gap_stride, len, gw, rows + off, lane);
    }
}

// Match table of one haplotype (a wave): row w + kHapLead holds columns
// 32w+1 .. 32w+32; lanes 0-31 take the columns of row w, lanes 32-63 those of
// row w+1, and the wave ballot of "hap base matches read code rc" gives both
// rows' words for rc at once (bit-reversed: column 1 is the MSB).
__device__ __forceinline__ void hap_table(const uint8_t* __restrict__ hb, int H, uint32_t* __restrict__ o, int lane)
{
    const int nw = (H + 31) / 32;
    // Zero rows: kHapLead before the data, one after.
    if (lane < 5 * kHapLead) o[lane] = 0u;
    if (lane < 5) o[(kHapLead + nw) * 5 + lane] = 0u;
    for (int w0 = 0; w0 < nw; w0 += 2) {
        const int col = w0 * 32 + lane;   // 0-based hap column
        const uint32_t hc = col < H ? base_code(hb[col]) : 7u;   // 7: past the hap, no match
        uint32_t word = 0u;
#pragma unroll
        for (int rc = 0; rc < 5; ++rc) {
            // read code rc matches: equal code, hap 'N' (matches every rc), or read 'N'
            const bool m = hc != 7u && (hc == uint32_t(rc) || hc == 4u || rc == 4);
            const uint64_t bl = __builtin_amdgcn_ballot_w64(m);
            const uint32_t lo = __builtin_bitreverse32(uint32_t(bl)), hi = __builtin_bitreverse32(uint32_t(bl >> 32));
            if (lane == rc) word = lo;
            if (lane == 5 + rc) word = hi;
        }
        if (lane < 5) o[(kHapLead + w0) * 5 + lane] = word;
        if (lane >= 5 && lane < 10 && w0 + 1 < nw) o[(kHapLead + w0 + 1) * 5 + lane - 5] = word;
    }
}

// One wave per haplotype (grid-stride); haps[h] = {byte offset, H, table word offset, 0}.
__device__ __forceinline__ void hap_tables(const uint8_t* __restrict__ hap_bytes, const int4* __restrict__ haps,
                                           int nhaps, uint32_t* __restrict__ hapw)
{
    const int lane = threadIdx.x & 63;
    for (int h = blockIdx.x * 4 + (threadIdx.x >> 6); h < nhaps; h += gridDim.x * 4) {
        const int4 hd = haps[h];
        const int off = __builtin_amdgcn_readfirstlane(hd.x), H = __builtin_amdgcn_readfirstlane(hd.y);
        hap_table(hap_bytes + off, H, hapw + __builtin_amdgcn_readfirstlane(hd.z), lane);
    }
}

__device__ __forceinline__ void grid_pairs(const GridBlock* __restrict__ blocks, int nblocks, long long npairs,
                                           const int4* __restrict__ rdesc, const int4* __restrict__ hdesc,
                                           PairDesc* __restrict__ pairs)
{
    for (long long k = blockIdx.x * 256ll + threadIdx.x; k < npairs; k += 256ll * gridDim.x) {
        int lo = 0, hi = nblocks;   // the last block with p0 <= k (empty blocks share their successor's p0)
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (blocks[mid].p0 <= k) lo = mid;
            else hi = mid;
        }
        const GridBlock b = blocks[lo];
        const long long off = k - b.p0;
        const int r = b.r0 + int(off / b.nh), h = b.h0 + int(off % b.nh);
        const int4 rd = rdesc[r], hd = hdesc[h];
        pairs[k] = make_int4(rd.x, rd.y, hd.z, hd.y);
    }
}

__device__ __forceinline__ void grid_waves(const GridSeg* __restrict__ segs, int nsegs, long long nslots, int nwaves,
                                           const int* __restrict__ rord, const int* __restrict__ hord,
                                           const int4* __restrict__ rdesc, int* __restrict__ order,
                                           LaneWave* __restrict__ waves)
{
    const long long stride = 256ll * gridDim.x;
    for (long long t = blockIdx.x * 256ll + threadIdx.x; t < nslots; t += stride) {
        int lo = 0, hi = nsegs;   // the last segment with slot0 <= t
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (segs[mid].slot0 <= t) lo = mid;
            else hi = mid;
        }
        const GridSeg g = segs[lo];
        const long long i = t - g.slot0;
        const int rr = int(i / g.G), hh = int(i % g.G);
        order[t] = int(g.p0 + (long long)(rord[g.r0 + rr] - g.r0) * g.nh + (hord[g.g0 + hh] - g.h0));
    }
    for (long long w = blockIdx.x * 256ll + threadIdx.x; w < nwaves; w += stride) {
        int lo = 0, hi = nsegs;   // the last segment with w0 <= w (segments without waves share w0)
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (segs[mid].w0 <= w) lo = mid;
            else hi = mid;
        }
        const GridSeg g = segs[lo];
        const int per = 64 / g.nb;
        const long long n = (long long)g.nr * g.G, a = (w - g.w0) * (long long)per;
        const long long e = a + per < n ? a + per : n;
        const int rmax = rdesc[rord[g.r0 + int(a / g.G)]].y;
        const int rmin = rdesc[rord[g.r0 + int((e - 1) / g.G)]].y;
        LaneWave v;
        v.slot0 = int(g.slot0 + a);
        v.rmax = rmax;
        v.rmin = rmin;
        v.ncols = g.bc;
        v.npairs = int(e - a);
        v.nsteps = rmax + g.nb - 1;
        v.carry_row = 0;
        waves[w] = v;
    }
}

__global__ __launch_bounds__(256) void grid_pairs_kernel(const GridBlock* __restrict__ blocks, int nblocks,
                                                         long long npairs, const int4* __restrict__ rdesc,
                                                         const int4* __restrict__ hdesc, PairDesc* __restrict__ pairs)
{
    grid_pairs(blocks, nblocks, npairs, rdesc, hdesc, pairs);
}

__global__ __launch_bounds__(256) void grid_waves_kernel(const GridSeg* __restrict__ segs, int nsegs,
                                                         long long nslots, int nwaves, const int* __restrict__ rord,
                                                         const int* __restrict__ hord, const int4* __restrict__ rdesc,
                                                         int* __restrict__ order, LaneWave* __restrict__ waves)
{
    grid_waves(segs, nsegs, nslots, nwaves, rord, hord, rdesc, order, waves);
}

__global__ __launch_bounds__(256) void pack_reads_kernel(const uint8_t* __restrict__ bases,
                                                         const uint8_t* __restrict__ quals,
                                                         const uint8_t* __restrict__ gaps, long long gap_stride,
                                                         const int4* __restrict__ rdesc, int nreads,
                                                         uint32_t* __restrict__ rows)
{
    pack_reads(bases, quals, gaps, gap_stride, rdesc, nreads, rows);
}

__global__ __launch_bounds__(256) void hap_tables_kernel(const uint8_t* __restrict__ hap_bytes,
                                                         const int4* __restrict__ haps, int nhaps,
                                                         uint32_t* __restrict__ hapw)
{
    hap_tables(hap_bytes, haps, nhaps, hapw);
}

// Everything a structured (region) part needs before its pass, in one launch
// (each step is a grid-stride loop over its own items; none reads another's
// output): the run counters zeroed, reads packed, hap tables, pair
// descriptors, slot order and waves — four fewer launches per region call.
__global__ __launch_bounds__(256) void prepare_grid_kernel(GridPrepArgs a)
{
    if (blockIdx.x == 0 && threadIdx.x < kNumCounters) a.counters[threadIdx.x] = 0;
    pack_reads(a.bases, a.quals, a.gaps, a.gap_stride, a.rdesc, a.nreads, a.rows);
    hap_tables(a.hap_bytes, a.hdesc, a.nhaps, a.hapw);
    grid_pairs(a.blocks, a.nblocks, a.npairs, a.rdesc, a.hdesc, a.pairs);
    grid_waves(a.segs, a.nsegs, a.nslots, a.nwaves, a.rord, a.hord, a.rdesc, a.order, a.waves);
}

// ---------------------------------------------------------------------------
// Flat batches planned on the device (kernels.hpp FlatPlanArgs).

// Flat records (flat_plan.cpp, kernels.hpp FlatDesc): the read's base
// qualities, its base codes as nibbles (ConvertChar, two per byte, row k in
// the low nibble of byte k/2 when k is even), its i / d / c planes when they
// vary, then the hap's base codes as nibbles; every field 4-byte aligned.
__host__ __device__ constexpr int align4(int x) { return (x + 3) & ~3; }

// Rows of one read from its record, four rows per lane (one 32-bit load of
// qualities, one 16-bit load of codes, one 128-bit store).
__device__ __forceinline__ void pack_read_rec(const uint8_t* __restrict__ quals, const uint8_t* __restrict__ codes,
                                              const uint8_t* __restrict__ gaps, int R, int gw,
                                              uint32_t* __restrict__ rows, int lane)
{
    const int qa = align4(R);
    for (int t = lane; 4 * t < R; t += 64) {
        const uint32_t q4 = reinterpret_cast<const uint32_t*>(quals)[t];
        const uint32_t c4 = reinterpret_cast<const uint16_t*>(codes)[t];
        uint32_t w[4];
        if (gw >= 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                w[j] = ((q4 >> (8 * j)) & 127u) | (uint32_t(gw) << 7) | (((c4 >> (4 * j)) & 15u) << 28);
            if (t == 0) w[0] |= 0x80000000u;   // constant-gap tag on the read's first row
        } else {
            const uint32_t i4 = reinterpret_cast<const uint32_t*>(gaps)[t];
            const uint32_t d4 = reinterpret_cast<const uint32_t*>(gaps + qa)[t];
            const uint32_t g4 = reinterpret_cast<const uint32_t*>(gaps + 2 * qa)[t];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                w[j] = ((q4 >> (8 * j)) & 127u) | (((i4 >> (8 * j)) & 127u) << 7) | (((d4 >> (8 * j)) & 127u) << 14) |
                       (((g4 >> (8 * j)) & 127u) << 21) | (((c4 >> (4 * j)) & 15u) << 28);
        }
        reinterpret_cast<uint4*>(rows)[t] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// Nibbles equal to zero (values <= 7): bit 0 of each such nibble.
__device__ __forceinline__ uint32_t zero_nibbles(uint32_t t) { return ~(t | (t >> 1) | (t >> 2)) & 0x11111111u; }

// Match table of one hap from its code nibbles: a lane takes 8 columns (one
// 32-bit load), forms for each read code the 8 match bits (MSB first), and
// each quad of lanes joins its four bytes into one table word (DPP
// quad_perm): 512 columns per wave step.
__device__ __forceinline__ void hap_table_rec(const uint8_t* __restrict__ hc, int H, uint32_t* __restrict__ o, int lane)
{
    const int nw = (H + 31) / 32;
    if (lane < 5 * kHapLead) o[lane] = 0u;
    if (lane < 5) o[(kHapLead + nw) * 5 + lane] = 0u;
    const uint32_t* __restrict__ h32 = reinterpret_cast<const uint32_t*>(hc);
    for (int base = 0; base < H; base += 512) {
        const int col0 = base + 8 * lane;
        const int nv = H - col0;   // valid columns of this lane (<= 0: none)
        const uint32_t x = nv > 0 ? h32[base / 8 + lane] : 0u;
        const uint32_t vmask = nv >= 8 ? 0x11111111u : (nv > 0 ? 0x11111111u & ((1u << (4 * nv)) - 1u) : 0u);
        const uint32_t isN = zero_nibbles(x ^ 0x44444444u);
        uint32_t word[5];
#pragma unroll
        for (int rc = 0; rc < 5; ++rc) {
            // read code rc matches: equal code, hap 'N' (matches every rc), or read 'N'
            const uint32_t eq = (rc == 4 ? 0x11111111u : (zero_nibbles(x ^ (uint32_t(rc) * 0x11111111u)) | isN)) & vmask;
            uint32_t m = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) m |= ((eq >> (4 * j)) & 1u) << (7 - j);
            const uint32_t m1 = __builtin_amdgcn_mov_dpp(int(m), 0x55, 0xf, 0xf, false);   // quad_perm [1,1,1,1]
            const uint32_t m2 = __builtin_amdgcn_mov_dpp(int(m), 0xaa, 0xf, 0xf, false);   // quad_perm [2,2,2,2]
            const uint32_t m3 = __builtin_amdgcn_mov_dpp(int(m), 0xff, 0xf, 0xf, false);   // quad_perm [3,3,3,3]
            word[rc] = (m << 24) | (m1 << 16) | (m2 << 8) | m3;
        }
        const int w = base / 32 + (lane >> 2);
        if ((lane & 3) == 0 && w < nw) {
#pragma unroll
            for (int rc = 0; rc < 5; ++rc) o[(kHapLead + w) * 5 + rc] = word[rc];
        }
    }
}

// One wave per pair (grid-stride): its rows, its hap table, its pair
// descriptor, and its plan key — the cheaper of its two (block width, lanes)
// candidates by the host planner's cost model, and the counting-sort bin of
// (candidate group, R descending).
__global__ __launch_bounds__(256) void flat_prep_kernel(FlatPlanArgs a)
{
    if (blockIdx.x == 0 && threadIdx.x < kNumCounters) a.counters[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63;
    for (int p = blockIdx.x * 4 + (threadIdx.x >> 6); p < a.n; p += gridDim.x * 4) {
        const FlatDesc d = a.desc[p];
        const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(d.rec & 0xffffffffll));
        const unsigned hi = __builtin_amdgcn_readfirstlane(unsigned(d.rec >> 32));
        const uint8_t* quals = a.img + (long long)(((unsigned long long)hi << 32) | lo);
        const int R = __builtin_amdgcn_readfirstlane(d.R), H = __builtin_amdgcn_readfirstlane(d.H);
        const int ro = __builtin_amdgcn_readfirstlane(d.row_off), ho = __builtin_amdgcn_readfirstlane(d.hapw_off);
        const int gw = __builtin_amdgcn_readfirstlane(d.gapw);
        const uint8_t* codes = quals + align4(R);
        const uint8_t* gaps = codes + align4((R + 1) / 2);
        pack_read_rec(quals, codes, gaps, R, gw, a.rows + ro, lane);
        hap_table_rec(gaps + (gw < 0 ? 3 * align4(R) : 0), H, a.hapw + ho, lane);
        if (lane == 0) {
            a.pairs[p] = make_int4(ro, R, ho, H);
            const int2 c = a.ctab[H];
            // modelled wave instructions of each candidate (plan_model.hpp seg_cost)
            const int bc0 = c.x & 0xff, nb0 = (c.x >> 8) & 0xff, bc1 = c.y & 0xff, nb1 = (c.y >> 8) & 0xff;
            const float k0 = float((long long)nb0 * (13 * bc0 + 26) * (R + nb0 - 1)) * a.waste[nb0];
            const float k1 = float((long long)nb1 * (13 * bc1 + 26) * (R + nb1 - 1)) * a.waste[nb1];
            const int g = k1 < k0 ? (c.y >> 16) : (c.x >> 16);
            const int bin = g * a.rspan + ((a.rmax - R) >> a.rshift);
            a.bin_of[p] = bin;
            atomicAdd(&a.hist[bin], 1);
        }
    }
}

// One workgroup: exclusive scan of the bins (bin starts = slot cursors), then
// per group its first slot, its pair count and its first wave (waves of
// floor(64 / nb) pairs), and the plan's wave count.
__global__ __launch_bounds__(1024) void flat_scan_kernel(FlatPlanArgs a)
{
    __shared__ int part[1024];
    const int t = threadIdx.x;
    const int nbins = a.nbins;
    const int C = (nbins + 1023) / 1024;
    const int b0 = min(nbins, t * C), b1 = min(nbins, b0 + C);
    int s = 0;
    for (int i = b0; i < b1; ++i) s += a.hist[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const int total = part[1023];
    int run = part[t] - s;
    for (int i = b0; i < b1; ++i) {
        const int c = a.hist[i];
        a.hist[i] = run;
        run += c;
    }
    __syncthreads();
    // groups (at most 1024: the host planner takes batches with more)
    int wc = 0, first = 0, cnt = 0;
    if (t < a.ngroups) {
        first = a.hist[t * a.rspan];
        const int end = t + 1 < a.ngroups ? a.hist[(t + 1) * a.rspan] : total;
        cnt = end - first;
        const int per = 64 / a.groups[t].y;
        wc = (cnt + per - 1) / per;
    }
    __syncthreads();
    part[t] = wc;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    if (t < a.ngroups) {
        a.gtab[3 * t] = first;
        a.gtab[3 * t + 1] = cnt;
        a.gtab[3 * t + 2] = part[t] - wc;
    }
    if (t == 0) *a.nwaves = part[1023];
}

// Thread per pair: its slot (order inside a bin is arbitrary: a pair's result
// does not depend on where it runs).
__global__ __launch_bounds__(256) void flat_scatter_kernel(FlatPlanArgs a)
{
    for (int p = blockIdx.x * 256 + threadIdx.x; p < a.n; p += gridDim.x * 256) {
        const int pos = atomicAdd(&a.hist[a.bin_of[p]], 1);
        a.order[pos] = p;
    }
}

// Thread per wave: its group by binary search over the groups' first waves,
// its slots, and its row bounds from its pairs.
__global__ __launch_bounds__(256) void flat_waves_kernel(FlatPlanArgs a)
{
    const int nw = *a.nwaves;
    for (int w = blockIdx.x * 256 + threadIdx.x; w < nw; w += gridDim.x * 256) {
        int lo = 0, hi = a.ngroups;   // the last group whose first wave is <= w
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (a.gtab[3 * mid + 2] <= w) lo = mid;
            else hi = mid;
        }
        const int2 g = a.groups[lo];
        const int per = 64 / g.y;
        const int s0 = a.gtab[3 * lo] + (w - a.gtab[3 * lo + 2]) * per;
        const int s1 = min(a.gtab[3 * lo] + a.gtab[3 * lo + 1], s0 + per);
        int rmax = 0, rmin = 0x7fffffff;
        for (int s = s0; s < s1; ++s) {
            const int R = a.pairs[a.order[s]].y;
            rmax = max(rmax, R);
            rmin = min(rmin, R);
        }
        LaneWave v;
        v.slot0 = s0;
        v.rmax = rmax;
        v.rmin = rmin;
        v.ncols = g.x;
        v.npairs = s1 - s0;
        v.nsteps = rmax + g.y - 1;
        v.carry_row = 0;
        a.waves[w] = v;
    }
}

int grid_for(long long waves)
{
    const long long blocks = (waves + 3) / 4;
    return int(blocks < 65536 ? (blocks > 0 ? blocks : 1) : 65536);
}

}  // namespace

hipError_t launch_pack_reads(const uint8_t* bases, const uint8_t* quals, const uint8_t* gaps, long long gap_stride,
                             const int4* rdesc, int nreads, uint32_t* rows, hipStream_t s)
{
    if (nreads <= 0) return hipSuccess;
    hipLaunchKernelGGL(pack_reads_kernel, dim3(grid_for(nreads)), dim3(256), 0, s, bases, quals, gaps, gap_stride,
                       rdesc, nreads, rows);
    return hipGetLastError();
}

hipError_t launch_hap_tables(const uint8_t* hap_bytes, const int4* haps, int nhaps, uint32_t* hapw, hipStream_t s)
{
    if (nhaps <= 0) return hipSuccess;
    hipLaunchKernelGGL(hap_tables_kernel, dim3(grid_for(nhaps)), dim3(256), 0, s, hap_bytes, haps, nhaps, hapw);
    return hipGetLastError();
}

hipError_t launch_grid_pairs(const GridBlock* blocks, int nblocks, long long npairs, const int4* rdesc,
                             const int4* hdesc, PairDesc* pairs, hipStream_t s)
{
    if (npairs <= 0 || nblocks <= 0) return hipSuccess;
    const long long g = (npairs + 255) / 256;
    hipLaunchKernelGGL(grid_pairs_kernel, dim3(unsigned(g < 8192 ? g : 8192)), dim3(256), 0, s, blocks, nblocks, npairs,
                       rdesc, hdesc, pairs);
    return hipGetLastError();
}

hipError_t launch_grid_waves(const GridSeg* segs, int nsegs, long long nslots, int nwaves, const int* rord,
                             const int* hord, const int4* rdesc, int* order, LaneWave* waves, hipStream_t s)
{
    if (nsegs <= 0 || (nslots <= 0 && nwaves <= 0)) return hipSuccess;
    const long long g = (nslots + 255) / 256;
    hipLaunchKernelGGL(grid_waves_kernel, dim3(unsigned(g < 4096 ? (g > 0 ? g : 1) : 4096)), dim3(256), 0, s, segs,
                       nsegs, nslots, nwaves, rord, hord, rdesc, order, waves);
    return hipGetLastError();
}

hipError_t launch_prepare_grid(const GridPrepArgs& a, hipStream_t s)
{
    const long long items = std::max<long long>({(long long)a.nreads, (long long)a.nhaps, a.npairs / 64, a.nslots / 64, 1});
    const int grid = grid_for(items);
    hipLaunchKernelGGL(prepare_grid_kernel, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_flat_plan(const FlatPlanArgs& a, hipStream_t s)
{
    if (a.n <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(a.hist, 0, sizeof(int) * size_t(a.nbins), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(flat_prep_kernel, dim3(grid_for(a.n)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(flat_scan_kernel, dim3(1), dim3(1024), 0, s, a);
    const int gs = std::min(8192, (a.n + 255) / 256);
    hipLaunchKernelGGL(flat_scatter_kernel, dim3(gs), dim3(256), 0, s, a);
    const int gw = std::max(1, std::min(8192, (a.max_waves + 255) / 256));
    hipLaunchKernelGGL(flat_waves_kernel, dim3(gw), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcphmm
