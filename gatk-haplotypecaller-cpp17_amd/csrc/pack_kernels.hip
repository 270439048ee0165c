// Device-side packing and planning of a batch (the reference's getData /
// precompute_masks work, intel_pairhmm.hpp:154-203 and
// avx-pairhmm-template.h:3-35, done once per read and once per haplotype
// instead of once per pair).
//
//   pack_batch   staged read bytes -> one uint32 row word per base
//                (kernels.hpp pack_row), four rows per lane; hap bytes ->
//                per-hap match table, (ceil(H/32) + 3) rows of 5 words: bit
//                (MSB first) per column for read codes 0..4, eight columns per
//                lane. The upload carries 2 bytes per base (base, quality); a
//                read whose gap qualities are constant — every read the
//                reference builds, sam.hpp:30-32,47-49 — sends them once in its
//                descriptor, the others send 3 more planes.
//   grid_*       descriptors, slot order and waves of a structured
//                (cross-product) plan from its block and segment tables.
//   flat_*       a flat batch planned on the device: rows, tables, each pair's
//                segmented shape, a counting sort and the waves (flat_plan.cpp).
//
// The packers are byte-streaming kernels, a wave per read / haplotype / pair,
// loading 4 or 8 bytes per lane and keeping several requests in flight per
// wave (the packing is latency-bound, not bandwidth-bound, at one chain each).
#include <algorithm>

#include "kernels.hpp"

namespace hcphmm {
namespace {

// Nibbles equal to zero (values <= 7): bit 0 of each such nibble.
__device__ __forceinline__ uint32_t zero_nibbles(uint32_t t) { return ~(t | (t >> 1) | (t >> 2)) & 0x11111111u; }

// Match-table words of 32 columns from a quad of lanes, each holding the
// codes of 8 columns as nibbles (column 8 * lane + j in nibble j) of which the
// first nv are real: per read code, the lane's 8 match bits (MSB first), the
// quad's four bytes joined by DPP quad_perm. Lane 4q + 0 stores the word of
// columns 32 * (w) + 1 .. 32 * (w + 1), w = base / 32 + q; all 64 lanes take part.
__device__ __forceinline__ void hap_words(uint32_t x, int nv, int base, int nw, uint32_t* __restrict__ o, int lane)
{
    // Nibble order reversed first (column 8 * lane + 7 - k in nibble k), so
    // the match bits come out MSB first by a three-step compress of the
    // nibbles' bit 0 (6 ops per read code instead of an 8-step gather of 24;
    // equal for every input, checked exhaustively over random words and nv).
    const uint32_t y = __builtin_bswap32(x);
    const uint32_t xr = ((y >> 4) & 0x0f0f0f0fu) | ((y & 0x0f0f0f0fu) << 4);
    const uint32_t vmask = nv >= 8 ? 0x11111111u : (nv > 0 ? 0x11111111u & ~((1u << (4 * (8 - nv))) - 1u) : 0u);
    const uint32_t isN = zero_nibbles(xr ^ 0x44444444u);
    uint32_t word[5];
#pragma unroll
    for (int rc = 0; rc < 5; ++rc) {
        // read code rc matches: equal code, hap 'N' (matches every rc), or read 'N'
        uint32_t m = (rc == 4 ? 0x11111111u : (zero_nibbles(xr ^ (uint32_t(rc) * 0x11111111u)) | isN)) & vmask;
        m = (m | (m >> 3)) & 0x03030303u;
        m = (m | (m >> 6)) & 0x000f000fu;
        m = (m | (m >> 12)) & 0xffu;
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

// Zero rows of a table: kHapLead before the data, one after.
__device__ __forceinline__ void hap_zero_rows(int nw, uint32_t* __restrict__ o, int lane)
{
    if (lane < 5 * kHapLead) o[lane] = 0u;
    if (lane < 5) o[(kHapLead + nw) * 5 + lane] = 0u;
}

// Four row words from a record: qualities q4 (byte j = row 4t + j), codes c4
// (nibble j), and the i / d / c planes' bytes when the gaps vary (gw < 0).
__device__ __forceinline__ uint4 rows_rec4(uint32_t q4, uint32_t c4, uint32_t i4, uint32_t d4, uint32_t g4, int gw,
                                           bool first)
{
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t q = (q4 >> (8 * j)) & 127u, code = ((c4 >> (4 * j)) & 15u) << 28;
        w[j] = gw >= 0 ? q | (uint32_t(gw) << 7) | code
                       : q | (((i4 >> (8 * j)) & 127u) << 7) | (((d4 >> (8 * j)) & 127u) << 14) |
                             (((g4 >> (8 * j)) & 127u) << 21) | code;
    }
    if (first && gw >= 0) w[0] |= 0x80000000u;   // constant-gap tag on the read's first row
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// A staged part's reads and haps, wave per item (grid-stride): item i packs
// read i's rows (4 per lane) and hap i's table (8 columns per lane) from the
// staged qualities, gap planes and code nibbles. Both
// descriptors, then the first chunk of both, are loaded before either is
// used, and the next item's descriptors while this one is packed: a wave keeps
// several HBM requests in flight instead of one dependent chain per read.
__device__ __forceinline__ void pack_items(const PackArgs& a)
{
    const int lane = threadIdx.x & 63;
    const int n = max(a.nreads, a.nhaps);
    const int stride = gridDim.x * 4;
    int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int4 z4 = make_int4(0, 0, 0, 0);
    int4 rdn = i < a.nreads ? a.rdesc[i] : z4;
    int4 hdn = i < a.nhaps ? a.hdesc[i] : z4;
    for (; i < n; i += stride) {
        const int off = __builtin_amdgcn_readfirstlane(rdn.x), len = __builtin_amdgcn_readfirstlane(rdn.y);
        const int gw = __builtin_amdgcn_readfirstlane(rdn.z), goff = __builtin_amdgcn_readfirstlane(rdn.w);
        const int hoff = __builtin_amdgcn_readfirstlane(hdn.x), H = __builtin_amdgcn_readfirstlane(hdn.y);
        const int tw = __builtin_amdgcn_readfirstlane(hdn.z);
        const int in = i + stride;
        rdn = in < a.nreads ? a.rdesc[in] : z4;
        hdn = in < a.nhaps ? a.hdesc[in] : z4;
        const uint16_t* __restrict__ b16 = reinterpret_cast<const uint16_t*>(a.bases + off / 2);
        const uint32_t* __restrict__ q32 = reinterpret_cast<const uint32_t*>(a.quals + off);
        const uint32_t* __restrict__ g32 = reinterpret_cast<const uint32_t*>(a.gaps + goff);
        const uint32_t* __restrict__ h32 = reinterpret_cast<const uint32_t*>(a.hap_bytes + hoff);
        const int gs4 = int(a.gap_stride >> 2);
        uint32_t b4 = 0, q4 = 0, i4 = 0, d4 = 0, c4 = 0, hx = 0;
        if (4 * lane < len) {
            b4 = b16[lane];
            q4 = q32[lane];
            if (gw < 0) {
                i4 = g32[lane];
                d4 = g32[gs4 + lane];
                c4 = g32[2 * gs4 + lane];
            }
        }
        if (8 * lane < H) hx = h32[lane];
        // rows (len == 0: no read for this item)
        uint4* __restrict__ rows = reinterpret_cast<uint4*>(a.rows + off);
        for (int t0 = 0; 4 * t0 < len; t0 += 64) {
            const int t = t0 + lane;
            if (t0 > 0) {
                if (4 * t < len) {
                    b4 = b16[t];
                    q4 = q32[t];
                    if (gw < 0) {
                        i4 = g32[t];
                        d4 = g32[gs4 + t];
                        c4 = g32[2 * gs4 + t];
                    }
                }
            }
            if (4 * t < len) rows[t] = rows_rec4(q4, b4, i4, d4, c4, gw, t == 0);
        }
        // table (H == 0: no hap for this item)
        if (H > 0) {
            uint32_t* __restrict__ o = a.hapw + tw;
            const int nw = (H + 31) / 32;
            hap_zero_rows(nw, o, lane);
            for (int base = 0; base < H; base += 512) {
                if (base > 0) hx = 8 * lane + base < H ? h32[base / 8 + lane] : 0u;
                hap_words(hx, H - base - 8 * lane, base, nw, o, lane);
            }
        }
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
                                           const int4* __restrict__ rdesc, const int4* __restrict__ hdesc,
                                           int* __restrict__ order, int* __restrict__ slot_of,
                                           int4* __restrict__ sdesc, LaneWave* __restrict__ waves)
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
        const int r = rord[g.r0 + rr], h = hord[g.g0 + hh];
        const int p = int(g.p0 + (long long)(r - g.r0) * g.nh + (h - g.h0));
        order[t] = p;
        slot_of[p] = int(t);
        const int4 rd = rdesc[r], hd = hdesc[h];   // as grid_pairs
        sdesc[t] = make_int4(rd.x, rd.y, hd.z, hd.y);
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

// Everything a structured (region) part needs before its pass, in one launch
// (each step is a grid-stride loop over its own items; none reads another's
// output): the run counters zeroed, reads packed, hap tables, pair
// descriptors, slot order and waves — four fewer launches per region call.
__global__ __launch_bounds__(256) void pack_batch_kernel(PackArgs a)
{
    pack_items(a);
    for (int s = blockIdx.x * 256 + threadIdx.x; s < a.nslots; s += gridDim.x * 256) a.sdesc[s] = a.pairs[a.order[s]];
}

__global__ __launch_bounds__(256) void prepare_grid_kernel(GridPrepArgs a)
{
    if (blockIdx.x == 0 && threadIdx.x < kNumCounters) a.counters[threadIdx.x] = 0;
    pack_items(a.pack);
    grid_pairs(a.blocks, a.nblocks, a.npairs, a.pack.rdesc, a.pack.hdesc, a.pairs);
    grid_waves(a.segs, a.nsegs, a.nslots, a.nwaves, a.rord, a.hord, a.pack.rdesc, a.pack.hdesc, a.order, a.slot_of,
               a.sdesc, a.waves);
}

// ---------------------------------------------------------------------------
// Flat batches planned on the device (kernels.hpp FlatPlanArgs).

// Flat records (flat_plan.cpp, kernels.hpp FlatDesc): the read — one byte per
// base, (q - qbase) << 2 | code (kFmtRead1B), or its base qualities then its
// base codes as nibbles (ConvertChar, two per byte, row k in the low nibble of
// byte k/2 when k is even) —, its i / d / c planes when they vary, then the
// hap's base codes, 2 bits (kFmtHap2b) or a nibble each; every field 4-byte
// aligned.
__host__ __device__ constexpr int align4(int x) { return (x + 3) & ~3; }

// kFmtRead1B: four rows' bytes -> their qualities (bytes) and code nibbles.
__device__ __forceinline__ void read_1b_unpack(uint32_t b4, uint32_t qbase4, uint32_t& q4, uint32_t& c4)
{
    q4 = ((b4 >> 2) & 0x3f3f3f3fu) + qbase4;   // (q & 127) <= 127: no carry between bytes
    uint32_t c = b4 & 0x03030303u;             // code j in byte j
    c = (c | (c >> 4)) & 0x00ff00ffu;          // codes 0,1 in the low byte, 2,3 in byte 2
    c4 = (c | (c >> 8)) & 0xffffu;             // code j in nibble j
}

// kFmtHap2b: the 2-bit codes of 8 columns -> nibbles (column j in nibble j).
__device__ __forceinline__ uint32_t hap_2b_nibbles(uint32_t h16)
{
    uint32_t x = h16 & 0xffffu;
    x = (x | (x << 8)) & 0x00ff00ffu;
    x = (x | (x << 4)) & 0x0f0f0f0fu;
    x = (x | (x << 2)) & 0x33333333u;
    return x;
}

// A flat pair's descriptor fields (wave-uniform) and the first chunk of its
// record as this lane loaded it (raw words: converted only when packed, so a
// prefetch never waits on its own loads).
struct PrepIn {
    const uint8_t* quals;
    int R, H, ro, ho, gw, fmt;
    uint32_t q4, c4, i4, d4, g4, hraw;
    int2 c;
};

__device__ __forceinline__ void prep_load(const FlatPlanArgs& a, const FlatDesc& dn, int lane, PrepIn& x)
{
    const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(dn.rec & 0xffffffffll));
    const unsigned hi = __builtin_amdgcn_readfirstlane(unsigned(dn.rec >> 32));
    x.quals = a.img + (long long)(((unsigned long long)hi << 32) | lo);
    x.R = __builtin_amdgcn_readfirstlane(dn.R);
    x.H = __builtin_amdgcn_readfirstlane(dn.H);
    x.ro = __builtin_amdgcn_readfirstlane(dn.row_off);
    x.ho = __builtin_amdgcn_readfirstlane(dn.hapw_off);
    x.gw = __builtin_amdgcn_readfirstlane(dn.gapw);
    x.fmt = __builtin_amdgcn_readfirstlane(dn.fmt);
    const bool r1b = (x.fmt & kFmtRead1B) != 0, h2b = (x.fmt & kFmtHap2b) != 0;
    const int qa = align4(x.R), qa4 = qa >> 2;
    const uint32_t* __restrict__ q32 = reinterpret_cast<const uint32_t*>(x.quals);
    const uint16_t* __restrict__ c16 = reinterpret_cast<const uint16_t*>(x.quals + qa);
    const uint32_t* __restrict__ g32 = reinterpret_cast<const uint32_t*>(x.quals + qa + (r1b ? 0 : align4((x.R + 1) / 2)));
    const uint32_t* __restrict__ h32 = g32 + (x.gw < 0 ? 3 * qa4 : 0);
    const uint16_t* __restrict__ h16 = reinterpret_cast<const uint16_t*>(h32);
    x.q4 = x.c4 = x.i4 = x.d4 = x.g4 = x.hraw = 0;
    if (4 * lane < x.R) {
        x.q4 = q32[lane];
        if (!r1b) x.c4 = c16[lane];
        if (x.gw < 0) {
            x.i4 = g32[lane];
            x.d4 = g32[qa4 + lane];
            x.g4 = g32[2 * qa4 + lane];
        }
    }
    if (8 * lane < x.H) x.hraw = h2b ? uint32_t(h16[lane]) : h32[lane];
    x.c = a.ctab[x.H];
}

// Pair p's rows, hap table, descriptor and plan key from its prefetched first
// chunk (longer reads and haps load their further chunks here).
__device__ __forceinline__ void prep_pack(const FlatPlanArgs& a, const PrepIn& x, int p, int lane)
{
    const int R = x.R, H = x.H, gw = x.gw, fmt = x.fmt;
    const bool r1b = (fmt & kFmtRead1B) != 0, h2b = (fmt & kFmtHap2b) != 0;
    const uint32_t qbase4 = uint32_t((fmt >> 8) & 127) * 0x01010101u;
    const int qa = align4(R), qa4 = qa >> 2;
    const uint32_t* __restrict__ q32 = reinterpret_cast<const uint32_t*>(x.quals);
    const uint16_t* __restrict__ c16 = reinterpret_cast<const uint16_t*>(x.quals + qa);
    const uint32_t* __restrict__ g32 = reinterpret_cast<const uint32_t*>(x.quals + qa + (r1b ? 0 : align4((R + 1) / 2)));
    const uint32_t* __restrict__ h32 = g32 + (gw < 0 ? 3 * qa4 : 0);
    const uint16_t* __restrict__ h16 = reinterpret_cast<const uint16_t*>(h32);
    uint32_t q4 = x.q4, c4 = x.c4, i4 = x.i4, d4 = x.d4, g4 = x.g4;
    uint4* __restrict__ rows = reinterpret_cast<uint4*>(a.rows + x.ro);
    for (int t0 = 0; 4 * t0 < R; t0 += 64) {
        const int t = t0 + lane;
        if (t0 > 0 && 4 * t < R) {
            q4 = q32[t];
            if (!r1b) c4 = c16[t];
            if (gw < 0) {
                i4 = g32[t];
                d4 = g32[qa4 + t];
                g4 = g32[2 * qa4 + t];
            }
        }
        if (4 * t < R) {
            uint32_t qq = q4, cc = c4;
            if (r1b) read_1b_unpack(q4, qbase4, qq, cc);
            rows[t] = rows_rec4(qq, cc, i4, d4, g4, gw, t == 0);
        }
    }
    uint32_t* __restrict__ o = a.hapw + x.ho;
    const int nw = (H + 31) / 32;
    hap_zero_rows(nw, o, lane);
    uint32_t hx = h2b ? hap_2b_nibbles(x.hraw) : x.hraw;
    for (int base = 0; base < H; base += 512) {
        const int nv = H - base - 8 * lane;   // valid columns of this lane (<= 0: none)
        if (base > 0) hx = nv > 0 ? (h2b ? hap_2b_nibbles(h16[base / 8 + lane]) : h32[base / 8 + lane]) : 0u;
        hap_words(hx, nv, base, nw, o, lane);
    }
    if (lane == 0) {
        const int2 c = x.c;
        a.pairs[p] = make_int4(x.ro, R, x.ho, H);
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

// Pairs in grid-stride order, software-pipelined two deep: while pair p is
// packed, pair p + stride's record chunk and table entry and pair p + 2 *
// stride's descriptor are in flight (one wave per pair left each wave's two
// dependent load rounds exposed: 185 us per 250k-pair part; the launcher now
// bounds the grid so each wave pipelines several pairs).
__global__ __launch_bounds__(256) void flat_prep_kernel(FlatPlanArgs a)
{
    if (blockIdx.x == 0 && threadIdx.x < kNumCounters) a.counters[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63;
    const int stride = gridDim.x * 4;
    int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= a.n) return;   // wave-uniform
    PrepIn cur, nxt;
    prep_load(a, a.desc[p], lane, cur);
    FlatDesc dn{};
    if (p + stride < a.n) dn = a.desc[p + stride];
    for (; p < a.n; p += stride) {
        const bool more = p + stride < a.n;
        if (more) prep_load(a, dn, lane, nxt);
        if (p + 2 * stride < a.n) dn = a.desc[p + 2 * stride];
        prep_pack(a, cur, p, lane);
        if (more) cur = nxt;
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
#pragma unroll 8
    for (int i = b0; i < b1; ++i) s += a.hist[i];   // (independent loads: eight in flight)
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
#pragma unroll 8
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
    if (t == 0) {
        a.nwaves[0] = part[1023];
        a.nwaves[1] = 1;   // the largest wave cost, raised by flat_waves_kernel
    }
}

// Thread per pair: its slot (order inside a bin is arbitrary: a pair's result
// does not depend on where it runs).
__global__ __launch_bounds__(256) void flat_scatter_kernel(FlatPlanArgs a)
{
    for (int p = blockIdx.x * 256 + threadIdx.x; p < a.n; p += gridDim.x * 256) {
        const int pos = atomicAdd(&a.hist[a.bin_of[p]], 1);
        a.order[pos] = p;
        a.slot_of[p] = pos;
        a.sdesc[pos] = a.pairs[p];
    }
}

// Modelled wave duration (plan_model.hpp).
__device__ __forceinline__ int wave_cost(const LaneWave& v) { return (13 * v.ncols + 26) * v.nsteps; }   // plan_model.hpp

// Thread per wave: its group by binary search over the groups' first waves,
// its slots, and its row bounds from its pairs.
__global__ __launch_bounds__(256) void flat_waves_kernel(FlatPlanArgs a)
{
    const int nw = *a.nwaves;
    int cmax = 1;
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
        (a.tail > 0 ? a.waves_tmp : a.waves)[w] = v;
        if (a.tail > 0) {
            const int c = wave_cost(v);
            a.wcost[w] = c;
            cmax = max(cmax, c);
        }
    }
    if (a.tail > 0) {   // the largest cost for flat_tail_kernel's buckets: wave max, one atomic per wave
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) cmax = max(cmax, __shfl_xor(cmax, d, 64));
        if ((threadIdx.x & 63) == 0 && cmax > 1) atomicMax(a.nwaves + 1, cmax);
    }
}

// Dispatch order (one workgroup), as the host planner's (planner.cpp): the
// bulk in packing order (co-resident waves share one width's code), the
// `tail` shortest waves (modelled duration BC x steps, in 1024 buckets) last,
// longest first, so the chip drains evenly; order inside a bucket arbitrary.

// One workgroup. The waves' costs and their maximum come from
// flat_waves_kernel (a 4-byte cost per wave, not the 32-byte wave); every
// pass reads coalesced (thread t takes waves t, t + 1024, ...; two loads in
// flight per thread: four spilled at this workgroup size) and the bucket prefix is a block scan: the first form walked a contiguous run of ~50 waves per
// thread (one dependent load per step) and found the tail threshold and the
// bucket cursors with two serial loops over the 1 024 buckets on one thread,
// 161 us of every 250k-pair part's preparation (profiles/r05_e2e_call_timeline.txt).
// The bulk keeps packing order through a stable compaction per tile of 1 024
// waves (wave ballots, then the block's wave counts).
__device__ __forceinline__ int block_incl_scan(int v, int* part)
{
    const int t = threadIdx.x;
    part[t] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int u = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += u;
        __syncthreads();
    }
    return part[t];
}

__global__ __launch_bounds__(1024) void flat_tail_kernel(FlatPlanArgs a)
{
    constexpr int NB = 1024, K = 2;
    __shared__ int hist[NB], cur[NB], part[1024];
    __shared__ int thr_s, acc_s, wcnt[16];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int nw = *a.nwaves;
    const LaneWave* __restrict__ in = a.waves_tmp;
    hist[t] = 0;
    __syncthreads();
    const long long cm = max(1, a.nwaves[1]);   // flat_waves_kernel's largest cost
    auto bucket_c = [&](int c) { return int((long long)c * (NB - 1) / cm); };
    for (int w0 = t; w0 < nw; w0 += K * 1024) {
        int b[K];
#pragma unroll
        for (int k = 0; k < K; ++k) b[k] = w0 + k * 1024 < nw ? bucket_c(a.wcost[w0 + k * 1024]) : -1;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (b[k] >= 0) atomicAdd(&hist[b[k]], 1);
    }
    __syncthreads();
    // incl[b] = waves in buckets 0..b. The tail threshold: the fewest lowest
    // buckets holding at least `tail` waves.
    const int hb = hist[t];
    const int incl = block_incl_scan(hb, part);
    if (t == 0) {
        thr_s = a.tail > 0 ? NB : 0;   // (NB: fewer than `tail` waves in all)
        acc_s = a.tail > 0 ? part[NB - 1] : 0;
    }
    __syncthreads();
    if (a.tail > 0 && incl >= a.tail && incl - hb < a.tail) {   // the one bucket where the prefix reaches tail
        thr_s = t + 1;
        acc_s = incl;
    }
    __syncthreads();
    const int thr = acc_s >= nw ? 0 : thr_s;   // nothing to gain when every wave is in the tail
    // tail buckets longest first: bucket b's first position is the count in buckets (b, thr)
    if (t < thr) cur[t] = part[thr - 1] - incl;
    const int nbulk = nw - (thr > 0 ? part[thr - 1] : 0);
    __syncthreads();
    int base = 0;
    for (int w0 = 0; w0 < nw; w0 += K * 1024) {
        LaneWave v[K];
        int c[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (w0 + k * 1024 + t < nw) {
                v[k] = in[w0 + k * 1024 + t];
                c[k] = a.wcost[w0 + k * 1024 + t];
            }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int w = w0 + k * 1024 + t;
            const int bk = w < nw ? bucket_c(c[k]) : -1;
            const bool bulk = bk >= thr;
            const uint64_t bal = __builtin_amdgcn_ballot_w64(bulk);
            if (lane == 0) wcnt[wv] = __popcll(bal);
            __syncthreads();
            int off = 0, tot = 0;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int c = wcnt[q];
                off += q < wv ? c : 0;
                tot += c;
            }
            __syncthreads();   // wcnt is rewritten by the next tile
            if (bulk)
                a.waves[base + off + __popcll(bal & ((1ull << lane) - 1))] = v[k];
            else if (bk >= 0)
                a.waves[nbulk + atomicAdd(&cur[bk], 1)] = v[k];
            base += tot;
        }
    }
}

__global__ __launch_bounds__(256) void store_to_host_kernel(uint4* __restrict__ host, const uint4* __restrict__ dev,
                                                            long long n16)
{
    for (long long k = blockIdx.x * 256ll + threadIdx.x; k < n16; k += 256ll * gridDim.x) host[k] = dev[k];
}

int grid_for(long long waves)
{
    const long long blocks = (waves + 3) / 4;
    return int(blocks < 65536 ? (blocks > 0 ? blocks : 1) : 65536);
}

}  // namespace

hipError_t launch_pack_batch(const PackArgs& a, hipStream_t s)
{
    const int items = std::max(a.nreads, a.nhaps);
    if (items <= 0) return hipSuccess;
    hipLaunchKernelGGL(pack_batch_kernel, dim3(grid_for(items)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_prepare_grid(const GridPrepArgs& a, hipStream_t s)
{
    const long long items =
        std::max<long long>({(long long)a.pack.nreads, (long long)a.pack.nhaps, a.npairs / 64, a.nslots / 64, 1});
    const int grid = grid_for(items);
    hipLaunchKernelGGL(prepare_grid_kernel, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_store_to_host(void* host, const void* dev, size_t bytes, hipStream_t s)
{
    const long long n16 = (long long)(bytes / 16);
    if (n16 <= 0) return hipSuccess;
    const long long g = std::min<long long>(1024, (n16 + 255) / 256);
    hipLaunchKernelGGL(store_to_host_kernel, dim3(unsigned(g)), dim3(256), 0, s, static_cast<uint4*>(host),
                       static_cast<const uint4*>(dev), n16);
    return hipGetLastError();
}

hipError_t launch_flat_plan(const FlatPlanArgs& a, hipStream_t s)
{
    if (a.n <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(a.hist, 0, sizeof(int) * size_t(a.nbins), s);
    if (e != hipSuccess) return e;
    // Bounded grid (HC_PHMM_PREP_BLOCKS; default 2 560 blocks, two rounds of
    // the kernel's 5 waves per SIMD at 92 VGPRs): each wave pipelines several
    // pairs. Per part beside the passes (tools/prep_prof.sh): 144 us vs 186
    // one wave per pair, 204 at 1 280 blocks, 250 at 640.
    const int pg = std::min(grid_for(a.n), a.prep_blocks > 0 ? a.prep_blocks : 2560);
    hipLaunchKernelGGL(flat_prep_kernel, dim3(pg), dim3(256), 0, s, a);
    hipLaunchKernelGGL(flat_scan_kernel, dim3(1), dim3(1024), 0, s, a);
    const int gs = std::min(8192, (a.n + 255) / 256);
    hipLaunchKernelGGL(flat_scatter_kernel, dim3(gs), dim3(256), 0, s, a);
    const int gw = std::max(1, std::min(8192, (a.max_waves + 255) / 256));
    hipLaunchKernelGGL(flat_waves_kernel, dim3(gw), dim3(256), 0, s, a);
    if (a.tail > 0) hipLaunchKernelGGL(flat_tail_kernel, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
}

}  // namespace hcphmm
