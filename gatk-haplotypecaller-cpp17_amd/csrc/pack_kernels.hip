// Device-side packing of a batch (the reference's getData / precompute_masks
// work, intel_pairhmm.hpp:154-203 and avx-pairhmm-template.h:3-35, done once
// per read and once per haplotype instead of once per pair).
//
//   pack_rows   raw SAM bytes (bases, q, i, d, c; one byte each per read base)
//               -> one uint32 row word per base (kernels.hpp pack_row)
//   hap_tables  raw hap bases -> per-hap match table, (ceil(H/32) + 3) rows of
//               5 words: bit (MSB first) per column for read codes 0..4
//
// Both are byte-streaming kernels (HBM/PCIe-staged data, read once, written
// once): 16-byte loads, one thread per 16 rows / one thread per table row.
#include "kernels.hpp"

namespace hcphmm {
namespace {

// ConvertChar (pairhmm_common.h:26-44): A0 C1 T2 G3 N4, every other byte -> 0.
__device__ __forceinline__ uint32_t base_code(uint32_t b)
{
    return b == 'C' ? 1u : b == 'T' ? 2u : b == 'G' ? 3u : b == 'N' ? 4u : 0u;
}

__global__ __launch_bounds__(256) void pack_rows_kernel(const uint8_t* __restrict__ raw, long long nrows,
                                                        long long stride, uint32_t* __restrict__ rows)
{
    // raw: 5 planes of `stride` bytes: bases, q, i, d, c (row k at offset k).
    const long long k0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 16;
    if (k0 >= nrows) return;
    if (k0 + 16 <= nrows) {
        uint4 pb = *reinterpret_cast<const uint4*>(raw + k0);
        uint4 pq = *reinterpret_cast<const uint4*>(raw + stride + k0);
        uint4 pi = *reinterpret_cast<const uint4*>(raw + 2 * stride + k0);
        uint4 pd = *reinterpret_cast<const uint4*>(raw + 3 * stride + k0);
        uint4 pc = *reinterpret_cast<const uint4*>(raw + 4 * stride + k0);
        const uint8_t* b = reinterpret_cast<const uint8_t*>(&pb);
        const uint8_t* q = reinterpret_cast<const uint8_t*>(&pq);
        const uint8_t* i = reinterpret_cast<const uint8_t*>(&pi);
        const uint8_t* d = reinterpret_cast<const uint8_t*>(&pd);
        const uint8_t* c = reinterpret_cast<const uint8_t*>(&pc);
        uint32_t w[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) w[u] = pack_row(q[u], i[u], d[u], c[u], base_code(b[u]));
        uint4* o = reinterpret_cast<uint4*>(rows + k0);
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = make_uint4(w[4 * u], w[4 * u + 1], w[4 * u + 2], w[4 * u + 3]);
    } else {
        for (long long k = k0; k < nrows; ++k)
            rows[k] = pack_row(raw[stride + k], raw[2 * stride + k], raw[3 * stride + k], raw[4 * stride + k],
                               base_code(raw[k]));
    }
}

// One thread per table row (kHapLead zero rows, data rows, one zero row) of
// every hap: a wave handles 64 consecutive table rows of one or more haps.
__global__ __launch_bounds__(256) void hap_tables_kernel(const uint8_t* __restrict__ hap_bytes,
                                                         const int4* __restrict__ haps, int nhaps,
                                                         const long long* __restrict__ tab_row0,
                                                         long long ntab_rows, uint32_t* __restrict__ hapw)
{
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= ntab_rows) return;
    // Which hap owns table row t: binary search over the first table row of each hap.
    int lo = 0, hi = nhaps - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab_row0[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const int4 hd = haps[lo];   // {byte offset, H, table word offset, 0}
    const int r = int(t - tab_row0[lo]);   // row inside the hap's table
    const int w = r - kHapLead;            // data word index, columns 32w+1 .. 32w+32
    uint32_t m[5] = {0u, 0u, 0u, 0u, 0u};
    const int H = hd.y;
    if (w >= 0 && 32 * w < H) {
        const uint8_t* src = hap_bytes + hd.x + 32 * w;
        const int n = min(32, H - 32 * w);
        for (int j = 0; j < n; ++j) {
            const uint32_t bit = 0x80000000u >> j;
            const uint32_t hc = base_code(src[j]);
            if (hc == 4) {
#pragma unroll
                for (int c = 0; c < 5; ++c) m[c] |= bit;
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c) m[c] |= (hc == uint32_t(c)) ? bit : 0u;
                m[4] |= bit;   // read 'N' matches every column
            }
        }
    }
    uint32_t* o = hapw + hd.z + r * 5;
#pragma unroll
    for (int c = 0; c < 5; ++c) o[c] = m[c];
}

// Constant-gap tag: bit 31 of a read's first row word is set when every row
// has the same (i, d, c) — the lane kernel's constant-gap path. One thread per read.
__global__ __launch_bounds__(256) void mark_cg_kernel(uint32_t* __restrict__ rows, const int2* __restrict__ reads,
                                                      int nreads)
{
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= nreads) return;
    const int2 rd = reads[r];   // {row offset, length}
    const uint32_t* w = rows + rd.x;
    const uint32_t g0 = w[0] & 0x0fffff80u;
    bool cg = true;
    int k = 1;
    for (; k + 4 <= rd.y; k += 4)
        cg &= ((w[k] & 0x0fffff80u) == g0) & ((w[k + 1] & 0x0fffff80u) == g0) &
              ((w[k + 2] & 0x0fffff80u) == g0) & ((w[k + 3] & 0x0fffff80u) == g0);
    for (; k < rd.y; ++k) cg &= (w[k] & 0x0fffff80u) == g0;
    if (cg) rows[rd.x] = w[0] | 0x80000000u;
}

}  // namespace

hipError_t launch_mark_cg(uint32_t* rows, const int2* reads, int nreads, hipStream_t s)
{
    if (nreads <= 0) return hipSuccess;
    hipLaunchKernelGGL(mark_cg_kernel, dim3(unsigned((nreads + 255) / 256)), dim3(256), 0, s, rows, reads, nreads);
    return hipGetLastError();
}

hipError_t launch_pack_rows(const uint8_t* raw, long long nrows, long long stride, uint32_t* rows,
                            hipStream_t s)
{
    if (nrows <= 0) return hipSuccess;
    const long long threads = (nrows + 15) / 16;
    hipLaunchKernelGGL(pack_rows_kernel, dim3(unsigned((threads + 255) / 256)), dim3(256), 0, s, raw, nrows,
                       stride, rows);
    return hipGetLastError();
}

hipError_t launch_hap_tables(const uint8_t* hap_bytes, const int4* haps, int nhaps, const long long* tab_row0,
                             long long ntab_rows, uint32_t* hapw, hipStream_t s)
{
    if (ntab_rows <= 0 || nhaps <= 0) return hipSuccess;
    hipLaunchKernelGGL(hap_tables_kernel, dim3(unsigned((ntab_rows + 255) / 256)), dim3(256), 0, s, hap_bytes,
                       haps, nhaps, tab_row0, ntab_rows, hapw);
    return hipGetLastError();
}

}  // namespace hcphmm
