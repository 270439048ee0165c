// Flat calls (hc_phmm_pairs_flat / hc_phmm_submit_pairs: independent pairs in
// the caller's host pools) planned on the device. The host does only what
// needs the caller's memory, in two parallel passes over the pairs:
//   pass 1  validate, lengths and record sizes per mini-task, a sample of
//           haplotype lengths for the width-cap model (lengths only: 8 bytes
//           per pair);
//   pass 2  write each pair's record — base qualities, read and hap base codes
//           as nibbles (1.5 bytes per read base, 0.5 per hap base instead of
//           2 + 1), gap planes only when they vary — and descriptor into the
//           device's pinned staging ring, chunk by chunk, each chunk's H2D
//           overlapping the fill of the next. The gap qualities' constancy
//           (the reference's constant 'I'/'+' strings, sam.hpp:30-32, travel
//           as three bytes per read) is checked while filling; a part that
//           turns out to hold a read with varying gap qualities is planned
//           again with the check in pass 1, so its records carry the planes;
//           one whose reads or haps do not fit the compact fields (an 'N') is
//           planned again with the nibble fields (pass 1 still lengths only).
// The device then packs rows and hap tables, chooses each pair's
// column-segmented shape by the planner's cost model (plan_model.hpp), sorts
// the pairs by (block width, lanes, R) and cuts the sorted runs into waves
// (pack_kernels.hip flat_*), and runs the pass. No per-call pinned allocation.
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <array>
#include <atomic>
#include <cstring>

#include "engine_core.hpp"
#include "plan_model.hpp"
#include "pool.hpp"

namespace hcphmm {
namespace eng {
namespace {

constexpr int kMini = 512;              // pairs per mini-task of the host passes
constexpr int kMaxGroups = 1024;        // flat_scan_kernel: one group per thread
constexpr int kMaxBins = 1 << 20;

// Per mini-task results of pass 1.
struct Mini {
    int64_t rec = 0, rows = 0, hapw = 0;   // sums, then (after the scan) offsets
    int rmax = 0, rmin = INT32_MAX, hmax = 0, hmin = INT32_MAX;
    int nwide = 0;
    bool bad = false;
};

struct FlatScratch {
    std::vector<int32_t> gapw;
    std::vector<uint8_t> fmtw;   // scanning pass 1: each pair's record format (kFmt* bits)
    std::vector<Mini> mini;
    std::vector<int32_t> hsamp;
};
thread_local FlatScratch t_fs;

template <typename T>
void grow(std::vector<T>& v, size_t n)
{
    if (v.size() < n) v.resize(n);
}

// Gap qualities of a read constant over its rows (blocks of 64 without early
// exit inside a block, so the compiler vectorises the compare).
bool constant_gaps_scalar(const uint8_t* i, const uint8_t* d, const uint8_t* c, int len)
{
    const uint8_t i0 = i[0], d0 = d[0], c0 = c[0];
    int k = 0;
    for (; k + 64 <= len; k += 64) {
        uint8_t a = 0;
        for (int j = 0; j < 64; ++j) a |= uint8_t((i[k + j] ^ i0) | (d[k + j] ^ d0) | (c[k + j] ^ c0));
        if (a) return false;
    }
    uint8_t a = 0;
    for (; k < len; ++k) a |= uint8_t((i[k] ^ i0) | (d[k] ^ d0) | (c[k] ^ c0));
    return a == 0;
}

// The same, 32 bytes of each plane per step; the last step overlaps the one
// before instead of a scalar tail.
__attribute__((target("avx2"))) inline __m256i gap_diff32(const uint8_t* i, const uint8_t* d, const uint8_t* c,
                                                           __m256i vi, __m256i vd, __m256i vc)
{
    const __m256i x = _mm256_xor_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(i)), vi);
    const __m256i y = _mm256_xor_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(d)), vd);
    const __m256i z = _mm256_xor_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(c)), vc);
    return _mm256_or_si256(_mm256_or_si256(x, y), z);
}

__attribute__((target("avx2"))) bool constant_gaps_avx2(const uint8_t* i, const uint8_t* d, const uint8_t* c,
                                                        int len)
{
    if (len < 32) return constant_gaps_scalar(i, d, c, len);
    const __m256i vi = _mm256_set1_epi8(char(i[0])), vd = _mm256_set1_epi8(char(d[0])),
                  vc = _mm256_set1_epi8(char(c[0]));
    __m256i acc = _mm256_setzero_si256();
    int k = 0;
    for (; k + 32 <= len; k += 32) acc = _mm256_or_si256(acc, gap_diff32(i + k, d + k, c + k, vi, vd, vc));
    if (k < len) {
        const int t = len - 32;
        acc = _mm256_or_si256(acc, gap_diff32(i + t, d + t, c + t, vi, vd, vc));
    }
    return _mm256_testz_si256(acc, acc) != 0;
}

bool has_avx2()
{
    static const bool v = __builtin_cpu_supports("avx2");
    return v;
}

bool constant_gaps(const uint8_t* i, const uint8_t* d, const uint8_t* c, int len)
{
    return has_avx2() ? constant_gaps_avx2(i, d, c, len) : constant_gaps_scalar(i, d, c, len);
}

constexpr int align4(int x) { return (x + 3) & ~3; }

// Record of a pair (pack_kernels.hip flat_prep_kernel), each field 4-byte
// aligned: the read — one byte per base (kFmtRead1B: quality delta and 2-bit
// code) or its qualities then its code nibbles —, [i, d, c planes], the hap —
// 2-bit codes (kFmtHap2b) or nibbles.
inline int64_t record_bytes(int R, int H, bool planes, int fmt)
{
    return align4(R) + ((fmt & kFmtRead1B) ? 0 : align4((R + 1) / 2)) + (planes ? 3 * int64_t(align4(R)) : 0) +
           ((fmt & kFmtHap2b) ? align4((H + 3) / 4) : align4((H + 1) / 2));
}

// ConvertChar (pairhmm_common.h:26-44): A0 C1 T2 G3 N4, every other byte -> 0.
const std::array<uint8_t, 256>& code_table()
{
    static const std::array<uint8_t, 256> t = [] {
        std::array<uint8_t, 256> x{};
        x['C'] = 1;
        x['T'] = 2;
        x['G'] = 3;
        x['N'] = 4;
        return x;
    }();
    return t;
}

// Base codes of n bytes as nibbles, two per byte (byte k/2: code k in the low
// nibble when k is even).
void pack_nibbles_scalar(const uint8_t* __restrict s, int n, uint8_t* __restrict d)
{
    const auto& ct = code_table();
    int k = 0;
    for (; k + 1 < n; k += 2) d[k >> 1] = uint8_t(ct[s[k]] | ct[s[k + 1]] << 4);
    if (k < n) d[k >> 1] = ct[s[k]];
}

__attribute__((target("avx2"))) inline __m256i codes32(__m256i v)
{
    // Two nibble lookups instead of four compares: the low nibble gives the
    // code (A 1 -> 0, C 3 -> 1, T 4 -> 2, G 7 -> 3, N E -> 4) and the high
    // nibble that byte must have (4, or 5 for T); any other byte -> 0.
    const __m256i lo = _mm256_and_si256(v, _mm256_set1_epi8(0x0f));
    const __m256i hi = _mm256_and_si256(_mm256_srli_epi16(v, 4), _mm256_set1_epi8(0x0f));
    const __m256i code_lut = _mm256_setr_epi8(0, 0, 0, 1, 2, 0, 0, 3, 0, 0, 0, 0, 0, 0, 4, 0,   //
                                              0, 0, 0, 1, 2, 0, 0, 3, 0, 0, 0, 0, 0, 0, 4, 0);
    const __m256i hi_lut = _mm256_setr_epi8(16, 16, 16, 4, 5, 16, 16, 4, 16, 16, 16, 16, 16, 16, 4, 16,   //
                                            16, 16, 16, 4, 5, 16, 16, 4, 16, 16, 16, 16, 16, 16, 4, 16);
    return _mm256_and_si256(_mm256_cmpeq_epi8(_mm256_shuffle_epi8(hi_lut, lo), hi), _mm256_shuffle_epi8(code_lut, lo));
}

// 32 bytes -> 16 nibble bytes.
__attribute__((target("avx2"))) inline __m128i nibbles32(const uint8_t* s)
{
    const __m256i pairmul = _mm256_set1_epi16(0x1001);   // even byte * 1 + odd byte * 16
    const __m256i p = _mm256_maddubs_epi16(codes32(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(s))), pairmul);
    const __m256i pk = _mm256_permute4x64_epi64(_mm256_packus_epi16(p, p), 0xD8);
    return _mm256_castsi256_si128(pk);
}

__attribute__((target("avx2"))) void pack_nibbles_avx2(const uint8_t* __restrict s, int n, uint8_t* __restrict d)
{
    if (n < 32) {
        pack_nibbles_scalar(s, n, d);
        return;
    }
    int k = 0;
    for (; k + 32 <= n; k += 32) _mm_storeu_si128(reinterpret_cast<__m128i*>(d + (k >> 1)), nibbles32(s + k));
    if (k < n) {
        // the last 32 bytes from an even start, overlapping what is written
        // (same values); an odd last byte beyond them alone
        const int t = (n - 32) & ~1;
        _mm_storeu_si128(reinterpret_cast<__m128i*>(d + (t >> 1)), nibbles32(s + t));
        if (t + 32 < n) d[(n - 1) >> 1] = code_table()[s[n - 1]];
    }
}

// Bytes copied 32 at a time, the last 32 overlapping (n >= 32), else memcpy.
__attribute__((target("avx2"))) void copy_bytes_avx2(const uint8_t* __restrict s, int n, uint8_t* __restrict d)
{
    if (n < 32) {
        std::memcpy(d, s, size_t(n));
        return;
    }
    int k = 0;
    for (; k + 32 <= n; k += 32)
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(d + k), _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + k)));
    if (k < n)
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(d + n - 32),
                            _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + n - 32)));
}

}  // namespace

void copy_bytes(const uint8_t* s, int n, uint8_t* d)
{
    if (has_avx2())
        copy_bytes_avx2(s, n, d);
    else
        std::memcpy(d, s, size_t(n));
}

void pack_nibbles(const uint8_t* s, int n, uint8_t* d)
{
    if (has_avx2())
        pack_nibbles_avx2(s, n, d);
    else
        pack_nibbles_scalar(s, n, d);
}

namespace {

// ---- compact record fields (kernels.hpp kFmtRead1B / kFmtHap2b)

// The compact fields, unless HC_PHMM_FLAT_COMPACT=0 (A/B: the nibble records).
int compact_fmt()
{
    static const int f = std::getenv("HC_PHMM_FLAT_COMPACT") && std::getenv("HC_PHMM_FLAT_COMPACT")[0] == '0'
                             ? 0
                             : (kFmtRead1B | kFmtHap2b);
    return f;
}

// A read fits one byte per base, ((q & 127) - 33) << 2 | code, when no base
// is 'N' and every quality (& 127) is in [33, 97): SAM's ASCII qualities
// (Phred 0-63 + 33) always are. The quality base is the fixed 33 so the
// check and the packing are one pass (kernels.hpp kFmtRead1B: qbase in the
// descriptor).
constexpr int kQBase = 33;

bool read_1b_scalar(const uint8_t* q, const uint8_t* b, int R, uint8_t* d)
{
    const auto& ct = code_table();
    bool ok = true;
    for (int k = 0; k < R; ++k) {
        const int v = (q[k] & 127) - kQBase;
        ok &= unsigned(v) < 64u && b[k] != 'N';
        if (d) d[k] = uint8_t((v << 2) | (ct[b[k]] & 3));
    }
    return ok;
}

// 32 bases: the packed bytes, and the running "bad" accumulator (a delta past
// 63 — qualities below 33 wrap — or an 'N').
__attribute__((target("avx2"))) inline __m256i read_1b32(const uint8_t* q, const uint8_t* b, __m256i& vmax, __m256i& vn)
{
    const __m256i v = _mm256_sub_epi8(
        _mm256_and_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(q)), _mm256_set1_epi8(0x7f)),
        _mm256_set1_epi8(char(kQBase)));
    const __m256i bb = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(b));
    vmax = _mm256_max_epu8(vmax, v);
    vn = _mm256_or_si256(vn, _mm256_cmpeq_epi8(bb, _mm256_set1_epi8('N')));
    // v < 64 where it matters (else the read is refused): the 16-bit shift
    // carries only zero bits across bytes
    return _mm256_or_si256(_mm256_slli_epi16(v, 2), codes32(bb));
}

__attribute__((target("avx2"))) bool read_1b_avx2(const uint8_t* q, const uint8_t* b, int R, uint8_t* d)
{
    if (R < 32) return read_1b_scalar(q, b, R, d);
    __m256i vmax = _mm256_setzero_si256(), vn = _mm256_setzero_si256();
    int k = 0;
    for (; k + 32 <= R; k += 32) {
        const __m256i x = read_1b32(q + k, b + k, vmax, vn);
        if (d) _mm256_storeu_si256(reinterpret_cast<__m256i*>(d + k), x);
    }
    if (k < R) {   // the last 32 overlapping what is written (same values)
        const __m256i x = read_1b32(q + R - 32, b + R - 32, vmax, vn);
        if (d) _mm256_storeu_si256(reinterpret_cast<__m256i*>(d + R - 32), x);
    }
    // every delta < 64: no byte of vmax has bit 6 or 7 set
    const __m256i hi = _mm256_and_si256(vmax, _mm256_set1_epi8(char(0xc0)));
    return _mm256_testz_si256(hi, hi) && _mm256_testz_si256(vn, vn);
}

// Pack the read (d may be null: check only); false if it does not fit.
bool read_1b(const uint8_t* q, const uint8_t* b, int R, uint8_t* d)
{
    return has_avx2() ? read_1b_avx2(q, b, R, d) : read_1b_scalar(q, b, R, d);
}

// Hap codes 2 bits each (a hap with no 'N'): false if it has one.
bool pack_hap_2b_scalar(const uint8_t* s, int n, uint8_t* d)
{
    const auto& ct = code_table();
    bool ok = true;
    for (int k = 0; k < n; k += 4) {
        uint8_t x = 0;
        for (int j = 0; j < 4 && k + j < n; ++j) {
            const uint8_t c = ct[s[k + j]];
            ok &= c != 4;
            x |= uint8_t((c & 3) << (2 * j));
        }
        d[k >> 2] = x;
    }
    return ok;
}

__attribute__((target("avx2"))) bool pack_hap_2b_avx2(const uint8_t* s, int n, uint8_t* d)
{
    const __m256i kN = _mm256_set1_epi8('N');
    const __m256i gather = _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                            0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    __m256i vn = _mm256_setzero_si256();
    int k = 0;
    for (; k + 32 <= n; k += 32) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + k));
        vn = _mm256_or_si256(vn, _mm256_cmpeq_epi8(v, kN));
        // codes c0 + 4 c1 per 16 bits, then (c0 + 4 c1) + 16 (c2 + 4 c3) per 32 bits
        const __m256i t = _mm256_maddubs_epi16(codes32(v), _mm256_set1_epi16(0x0401));
        const __m256i u = _mm256_madd_epi16(t, _mm256_set1_epi32(0x00100001));
        const __m256i g = _mm256_shuffle_epi8(u, gather);
        const uint64_t w = uint64_t(uint32_t(_mm256_extract_epi32(g, 0))) |
                           (uint64_t(uint32_t(_mm256_extract_epi32(g, 4))) << 32);
        std::memcpy(d + (k >> 2), &w, 8);
    }
    const bool ok = k < n ? pack_hap_2b_scalar(s + k, n - k, d + (k >> 2)) : true;
    return ok && _mm256_testz_si256(vn, vn);
}

bool pack_hap_2b(const uint8_t* s, int n, uint8_t* d)
{
    return has_avx2() ? pack_hap_2b_avx2(s, n, d) : pack_hap_2b_scalar(s, n, d);
}

bool has_n(const uint8_t* s, int n) { return std::memchr(s, 'N', size_t(n)) != nullptr; }

}  // namespace

// (test hooks below)
bool read_1b_hook(const uint8_t* q, const uint8_t* b, int R, uint8_t* d) { return read_1b(q, b, R, d); }
bool pack_hap_2b_hook(const uint8_t* s, int n, uint8_t* d) { return pack_hap_2b(s, n, d); }

namespace {

// Why pass 2 refused a part planned without scanning (fill_chunk `retry` bits).
constexpr int kGapsVary = 1;     // a read's gap qualities vary: plan again scanning them (planes)
constexpr int kNotCompact = 2;   // a read or hap does not fit the compact fields: plan again with nibbles

// Pass 2 over mini-tasks [m0, m1): each pair's record at buf + (its offset
// - r0) and its descriptor at dd[k - p0]. With scan_gaps false (pass 1 assumed
// constant gap qualities and format fmt0 everywhere), a read whose gap
// qualities vary sets kGapsVary in `retry` (the part is planned again with
// pass 1 scanning: gapw[k], fmtw[k]); a read that does not fit one byte per
// base, or a hap with an 'N', where fmt0 assumed so, sets kNotCompact (planned
// again with fmt0 = 0, still without scanning).
void fill_chunk(const Src& src, int64_t lo, int64_t n, int64_t m0, int64_t m1, const Mini* mini,
                const int32_t* gapw, const uint8_t* fmtw, bool scan_gaps, int fmt0, char* buf, int64_t r0,
                FlatDesc* dd, int64_t p0, std::atomic<int>& retry)
{
    parallel_for(m1 - m0, [&](int64_t a, int64_t e) {
        for (int64_t m = m0 + a; m < m0 + e; ++m) {
            int64_t ro = mini[m].rec, rw = mini[m].rows, hw = mini[m].hapw;
            const int64_t k1 = std::min(n, (m + 1) * kMini);
            for (int64_t k = m * kMini; k < k1; ++k) {
                const int64_t p = lo + k;
                const int R = src.R[p], H = src.H[p];
                const int64_t o = src.read_off[p];
                int32_t g;
                int fmt;
                if (scan_gaps) {
                    g = gapw[k];
                    fmt = fmtw[k];
                } else {
                    const uint8_t *ip = src.ins + o, *dp = src.del + o, *cp = src.gcp + o;
                    if (!constant_gaps(ip, dp, cp, R)) {
                        retry.fetch_or(kGapsVary, std::memory_order_relaxed);
                        return;
                    }
                    g = int32_t((ip[0] & 127) | ((dp[0] & 127) << 7) | ((cp[0] & 127) << 14));
                    fmt = fmt0;
                }
                const int qa = align4(R);
                uint8_t* d = reinterpret_cast<uint8_t*>(buf + (ro - r0));
                size_t at = size_t(qa);
                const int qbase = (fmt & kFmtRead1B) ? kQBase : 0;
                if (fmt & kFmtRead1B) {
                    if (!read_1b(src.q + o, src.rs + o, R, d)) {
                        retry.fetch_or(kNotCompact, std::memory_order_relaxed);   // (scan mode never lists such a read)
                        return;
                    }
                } else {
                    copy_bytes(src.q + o, R, d);
                    pack_nibbles(src.rs + o, R, d + qa);
                    at += size_t(align4((R + 1) / 2));
                }
                if (g < 0) {
                    std::memcpy(d + at, src.ins + o, size_t(R));
                    std::memcpy(d + at + qa, src.del + o, size_t(R));
                    std::memcpy(d + at + 2 * qa, src.gcp + o, size_t(R));
                    at += 3 * size_t(qa);
                }
                if (fmt & kFmtHap2b) {
                    if (!pack_hap_2b(src.hap + src.hap_off[p], H, d + at)) {
                        retry.fetch_or(kNotCompact, std::memory_order_relaxed);
                        return;
                    }
                } else {
                    pack_nibbles(src.hap + src.hap_off[p], H, d + at);
                }
                dd[k - p0] = FlatDesc{ro, int(rw), R, H, int(hw), g, fmt | (qbase << 8)};
                ro += record_bytes(R, H, g < 0, fmt);
                rw += qa;
                hw += hap_table_words(H);
            }
        }
    }, 1);
}

// Pass 1 over pairs [lo, lo + n): per mini-task sums and bounds; with
// scan_gaps, each read's constant gap triple (or -1) in gapw and its format
// (compact fields where they fit, if compact_fmt() allows) in fmtw; without,
// every pair is assumed to take format fmt0; every stride-th hap length in hsamp.
void scan_pass(const Src& src, int64_t lo, int64_t n, bool scan_gaps, int fmt0, Mini* mini, int32_t* gapw,
               uint8_t* fmtw, int32_t* hsamp, int64_t stride)
{
    const int64_t nmini = (n + kMini - 1) / kMini;
    parallel_for(nmini, [&](int64_t m0, int64_t m1) {
        for (int64_t m = m0; m < m1; ++m) {
            Mini& M = mini[m];
            const int64_t a = m * kMini, e = std::min(n, a + kMini);
            for (int64_t k = a; k < e; ++k) {
                const int64_t p = lo + k;
                const int R = src.R[p], H = src.H[p];
                if (R <= 0 || R > HC_PHMM_MAX_READ_LEN || H <= 0 || H > HC_PHMM_MAX_HAP_LEN) {
                    M.bad = true;
                    gapw[k] = 0;
                    continue;
                }
                int32_t g = 0;
                int fmt = fmt0;   // assumed (checked by pass 2) unless scanning
                if (scan_gaps) {
                    const int64_t o = src.read_off[p];
                    const uint8_t *ip = src.ins + o, *dp = src.del + o, *cp = src.gcp + o;
                    g = constant_gaps(ip, dp, cp, R)
                            ? int32_t((ip[0] & 127) | ((dp[0] & 127) << 7) | ((cp[0] & 127) << 14))
                            : -1;
                    gapw[k] = g;
                    fmt = compact_fmt() == 0 ? 0
                                             : (read_1b(src.q + o, src.rs + o, R, nullptr) ? kFmtRead1B : 0) |
                                                   (has_n(src.hap + src.hap_off[p], H) ? 0 : kFmtHap2b);
                    fmtw[k] = uint8_t(fmt);
                }
                M.rec += record_bytes(R, H, g < 0, fmt);
                M.rows += align4(R);
                M.hapw += hap_table_words(H);
                M.rmax = std::max(M.rmax, R);
                M.rmin = std::min(M.rmin, R);
                M.hmax = std::max(M.hmax, H);
                M.hmin = std::min(M.hmin, H);
                M.nwide += H > kSeg64MaxH;
                if (k % stride == 0) hsamp[k / stride] = H;
            }
        }
    }, 8);
}

constexpr int kRetryWithPlanes = 1;   // plan_flat_try: a read's gap qualities vary
constexpr int kRetryNibbles = 2;      // plan_flat_try: a read or hap does not fit the compact fields

// Does a sample of the part's pairs (every stride-th, at most ~1 024) all fit
// the compact fields? Real reads often hold an 'N': such a part then starts
// with the nibble fields instead of finding out in pass 2, where the refusal
// costs the chunks filled so far and a second planning (advisor round 5).
bool sample_fits_compact(const Src& src, int64_t lo, int64_t n)
{
    if (compact_fmt() == 0) return false;
    const int64_t stride = std::max<int64_t>(1, n / 1024);
    for (int64_t k = 0; k < n; k += stride) {
        const int64_t p = lo + k, o = src.read_off[p];
        const int R = src.R[p], H = src.H[p];
        if (R <= 0 || H <= 0) continue;   // (pass 1 refuses the part)
        if (!read_1b(src.q + o, src.rs + o, R, nullptr) || has_n(src.hap + src.hap_off[p], H)) return false;
    }
    return true;
}

bool default_policies()
{
    for (const char* e : {"HC_PHMM_KERNEL", "HC_PHMM_LANE_SEG"}) {
        const char* v = std::getenv(e);
        if (v && *v && std::strcmp(v, "auto") != 0) return false;
    }
    return env_i64("HC_PHMM_SEG_CAP", 0) <= 0 && env_i64("HC_PHMM_SEG_Q", -1) < 0 &&
           env_i64("HC_PHMM_FLAT_PLAN", 1) != 0;
}

}  // namespace

namespace {

// One attempt: scan_gaps = false assumes constant gap qualities and format
// fmt0 everywhere (checked in pass 2; kRetryWithPlanes / kRetryNibbles if
// not), true finds each pair's in pass 1. record_rate: this attempt's host
// staging time updates the device's measured rate (not after a refused
// attempt, whose wasted work would read as slow staging).
int plan_flat_try(Device& dv, const Src& src, const PartSpec& spec, Slot* slot, bool with_run, bool scan_gaps,
                  int fmt0, bool record_rate, Part** out)
{
    *out = nullptr;
    PhaseTimer tm;
    using clk = std::chrono::steady_clock;
    const clk::time_point t_begin = clk::now();
    clk::duration t_stage{};   // scan + fill: the host staging rate (Device::stage_ps_per_cell)
    const int64_t lo = spec.lo, n = spec.hi - spec.lo;
    if (n <= 0 || n > (int64_t(1) << 31) - 1) return HC_PHMM_OK;
    FlatScratch& S = t_fs;
    grow(S.gapw, size_t(n));
    grow(S.fmtw, size_t(n));
    const int64_t nmini = (n + kMini - 1) / kMini;
    S.mini.assign(size_t(nmini), Mini{});
    const int64_t stride = std::max<int64_t>(1, n / 8192);   // cap-model sample of hap lengths
    const int64_t nsamp = (n + stride - 1) / stride;
    grow(S.hsamp, size_t(nsamp));
    int32_t* gapw = S.gapw.data();
    uint8_t* fmtw = S.fmtw.data();
    Mini* mini = S.mini.data();
    int32_t* hsamp = S.hsamp.data();

    scan_pass(src, lo, n, scan_gaps, fmt0, mini, gapw, fmtw, hsamp, stride);
    t_stage += clk::now() - t_begin;
    tm.mark("flat: scan");

    int rmax = 0, rmin = INT32_MAX, hmax = 0, hmin = INT32_MAX;
    int64_t nwide = 0, rec = 0, rows = 0, hapw = 0;
    for (int64_t m = 0; m < nmini; ++m) {
        Mini& M = mini[m];
        if (M.bad) return fail(HC_PHMM_EINVAL, "pair with invalid read length (1.." +
                                                   std::to_string(HC_PHMM_MAX_READ_LEN) + ") or hap length (1.." +
                                                   std::to_string(HC_PHMM_MAX_HAP_LEN) + ")");
        rmax = std::max(rmax, M.rmax);
        rmin = std::min(rmin, M.rmin);
        hmax = std::max(hmax, M.hmax);
        hmin = std::min(hmin, M.hmin);
        nwide += M.nwide;
        const int64_t r = M.rec, w = M.rows, h = M.hapw;
        M.rec = rec;
        M.rows = rows;
        M.hapw = hapw;
        rec += r;
        rows += w;
        hapw += h;
    }
    // Every pair must fit the column-segmented kernel (64 lanes of 64 columns);
    // the host planner takes the others. So must the row and table pools.
    if (hmax > 64 * kSegMaxBC || rows > INT32_MAX - 4096 || hapw > INT32_MAX) return HC_PHMM_OK;

    // Width cap and the per-length candidates; groups = distinct (BC, nb),
    // widest block first.
    const double ravg = double(rows) / double(n);
    int64_t lanes_at[kNCaps] = {};
    double work_at[kNCaps] = {};
    {   // the model over the sample's distinct lengths, weighted by their counts
        std::vector<int32_t> hist(size_t(std::min(hmax, 64 * kSegMaxBC)) + 1, 0);
        for (int64_t s = 0; s < nsamp; ++s) ++hist[size_t(std::min(hsamp[s], 64 * kSegMaxBC))];
        for (int H = 1; H < int(hist.size()); ++H)
            if (hist[size_t(H)]) cap_sample(H, ravg, stride * hist[size_t(H)], lanes_at, work_at);
    }
    const CapChoice cc = choose_cap(lanes_at, work_at, dv.n_cu);
    const float* waste = cc.few_waves ? waste_per_lane() : waste_full();
    std::vector<Cand> cand(size_t(hmax) + 1);
    std::vector<uint16_t> keys;
    for (int H = hmin; H <= hmax; ++H) {
        cand[size_t(H)] = cand_of(H, cc.cap);
        for (int q = 0; q < 2; ++q) keys.push_back(uint16_t(cand[size_t(H)].bc[q] << 8 | cand[size_t(H)].nb[q]));
    }
    std::sort(keys.begin(), keys.end(), std::greater<uint16_t>());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    const int ngroups = int(keys.size());
    if (ngroups > kMaxGroups) return HC_PHMM_OK;
    std::vector<int> gid(1 << 16, -1);
    for (int g = 0; g < ngroups; ++g) gid[keys[size_t(g)]] = g;
    // Counting-sort bins: (group, R descending), R coarsened if the span is wide.
    int rshift = 0;
    while (int64_t(ngroups) * (((rmax - rmin) >> rshift) + 1) > kMaxBins) ++rshift;
    const int rspan = ((rmax - rmin) >> rshift) + 1;
    const int nbins = ngroups * rspan;
    // Waves the launch must cover: at most ceil(pairs / per) per group, per =
    // floor(64 / nb) with nb the larger of a length's two candidates.
    std::vector<float> inv_per(size_t(hmax) + 1, 0.f);
    for (int H = hmin; H <= hmax; ++H)
        inv_per[size_t(H)] = 1.f / float(64 / std::max(cand[size_t(H)].nb[0], cand[size_t(H)].nb[1]));
    std::atomic<int64_t> wsum{0};
    parallel_for(n, [&](int64_t a, int64_t e) {
        double s = 0;
        for (int64_t k = a; k < e; ++k) s += inv_per[size_t(src.H[lo + k])];
        wsum += int64_t(s) + 2;
    }, 16384);
    const int64_t max_waves = wsum.load() + ngroups + 1;
    if (max_waves > INT32_MAX / 4) return HC_PHMM_OK;
    tm.mark("flat: model");

    // Upload chunks: runs of mini-tasks whose records + descriptors fit a ring chunk.
    std::vector<int64_t> chunk_m{0};
    {
        int64_t m = 0;
        while (m < nmini) {
            int64_t e = m;
            auto bytes = [&](int64_t m1) {
                const int64_t r1 = m1 < nmini ? mini[m1].rec : rec;
                const int64_t pairs = std::min(n, m1 * kMini) - m * kMini;
                return ((r1 - mini[m].rec + 255) & ~int64_t(255)) + int64_t(sizeof(FlatDesc)) * pairs;
            };
            while (e < nmini && bytes(e + 1) <= int64_t(kRingChunk)) ++e;
            if (e == m) return HC_PHMM_OK;   // one mini-task larger than a chunk: host planner
            chunk_m.push_back(e);
            m = e;
        }
    }

    // Device layout: the upload image, descriptors and tables, then what the
    // device builds, the outputs and the rescue scratch.
    const size_t n1 = size_t(n);
    const ResLayout RL = res_layout(n1);
    const size_t res_bytes = RL.bytes;
    struct Lay {
        size_t off = 0;
        size_t take(size_t b)
        {
            const size_t o = off;
            off += (b + 255) & ~size_t(255);
            return o;
        }
    } L;
    const size_t o_img = L.take(size_t(rec) + 16);
    const size_t o_desc = L.take(sizeof(FlatDesc) * n1);
    const size_t tab_bytes = sizeof(int2) * (size_t(hmax) + 1) + sizeof(float) * 65 + sizeof(int2) * size_t(ngroups);
    const size_t o_tab = L.take(tab_bytes);
    const size_t row_pad = kRowPadBefore + size_t(rmax) + 256;
    if (int64_t(rows) + int64_t(row_pad) > kMaxRowWords)
        return fail(HC_PHMM_EINVAL, "batch too large (read bases of one part exceed 2^30)");
    if (int64_t(hapw) + 16 > kMaxHapWords)
        return fail(HC_PHMM_EINVAL, "batch too large (hap match tables of one part exceed 2^30 words)");
    const size_t o_rows = L.take(sizeof(uint32_t) * (size_t(rows) + row_pad));
    const size_t o_hapw = L.take(sizeof(uint32_t) * (size_t(hapw) + 16));
    const size_t o_pairs = L.take(sizeof(PairDesc) * n1);
    const size_t o_binof = L.take(sizeof(int) * n1);
    const size_t o_hist = L.take(sizeof(int) * size_t(nbins));
    const size_t o_gtab = L.take(sizeof(int) * 3 * size_t(ngroups));
    const size_t o_order = L.take(sizeof(int) * n1);
    const size_t o_waves = L.take(sizeof(LaneWave) * size_t(max_waves));
    // The last two rounds of wave slots (3 per SIMD) dispatched longest first
    // (planner.cpp: 125k-pair shard 1.39 -> 1.25 ms with it on the host plan).
    const int tail = int(std::max<int64_t>(0, env_i64("HC_PHMM_TAIL_ROUNDS", 2))) * 4 * dv.n_cu * 3;
    const size_t o_wtmp = L.take(tail > 0 ? sizeof(LaneWave) * size_t(max_waves) : 0);
    const size_t o_wcost = L.take(tail > 0 ? sizeof(int) * size_t(max_waves) : 0);
    const size_t o_nw = L.take(2 * sizeof(int));   // wave count, then the largest modelled wave cost
    const size_t o_res = L.take(res_bytes);
    const size_t o_list = L.take(2 * sizeof(int) * n1);   // pair ids, then pack_rh (Seg64Args::list_rh)
    const size_t o_rec = L.take(sizeof(uint4) * n1);   // seg slot records (every pair is a seg pair)
    const size_t o_slotof = L.take(sizeof(int) * n1);
    const size_t o_sdesc = L.take(sizeof(PairDesc) * n1);
    const size_t o_sorted = L.take(sizeof(int) * n1);
    const size_t o_worder = L.take(sizeof(int) * n1);
    const size_t o_big = L.take(sizeof(int) * n1);
    const size_t o_bigc = L.take(sizeof(int));
    const size_t o_plan = L.take(sizeof(Seg64Plan));
    const size_t total = L.off;
    const size_t host_res_off = (tab_bytes + 255) & ~size_t(255);
    // Jobs borrow their slot's workspace; batches (slot == nullptr) own their
    // device memory, and their tables go up from plain host memory.
    std::vector<char> own_tab;
    char* dev = nullptr;
    char* host = nullptr;
    int rc = HC_PHMM_OK;
    if (slot) {
        tm.mark("flat: layout (sizes)");
        rc = slot_reserve(*slot, total, host_res_off + res_bytes);
        if (rc) return rc;
        dev = slot->dev;
        host = slot->host;
    } else {
        if (hipMalloc(&dev, total) != hipSuccess)
            return fail(HC_PHMM_ENOMEM, "device allocation failed (" + std::to_string(total >> 20) + " MiB)");
        own_tab.resize(tab_bytes);
        host = own_tab.data();
    }
    tm.mark("flat: layout");

    // Tables (the slot's pinned area; its results image follows).
    {
        int2* ct = reinterpret_cast<int2*>(host);
        for (int H = 0; H <= hmax; ++H) {
            if (H < hmin) {
                ct[H] = make_int2(0, 0);
                continue;
            }
            const Cand c = cand[size_t(H)];
            ct[H] = make_int2(c.bc[0] | c.nb[0] << 8 | gid[size_t(c.bc[0] << 8 | c.nb[0])] << 16,
                              c.bc[1] | c.nb[1] << 8 | gid[size_t(c.bc[1] << 8 | c.nb[1])] << 16);
        }
        float* wt = reinterpret_cast<float*>(ct + hmax + 1);
        std::memcpy(wt, waste, sizeof(float) * 65);
        int2* gt = reinterpret_cast<int2*>(wt + 65);
        for (int g = 0; g < ngroups; ++g) gt[g] = make_int2(keys[size_t(g)] >> 8, keys[size_t(g)] & 0xff);
    }

    Part* b = nullptr;
    try {
        b = new_part(&dv);
    } catch (...) {
        if (!slot) (void)hipFree(dev);
        throw;
    }
    PartGuard guard(b);   // error returns and exceptions discard it (and a batch's own allocation)
    b->slot = slot;
    b->dev_base = dev;   // a batch's own allocation (freed with it), or the slot's
    b->spec = spec;
    b->n = n;
    b->Hmax = hmax;
    b->n_lane = int(n);
    b->n_seg_waves = int(max_waves);
    b->lane_waves = int(max_waves);
    b->d_nwaves = reinterpret_cast<int*>(dev + o_nw);
    b->d_pairs = reinterpret_cast<PairDesc*>(dev + o_pairs);
    b->d_rows = reinterpret_cast<uint32_t*>(dev + o_rows) + kRowPadBefore;
    b->d_hapw = reinterpret_cast<uint32_t*>(dev + o_hapw);
    b->d_lane_order = reinterpret_cast<int*>(dev + o_order);
    b->d_lane_waves = reinterpret_cast<LaneWave*>(dev + o_waves);
    b->res_bytes = res_bytes;
    b->res_o64 = RL.o64;
    b->res_ofl = RL.ofl;
    b->res_ocnt = RL.ocnt;
    b->own_raw32 = b->d_raw32 = reinterpret_cast<float*>(dev + o_res);
    b->own_raw64 = b->d_raw64 = reinterpret_cast<double*>(dev + o_res + RL.o64);
    b->own_flag = b->d_flag = reinterpret_cast<uint8_t*>(dev + o_res + RL.ofl);
    b->d_list = reinterpret_cast<int*>(dev + o_list);
    b->d_count = reinterpret_cast<int*>(dev + o_res + RL.ocnt);   // run counters: the results block's tail
    b->d_sorted = reinterpret_cast<int*>(dev + o_sorted);
    b->d_worder = reinterpret_cast<int*>(dev + o_worder);
    b->d_big = reinterpret_cast<int*>(dev + o_big);
    b->d_big_count = reinterpret_cast<int*>(dev + o_bigc);
    b->d_plan = reinterpret_cast<Seg64Plan*>(dev + o_plan);
    b->d_rec = reinterpret_cast<uint4*>(dev + o_rec);
    b->d_slot_of = reinterpret_cast<int*>(dev + o_slotof);
    b->d_sdesc = reinterpret_cast<PairDesc*>(dev + o_sdesc);
    b->n_wide = nwide;
    if (slot) {
        b->host_res = host + host_res_off;
        b->stream = slot->stream;
        b->side = slot->side;
        b->fork = slot->fork;
        b->join = slot->join;
        b->slot_ev = true;
        b->pack_ev[0] = slot->ev[0];
        b->pack_ev[1] = slot->ev[1];
        b->ev_pool.push_back({slot->ev[2], slot->ev[3], slot->ev[4]});
        b->done = slot->ev[5];
        b->early = slot->ev[6];
    } else {
        b->stream = dv.stream;
        b->side = dv.side;
        b->fork = dv.fork;
        b->join = dv.join;
    }
    b->upload_bytes = size_t(rec) + sizeof(FlatDesc) * n1 + tab_bytes;
    hipStream_t s = b->stream;

    // Uploads and preparation on the part's own stream (a greatest-priority
    // stream for them gained ~0.2 ms with four equal parts and lost with the
    // growing parts, profiles/r05_e2e_parts_ab.txt; removed).
    const hipStream_t ps = s;
    std::atomic<int> retry{0};
    auto enqueue = [&]() -> int {
        // Pass 2: chunks through the ring, each H2D'd as soon as it is filled.
        // The staging rate counts the fills only: not the wait for the ring's
        // lock (another part's fill) nor for a chunk's previous H2D (device
        // backpressure), which are not host staging (advisor round 5).
        {
            std::lock_guard<std::mutex> lk(dv.ring.mu);
            for (size_t c = 0; c + 1 < chunk_m.size(); ++c) {
                const int64_t m0 = chunk_m[c], m1 = chunk_m[c + 1];
                const int64_t p0 = m0 * kMini, p1 = std::min(n, m1 * kMini);
                const int64_t r0 = mini[m0].rec, r1 = m1 < nmini ? mini[m1].rec : rec;
                const int ri = dv.ring.next;
                dv.ring.next = (ri + 1) % kRingN;
                if (dv.ring.used[ri]) HIP_TRY(hipEventSynchronize(dv.ring.ev[ri]));
                char* buf = dv.ring.buf[ri];
                const size_t dbase = (size_t(r1 - r0) + 255) & ~size_t(255);
                FlatDesc* dd = reinterpret_cast<FlatDesc*>(buf + dbase);
                const clk::time_point t_fill = clk::now();
                fill_chunk(src, lo, n, m0, m1, mini, gapw, fmtw, scan_gaps, fmt0, buf, r0, dd, p0, retry);
                t_stage += clk::now() - t_fill;
                if (const int why = retry.load()) return (why & kGapsVary) ? kRetryWithPlanes : kRetryNibbles;
                HIP_TRY(hipMemcpyAsync(dev + o_img + r0, buf, size_t(r1 - r0), hipMemcpyHostToDevice, ps));
                HIP_TRY(hipMemcpyAsync(dev + o_desc + sizeof(FlatDesc) * size_t(p0), dd,
                                       sizeof(FlatDesc) * size_t(p1 - p0), hipMemcpyHostToDevice, ps));
                HIP_TRY(hipEventRecord(dv.ring.ev[ri], ps));
                dv.ring.used[ri] = true;
            }
        }
        tm.mark("flat: fill + H2D");
        // Running mean over calls (weight 1/2 to the newest part), of parts
        // large enough to be pipeline parts (a small call's rate is its fixed
        // costs': hc_phmm_init's warm-up call would read as slow staging).
        if (record_rate && spec.cells >= 5e8) {
            const double ps = std::chrono::duration<double, std::pico>(t_stage).count() / spec.cells;
            double old_ps = dv.stage_ps_per_cell.load(std::memory_order_relaxed);
            while (!dv.stage_ps_per_cell.compare_exchange_weak(old_ps, old_ps > 0 ? 0.5 * (old_ps + ps) : ps,
                                                               std::memory_order_relaxed)) {
            }
        }
        if (!b->slot_ev)
            for (auto& e : b->pack_ev) HIP_TRY(hipEventCreate(&e));
        HIP_TRY(hipMemcpyAsync(dev + o_tab, host, tab_bytes, hipMemcpyHostToDevice, ps));
        HIP_TRY(hipEventRecord(b->pack_ev[0], ps));
        FlatPlanArgs a{};
        a.img = reinterpret_cast<const uint8_t*>(dev + o_img);
        a.desc = reinterpret_cast<const FlatDesc*>(dev + o_desc);
        a.n = int(n);
        a.rows = b->d_rows;
        a.hapw = b->d_hapw;
        a.pairs = b->d_pairs;
        a.ctab = reinterpret_cast<const int2*>(dev + o_tab);
        a.waste = reinterpret_cast<const float*>(dev + o_tab + sizeof(int2) * (size_t(hmax) + 1));
        a.groups = reinterpret_cast<const int2*>(dev + o_tab + sizeof(int2) * (size_t(hmax) + 1) + sizeof(float) * 65);
        a.rmax = rmax;
        a.rshift = rshift;
        a.rspan = rspan;
        a.bin_of = reinterpret_cast<int*>(dev + o_binof);
        a.hist = reinterpret_cast<int*>(dev + o_hist);
        a.nbins = nbins;
        a.ngroups = ngroups;
        a.gtab = reinterpret_cast<int*>(dev + o_gtab);
        a.order = b->d_lane_order;
        a.slot_of = b->d_slot_of;
        a.sdesc = b->d_sdesc;
        a.waves = b->d_lane_waves;
        a.waves_tmp = reinterpret_cast<LaneWave*>(dev + o_wtmp);
        a.wcost = reinterpret_cast<int*>(dev + o_wcost);
        a.tail = tail;
        a.max_waves = int(max_waves);
        a.nwaves = reinterpret_cast<int*>(dev + o_nw);
        a.counters = b->d_count;
        a.prep_blocks = int(env_i64("HC_PHMM_PREP_BLOCKS", 0));
        HIP_TRY(launch_flat_plan(a, ps));
        HIP_TRY(hipEventRecord(b->pack_ev[1], ps));
        if (with_run) {
            const int r = run_part(b, s);
            if (r) return r;
            return enqueue_results(b, s);
        }
        if (!slot) HIP_TRY(hipStreamSynchronize(s));   // the tables' host memory goes with this call
        return HC_PHMM_OK;
    };
    rc = enqueue();
    tm.mark("flat: enqueue");
    if (rc) return rc;   // the guard drains the stream and discards the part (the caller returns the slot)
    *out = guard.release();
    return HC_PHMM_OK;
}

}  // namespace

int plan_flat_device(Device& dv, const Src& src, const PartSpec& spec, Slot* slot, bool with_run, Part** out)
{
    *out = nullptr;
    if (!spec.flat || !src.R || !default_policies() || (!slot && with_run)) return HC_PHMM_OK;
    // Compact fields unless a sample of the part shows a pair that does not
    // fit them; refused in pass 2: the nibble fields (pass 1 still lengths
    // only), and varying gap qualities: pass 1 scanning every read.
    // After a refusal the device's next kNibbleParts parts skip the compact
    // attempt (rare 'N's the sample misses: 1 read in 10 000 made every S2
    // part refuse in pass 2, 25.7 vs 12.6 ms a call).
    const int64_t n = spec.hi - spec.lo;
    const bool skip_compact = dv.nibble_parts.load(std::memory_order_relaxed) > 0 &&
                              dv.nibble_parts.fetch_sub(1, std::memory_order_relaxed) > 0;
    int fmt0 = !skip_compact && n > 0 && sample_fits_compact(src, spec.lo, n) ? compact_fmt() : 0;
    int rc = plan_flat_try(dv, src, spec, slot, with_run, false, fmt0, true, out);
    if (rc == kRetryNibbles) {
        dv.nibble_parts.store(kNibbleParts, std::memory_order_relaxed);
        rc = plan_flat_try(dv, src, spec, slot, with_run, false, 0, false, out);
    }
    if (rc == kRetryWithPlanes) rc = plan_flat_try(dv, src, spec, slot, with_run, true, 0, false, out);
    return rc;
}

}  // namespace eng
}  // namespace hcphmm

// Host-logic test hook (not part of the ABI): the record's nibble packing.
extern "C" void hcx_pack_nibbles(const uint8_t* s, int n, uint8_t* d) { hcphmm::eng::pack_nibbles(s, n, d); }
// Host-logic test hooks (not part of the ABI): the compact record fields.
// Returns 1 if the read fits one byte per base (d holds it), else 0.
extern "C" int hcx_pack_read_1b(const uint8_t* q, const uint8_t* b, int n, uint8_t* d)
{
    return hcphmm::eng::read_1b_hook(q, b, n, d) ? 1 : 0;
}
// Returns 1 if the hap has no 'N' (d holds its 2-bit codes), else 0.
extern "C" int hcx_pack_hap_2b(const uint8_t* s, int n, uint8_t* d) { return hcphmm::eng::pack_hap_2b_hook(s, n, d) ? 1 : 0; }

// Host-pass timing without a GPU (not part of the ABI: tools/flat_host_bench.py):
// pass 1 and pass 2 of a flat call over pairs [0, n) into host memory, `reps`
// times; ms[0] = pass 1, ms[1] = pass 2 (mean per call).
extern "C" void hcx_flat_host_passes(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                                     const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                                     const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, int reps, double* ms)
{
    using namespace hcphmm;
    using namespace hcphmm::eng;
    Src src;
    src.read_off = read_off;
    src.R = R;
    src.hap_off = hap_off;
    src.H = H;
    src.rs = rs;
    src.q = q;
    src.ins = ins;
    src.del = del;
    src.gcp = gcp;
    src.hap = hap;
    const int64_t nmini = (n + kMini - 1) / kMini;
    std::vector<Mini> mini;
    std::vector<int32_t> gapw(static_cast<size_t>(n)), hsamp(static_cast<size_t>(n));
    std::vector<uint8_t> fmtw(static_cast<size_t>(n));
    std::vector<char> buf;
    std::vector<FlatDesc> dd(static_cast<size_t>(n));
    ms[0] = ms[1] = 0;
    for (int r = 0; r <= reps; ++r) {   // rep 0 sizes the buffers (untimed)
        auto t0 = std::chrono::steady_clock::now();
        mini.assign(size_t(nmini), Mini{});
        const int fmt0 = sample_fits_compact(src, 0, n) ? compact_fmt() : 0;
        scan_pass(src, 0, n, false, fmt0, mini.data(), gapw.data(), fmtw.data(), hsamp.data(),
                  std::max<int64_t>(1, n / 8192));
        int64_t rec = 0;
        for (auto& M : mini) {
            const int64_t x = M.rec;
            M.rec = rec;
            rec += x;
        }
        if (buf.size() < size_t(rec)) buf.resize(size_t(rec));
        auto t1 = std::chrono::steady_clock::now();
        std::atomic<int> retry{0};
        fill_chunk(src, 0, n, 0, nmini, mini.data(), gapw.data(), fmtw.data(), false, fmt0, buf.data(), 0, dd.data(),
                   0, retry);
        auto t2 = std::chrono::steady_clock::now();
        if (r == 0) continue;
        ms[0] += std::chrono::duration<double, std::milli>(t1 - t0).count() / reps;
        ms[1] += std::chrono::duration<double, std::milli>(t2 - t1).count() / reps;
    }
}
