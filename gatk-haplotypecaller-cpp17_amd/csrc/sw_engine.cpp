// Host engine + C ABI of the Smith-Waterman aligner (include/hc_sw.h).
//
// One batch = the loop of assembler/graph_wrapper.hpp:232-240 (every haplotype
// of a region against the region's reference window), for any number of
// regions at once:
//   create   order pairs longest first, lay out backtrack/element space, one H2D
//   run      sw_dp_kernel (DP + backtrack words + end point), sw_trace_kernel
//            (getCIGAR + compaction)                              [device only]
//   results  D2H offsets + packed CIGAR elements, "%d%c" formatting on the host
//            (PairWiseSW.h:388-413)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/hc_pairhmm.h"
#include "../../include/hc_sw.h"
#include "sw_kernels.hpp"

namespace hcphmm {
void set_last_error(const std::string& msg);
int primary_device();
void sw_release();
}

using namespace hcsw;

namespace {

std::mutex g_mu;
hipStream_t g_stream = nullptr;

// Grow-only workspace of the synchronous entry point (hc_sw_align_flat): a
// warm call does no hipMalloc / hipHostMalloc and one H2D + one D2H.
struct Workspace {
    char* dev = nullptr;
    size_t dev_bytes = 0;
    char* host = nullptr;   // pinned
    size_t host_bytes = 0;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
} g_ws;

int fail(int code, const std::string& msg)
{
    hcphmm::set_last_error(msg);
    return code;
}

#define HIP_TRY(expr)                                                                 \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(HC_SW_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// The aligner runs on the engine's first device slot (hc_phmm_init /
// hc_phmm_init_devices); every entry point makes that device current on the
// calling thread.
int ensure_init(int device)
{
    const int rc = hc_phmm_init(0, device);   // device selection + gfx950 check (no-op once initialised)
    if (rc != HC_PHMM_OK) return rc;
    HIP_TRY(hipSetDevice(hcphmm::primary_device()));
    if (!g_stream) HIP_TRY(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking));
    return HC_SW_OK;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// The DP kernel's fast variant drops the MATRIX_MIN_CUTOFF max and reads its
// backtrack bits as signs of differences. Both are exact when every H stays
// at or above the cutoff and every difference fits in int32. Along any
// diagonal chain H(i,j) >= boundary + min(i,j) * min(0, match, mismatch), and
// |H| <= |boundary| + max(n1,n2) * max|score|; E and F stay within one gap
// score of H, or sit at LOW_INIT_VALUE (+ one extension) on the borders.
bool fast_ok(const hc_sw_params& p, int overhang, int n1max, int n2max)
{
    const int64_t M = std::max(n1max, n2max);
    const int64_t mt = p.match, mm = p.mismatch, op = p.open, ex = p.extend;
    int64_t bmin = 0, bmax = 0;
    if (overhang == HC_SW_INDEL || overhang == HC_SW_LEADING_INDEL) {
        bmin = std::min({int64_t(0), op, op + (M - 1) * ex});
        bmax = std::max({int64_t(0), op, op + (M - 1) * ex});
    }
    const int64_t hlow = bmin + M * std::min({int64_t(0), mt, mm});
    const int64_t hhigh = bmax + M * std::max({int64_t(0), mt, mm});
    if (hlow < kMinCutoff) return false;
    const int64_t v = std::max(-hlow, hhigh) + std::abs(op) + M * std::abs(ex) + std::abs(mt) + std::abs(mm);
    return v < (int64_t(1) << 28);
}

// IntelSWAligner::is_all_match (intel_smithwaterman.hpp:47-58): equal lengths
// and at most MINIMAL_MISMATCH_TO_TOLERANCE = 2 mismatching bytes.
bool all_match(const uint8_t* ref, const uint8_t* alt, int n1, int n2)
{
    if (n1 != n2) return false;
    int mm = 0;
    for (int i = 0; mm <= 2 && i < n1; ++i) mm += ref[i] != alt[i];
    return mm <= 2;
}

}  // namespace

struct hc_sw_batch {
    int64_t n = 0;                  // caller's pairs
    int64_t nd = 0;                 // pairs on the device (the rest: host all-match shortcut)
    std::vector<int64_t> dev_ids;   // caller index of device pair d
    std::vector<std::pair<int64_t, int32_t>> host_sc;   // {caller index, length}: shortcut answered on the host
    int n1max = 0, n2max = 0;
    int64_t cells = 0;
    hc_sw_params params{};
    int overhang = 9, shortcut = 1;
    int fast = 0;
    char* dev = nullptr;
    SwPair* pairs = nullptr;
    int32_t* order = nullptr;
    uint8_t* refs = nullptr;
    uint8_t* alts = nullptr;
    SwResult* res = nullptr;
    uint32_t* bt = nullptr;
    uint32_t* elems = nullptr;
    uint16_t* slots = nullptr;
    int32_t* n_elems = nullptr;
    int32_t* offsets = nullptr;
    int64_t n_el_cap = 0;
    size_t tail_off = 0, tail_bytes = 0;   // [slots | n_elems | offsets], one D2H
    bool owns = true;                      // false: borrows g_ws
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    double dp_ms = 0, trace_ms = 0, run_ms = 0;
    int64_t n_runs = 0;
    bool ran = false;
};

namespace {

void free_batch(hc_sw_batch* b)
{
    if (!b) return;
    if (b->owns) {
        for (auto& e : b->ev)
            if (e) (void)hipEventDestroy(e);
        if (b->dev) (void)hipFree(b->dev);
    }
    delete b;
}

int ws_reserve(size_t dev_bytes, size_t host_bytes)
{
    if (dev_bytes > g_ws.dev_bytes) {
        if (g_ws.dev) (void)hipFree(g_ws.dev);
        g_ws.dev = nullptr;
        g_ws.dev_bytes = 0;
        const size_t want = dev_bytes + dev_bytes / 4;
        if (hipMalloc(&g_ws.dev, want) != hipSuccess) return fail(HC_SW_ENOMEM, "workspace device allocation");
        g_ws.dev_bytes = want;
    }
    if (host_bytes > g_ws.host_bytes) {
        if (g_ws.host) (void)hipHostFree(g_ws.host);
        g_ws.host = nullptr;
        g_ws.host_bytes = 0;
        const size_t want = host_bytes + host_bytes / 4;
        if (hipHostMalloc(&g_ws.host, want, hipHostMallocDefault) != hipSuccess)
            return fail(HC_SW_ENOMEM, "workspace pinned allocation");
        g_ws.host_bytes = want;
    }
    for (auto& e : g_ws.ev)
        if (!e) HIP_TRY(hipEventCreate(&e));
    return HC_SW_OK;
}

int create(int64_t n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
           const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts, hc_sw_params params,
           int32_t overhang, int32_t shortcut, hc_sw_batch** out, bool transient = false)
{
    if (!out || n < 0) return fail(HC_SW_EINVAL, "null output / negative count");
    if (overhang < HC_SW_SOFTCLIP || overhang > HC_SW_IGNORE) return fail(HC_SW_EINVAL, "bad overhang strategy");
    if (n > 0 && (!ref_off || !ref_len || !refs || !alt_off || !alt_len || !alts))
        return fail(HC_SW_EINVAL, "null input array");
    if (n > INT32_MAX / 2) return fail(HC_SW_EINVAL, "too many pairs");
    auto* b = new (std::nothrow) hc_sw_batch;
    if (!b) return fail(HC_SW_ENOMEM, "host allocation");
    b->n = n;
    b->params = params;
    b->overhang = overhang;
    b->shortcut = shortcut ? 1 : 0;

    std::vector<SwPair> pairs;
    pairs.reserve(static_cast<size_t>(n));
    int64_t ref_ext = 0, alt_ext = 0, bt_total = 0, el_total = 0;
    for (int64_t k = 0; k < n; ++k) {
        const int n1 = ref_len[k], n2 = alt_len[k];
        const bool in_range = n1 >= 1 && n2 >= 1 && n1 <= HC_SW_MAX_LEN1 && n2 <= HC_SW_MAX_LEN2;
        if (n1 >= 1 && n2 >= 1 && ref_off[k] >= 0 && alt_off[k] >= 0 && !in_range && shortcut &&
            all_match(refs + ref_off[k], alts + alt_off[k], n1, n2)) {
            // IntelSWAligner::align answers an equal-length pair with <= 2
            // mismatches before runSWOnePairBT_avx2 sees it (intel_smithwaterman.hpp:
            // 36-37), so the aligner's length limit does not apply to it.
            b->host_sc.emplace_back(k, n1);
            continue;
        }
        if (!in_range || ref_off[k] < 0 || alt_off[k] < 0) {
            free_batch(b);
            return fail(HC_SW_EINVAL, "pair " + std::to_string(k) + ": sequence length out of range [1, " +
                                          std::to_string(HC_SW_MAX_LEN1) + "] x [1, " +
                                          std::to_string(HC_SW_MAX_LEN2) + "] or negative offset");
        }
        SwPair P;
        P.ref_off = ref_off[k];
        P.alt_off = alt_off[k];
        P.n1 = n1;
        P.n2 = n2;
        P.el_off = el_total;
        el_total += n1 + n2 + 3;
        ref_ext = std::max(ref_ext, ref_off[k] + n1);
        alt_ext = std::max(alt_ext, alt_off[k] + n2);
        b->n1max = std::max(b->n1max, n1);
        b->n2max = std::max(b->n2max, n2);
        b->cells += int64_t(n1) * n2;
        pairs.push_back(P);
        b->dev_ids.push_back(k);
    }
    n = int64_t(pairs.size());
    b->nd = n;
    // Longest pairs first: the tail of the launch is made of short waves.
    std::vector<int32_t> order(static_cast<size_t>(n));
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) {
        return int64_t(pairs[x].n1) * pairs[x].n2 > int64_t(pairs[y].n1) * pairs[y].n2;
    });
    b->n_el_cap = el_total;
    b->fast = fast_ok(params, overhang, b->n1max, b->n2max) ? 1 : 0;
    if (const char* e = std::getenv("HC_SW_GENERIC"))   // parity tests of the generic variant
        if (e[0] == '1') b->fast = 0;
    // (An LDS substitution profile and a spiral layout of the fast path were
    // measured slower — W2 DP 10.8 / 9.33 vs 8.72 ms — and removed, round 6.)
    for (auto& P : pairs) {
        P.bt_off = bt_total;
        bt_total += bt_words(P.n1, P.n2);
    }

    // One device allocation: descriptors, inputs, outputs, scratch.
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        const size_t at = off;
        off = align_up(off + std::max<size_t>(bytes, 1), 256);
        return at;
    };
    const size_t o_pairs = carve(sizeof(SwPair) * size_t(n));
    const size_t o_order = carve(sizeof(int32_t) * size_t(n));
    const size_t o_refs = carve(size_t(ref_ext));
    const size_t o_alts = carve(size_t(alt_ext));
    const size_t in_bytes = off;
    const size_t o_res = carve(sizeof(SwResult) * size_t(n));
    const size_t o_bt = carve(sizeof(uint32_t) * size_t(bt_total));
    const size_t o_el = carve(sizeof(uint32_t) * size_t(el_total));
    const size_t o_slots = carve(sizeof(uint16_t) * kSlotElems * size_t(n));
    const size_t o_nel = carve(sizeof(int32_t) * size_t(n));
    const size_t o_offs = carve(sizeof(int32_t) * size_t(n));
    b->tail_off = o_slots;
    b->tail_bytes = off - o_slots;
    char* stage_mem = nullptr;
    std::vector<char> stage_vec;
    if (transient) {
        const int rc = ws_reserve(off, std::max(in_bytes, b->tail_bytes));
        if (rc) {
            free_batch(b);
            return rc;
        }
        b->owns = false;
        b->dev = g_ws.dev;
        for (int k = 0; k < 3; ++k) b->ev[k] = g_ws.ev[k];
        stage_mem = g_ws.host;
    } else {
        if (hipMalloc(&b->dev, off) != hipSuccess) {
            free_batch(b);
            return fail(HC_SW_ENOMEM, "device allocation of " + std::to_string(off) + " bytes");
        }
        for (auto& e : b->ev) {
            if (hipEventCreate(&e) != hipSuccess) {
                free_batch(b);
                return fail(HC_SW_EHIP, "hipEventCreate");
            }
        }
        stage_vec.resize(in_bytes);
        stage_mem = stage_vec.data();
    }
    b->pairs = reinterpret_cast<SwPair*>(b->dev + o_pairs);
    b->order = reinterpret_cast<int32_t*>(b->dev + o_order);
    b->refs = reinterpret_cast<uint8_t*>(b->dev + o_refs);
    b->alts = reinterpret_cast<uint8_t*>(b->dev + o_alts);
    b->res = reinterpret_cast<SwResult*>(b->dev + o_res);
    b->bt = reinterpret_cast<uint32_t*>(b->dev + o_bt);
    b->elems = reinterpret_cast<uint32_t*>(b->dev + o_el);
    b->slots = reinterpret_cast<uint16_t*>(b->dev + o_slots);
    b->n_elems = reinterpret_cast<int32_t*>(b->dev + o_nel);
    b->offsets = reinterpret_cast<int32_t*>(b->dev + o_offs);

    // Stage the inputs in one host block, one H2D.
    char* stage = stage_mem;
    std::memcpy(stage + o_pairs, pairs.data(), sizeof(SwPair) * size_t(n));
    std::memcpy(stage + o_order, order.data(), sizeof(int32_t) * size_t(n));
    if (ref_ext) std::memcpy(stage + o_refs, refs, size_t(ref_ext));
    if (alt_ext) std::memcpy(stage + o_alts, alts, size_t(alt_ext));
    if (hipMemcpyAsync(b->dev, stage, in_bytes, hipMemcpyHostToDevice, g_stream) != hipSuccess ||
        (!transient && hipStreamSynchronize(g_stream) != hipSuccess)) {
        free_batch(b);
        return fail(HC_SW_EHIP, "H2D of the batch inputs");
    }
    *out = b;
    return HC_SW_OK;
}

int run(hc_sw_batch* b, hipStream_t s)
{
    if (b->nd == 0) {
        b->ran = true;
        return HC_SW_OK;
    }
    SwDpArgs d{};
    d.pairs = b->pairs;
    d.order = b->order;
    d.n = int(b->nd);
    d.refs = b->refs;
    d.alts = b->alts;
    d.bt = b->bt;
    d.res = b->res;
    d.elems = b->elems;
    d.match = b->params.match;
    d.mismatch = b->params.mismatch;
    d.open = b->params.open;
    d.extend = b->params.extend;
    d.overhang = b->overhang;
    d.shortcut = b->shortcut;
    d.n1max = b->n1max;
    d.n2max = b->n2max;
    d.fast = b->fast;
    // Pairs per workgroup: one for region-sized windows (W2, n2 <= ~650: 8.62 /
    // 9.09 / 9.20 ms at 1 / 2 / 4), four for long ones (W3, n2 ~ 1000: 3.54 /
    // 3.25 / 2.90 ms); HC_SW_WPG overrides.
    d.wpg = b->n2max > 800 ? 4 : 1;
    if (const char* e = std::getenv("HC_SW_WPG"))
        if (std::atoi(e) > 0) d.wpg = std::atoi(e);
    SwTraceArgs t{};
    t.pairs = b->pairs;
    t.res = b->res;
    t.bt = b->bt;
    t.n = int(b->nd);
    t.overhang = b->overhang;
    t.elems = b->elems;
    t.slots = b->slots;
    t.n_elems = b->n_elems;
    t.offsets = b->offsets;
    HIP_TRY(hipEventRecord(b->ev[0], s));
    HIP_TRY(launch_dp(d, b->n1max, s));
    HIP_TRY(hipEventRecord(b->ev[1], s));
    HIP_TRY(launch_trace(t, s));
    HIP_TRY(hipEventRecord(b->ev[2], s));
    HIP_TRY(hipEventSynchronize(b->ev[2]));
    float a = 0, c = 0, w = 0;
    HIP_TRY(hipEventElapsedTime(&a, b->ev[0], b->ev[1]));
    HIP_TRY(hipEventElapsedTime(&c, b->ev[1], b->ev[2]));
    HIP_TRY(hipEventElapsedTime(&w, b->ev[0], b->ev[2]));
    b->dp_ms += a;
    b->trace_ms += c;
    b->run_ms += w;
    ++b->n_runs;
    b->ran = true;
    return HC_SW_OK;
}

int results(hc_sw_batch* b, int32_t* offsets, char* cigars, int32_t stride, int32_t* scores)
{
    if (!b->ran) return fail(HC_SW_EINVAL, "batch has not run");
    if (b->n == 0) return HC_SW_OK;
    if (!offsets || !cigars || stride < 2) return fail(HC_SW_EINVAL, "null output / stride < 2");
    bool too_long = false;
    // Over-length pairs the all-match shortcut answered on the host: {0, <n>M}
    // (intel_smithwaterman.hpp:36-37).
    for (const auto& [k, len] : b->host_sc) {
        char* o = cigars + size_t(k) * size_t(stride);
        offsets[k] = 0;
        if (scores) scores[k] = 0;
        const int w = std::snprintf(o, size_t(stride), "%dM", len);
        if (w < 0 || w >= stride) {
            too_long = true;
            o[0] = 0;
        }
    }
    const int64_t n = b->nd;   // device pairs; caller index b->dev_ids[k]
    if (n > 0) {
        // [slots | n_elems | offsets] are contiguous on the device: one D2H.
        std::vector<char> tail_vec;
        char* tail = nullptr;
        if (!b->owns && g_ws.host_bytes >= b->tail_bytes) {
            tail = g_ws.host;
        } else {
            tail_vec.resize(b->tail_bytes);
            tail = tail_vec.data();
        }
        HIP_TRY(hipMemcpy(tail, b->dev + b->tail_off, b->tail_bytes, hipMemcpyDeviceToHost));
        const uint16_t* slotv = reinterpret_cast<const uint16_t*>(tail);
        const int32_t* cntv = reinterpret_cast<const int32_t*>(tail + (reinterpret_cast<char*>(b->n_elems) - (b->dev + b->tail_off)));
        const int32_t* offv = reinterpret_cast<const int32_t*>(tail + (reinterpret_cast<char*>(b->offsets) - (b->dev + b->tail_off)));
        for (int64_t k = 0; k < n; ++k) offsets[b->dev_ids[size_t(k)]] = offv[k];
        std::vector<int32_t> cnt(cntv, cntv + n);
        // Pairs with more than kSlotElems elements: their whole scratch (rare).
        std::vector<uint32_t> big;
        std::vector<size_t> big_at(static_cast<size_t>(n), SIZE_MAX);
        std::vector<SwPair> P;
        for (int64_t k = 0; k < n; ++k) {
            if (cnt[size_t(k)] <= kSlotElems) continue;
            if (P.empty()) {
                P.resize(size_t(n));
                HIP_TRY(hipMemcpy(P.data(), b->pairs, sizeof(SwPair) * size_t(n), hipMemcpyDeviceToHost));
            }
            big_at[size_t(k)] = big.size();
            big.resize(big.size() + size_t(cnt[size_t(k)]));
            HIP_TRY(hipMemcpy(big.data() + big_at[size_t(k)], b->elems + P[size_t(k)].el_off,
                              sizeof(uint32_t) * size_t(cnt[size_t(k)]), hipMemcpyDeviceToHost));
        }
        if (scores) {
            std::vector<SwResult> r(static_cast<size_t>(n));
            HIP_TRY(hipMemcpy(r.data(), b->res, sizeof(SwResult) * size_t(n), hipMemcpyDeviceToHost));
            for (int64_t k = 0; k < n; ++k) scores[b->dev_ids[size_t(k)]] = r[size_t(k)].score;
        }
        for (int64_t k = 0; k < n; ++k) {
            char* o = cigars + size_t(b->dev_ids[size_t(k)]) * size_t(stride);
            int pos = 0;
            // Elements are in traceback order: print them back to front (:388-413).
            for (int e = cnt[size_t(k)] - 1; e >= 0 && pos >= 0; --e) {
                const uint32_t v = cnt[size_t(k)] <= kSlotElems ? uint32_t(slotv[size_t(k) * kSlotElems + size_t(e)])
                                                                 : big[big_at[size_t(k)] + size_t(e)];
                const int op = int(v & 15);
                const char ch = op == kOpM ? 'M' : op == kOpI ? 'I' : op == kOpD ? 'D' : op == kOpS ? 'S' : 'R';
                const int w = std::snprintf(o + pos, size_t(stride - pos), "%u%c", v >> 4, ch);
                pos = (w < 0 || pos + w >= stride) ? -1 : pos + w;
            }
            if (pos < 0) {
                too_long = true;
                o[0] = 0;
            } else if (cnt[size_t(k)] == 0) {
                o[0] = 0;
            }
        }
    }
    if (too_long) return fail(HC_SW_ERANGE, "a CIGAR does not fit in the stride");
    return HC_SW_OK;
}

}  // namespace

extern "C" {

int hc_sw_init(int device)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return ensure_init(device);
}

int hc_sw_batch_create(int64_t n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
                       const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts, hc_sw_params params,
                       int32_t overhang, int32_t shortcut, hc_sw_batch** out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    const int rc = ensure_init(-1);
    if (rc) return rc;
    return create(n, ref_off, ref_len, refs, alt_off, alt_len, alts, params, overhang, shortcut, out);
}

int hc_sw_batch_run(hc_sw_batch* b, void* stream)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!b) return fail(HC_SW_EINVAL, "null batch");
    const int rc = ensure_init(-1);
    if (rc) return rc;
    return run(b, stream ? static_cast<hipStream_t>(stream) : g_stream);
}

int hc_sw_batch_results(hc_sw_batch* b, int32_t* offsets, char* cigars, int32_t stride, int32_t* scores)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!b) return fail(HC_SW_EINVAL, "null batch");
    const int rc = ensure_init(-1);
    if (rc) return rc;
    return results(b, offsets, cigars, stride, scores);
}

int hc_sw_batch_stats(hc_sw_batch* b, hc_sw_stats* st)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!b || !st) return fail(HC_SW_EINVAL, "null batch / stats");
    const int rc = ensure_init(-1);
    if (rc) return rc;
    st->n_pairs = b->n;
    st->cells = b->cells;
    st->n_shortcut = int64_t(b->host_sc.size());
    if (b->ran && b->nd) {
        const size_t nd = size_t(b->nd);
        std::vector<SwResult> r(nd);
        HIP_TRY(hipMemcpy(r.data(), b->res, sizeof(SwResult) * nd, hipMemcpyDeviceToHost));
        std::vector<SwPair> P(nd);
        HIP_TRY(hipMemcpy(P.data(), b->pairs, sizeof(SwPair) * nd, hipMemcpyDeviceToHost));
        st->cells = 0;
        for (size_t k = 0; k < nd; ++k) {
            if (r[k].shortcut) ++st->n_shortcut;
            else st->cells += int64_t(P[k].n1) * P[k].n2;
        }
    }
    const double k = b->n_runs ? 1.0 / double(b->n_runs) : 0.0;
    st->dp_ms = b->dp_ms * k;
    st->trace_ms = b->trace_ms * k;
    st->run_ms = b->run_ms * k;
    st->n_runs = b->n_runs;
    b->dp_ms = b->trace_ms = b->run_ms = 0;
    b->n_runs = 0;
    return HC_SW_OK;
}

int hc_sw_batch_destroy(hc_sw_batch* b)
{
    std::lock_guard<std::mutex> lk(g_mu);
    free_batch(b);
    return HC_SW_OK;
}

int hc_sw_align_flat(int64_t n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
                     const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts, hc_sw_params params,
                     int32_t overhang, int32_t shortcut, int32_t* offsets, char* cigars, int32_t stride)
{
    std::lock_guard<std::mutex> lk(g_mu);
    int rc = ensure_init(-1);
    if (rc) return rc;
    hc_sw_batch* b = nullptr;
    rc = create(n, ref_off, ref_len, refs, alt_off, alt_len, alts, params, overhang, shortcut, &b, true);
    if (rc) return rc;
    rc = run(b, g_stream);
    if (!rc) rc = results(b, offsets, cigars, stride, nullptr);
    free_batch(b);
    return rc;
}

}  // extern "C"

// Called by hc_phmm_shutdown: the next call re-creates the stream and workspace
// on whatever device the engine is then initialised on.
void hcphmm::sw_release()
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_stream) return;
    (void)hipStreamSynchronize(g_stream);
    if (g_ws.dev) (void)hipFree(g_ws.dev);
    if (g_ws.host) (void)hipHostFree(g_ws.host);
    for (auto& e : g_ws.ev)
        if (e) (void)hipEventDestroy(e);
    g_ws = Workspace{};
    (void)hipStreamDestroy(g_stream);
    g_stream = nullptr;
}
