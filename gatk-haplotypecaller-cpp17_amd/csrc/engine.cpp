// Host engine + C ABI of libhcpairhmm.so (include/hc_pairhmm.h).
//
// Flow of one batch (the reference's computeLikelihoodsNative,
// intel_pairhmm.hpp:115-152, split into plan and execute):
//   plan     pack reads into 32-bit row words and haps into match tables,
//            length-bin the pairs (W class by H, then stripes, then H), H2D
//   execute  fp32 anti-diagonal kernel per W class -> raw f32 + rescue list
//            fp64 kernel over the rescue list (raw < 1e-28f)      [device only]
//   finish   D2H, then glibc log10f/log10 exactly as intel_pairhmm.hpp:137-143
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hc_pairhmm.h"
#include "kernels.hpp"
#include "luts.hpp"

using namespace hcphmm;

namespace {

thread_local std::string g_err;
std::mutex g_mu;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(HC_PHMM_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Engine {
    bool ready = false;
    int device = -1;
    int n_cu = 256;   // compute units (4 SIMDs each): sizes the lane-wave latency ceiling
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;                  // segmented lane waves run here, concurrently
    hipEvent_t fork = nullptr, join = nullptr;   // side-stream fork / join (timing disabled)
    float* lut_f = nullptr;
    double* lut_d = nullptr;
};
Engine g_eng;

// ConvertChar (pairhmm_common.h:26-44).
inline int base_code(uint8_t b)
{
    switch (b) {
    case 'C': return 1;
    case 'T': return 2;
    case 'G': return 3;
    case 'N': return 4;
    default: return 0;
    }
}

int ensure_init(int device)
{
    if (g_eng.ready) return HC_PHMM_OK;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(HC_PHMM_ENODEV, "no HIP device visible");
    int dev = device;
    if (dev < 0) HIP_TRY(hipGetDevice(&dev));
    if (dev >= n) return fail(HC_PHMM_ENODEV, "device ordinal out of range");
    HIP_TRY(hipSetDevice(dev));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(HC_PHMM_ENODEV, std::string("device is ") + prop.gcnArchName + ", need gfx950");
    HIP_TRY(configure_kernels());
    g_eng.n_cu = std::max(1, prop.multiProcessorCount);
    HIP_TRY(hipStreamCreateWithFlags(&g_eng.stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&g_eng.side, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&g_eng.fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&g_eng.join, hipEventDisableTiming));
    const Luts& L = luts();
    HIP_TRY(hipMalloc(&g_eng.lut_f, sizeof(float) * kTableLen));
    HIP_TRY(hipMalloc(&g_eng.lut_d, sizeof(double) * kTableLen));
    HIP_TRY(hipMemcpy(g_eng.lut_f, L.dev_f.data(), sizeof(float) * kTableLen, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(g_eng.lut_d, L.dev_d.data(), sizeof(double) * kTableLen, hipMemcpyHostToDevice));
    g_eng.device = dev;
    g_eng.ready = true;
    return HC_PHMM_OK;
}

template <typename F>
void parallel_for(int64_t n, F&& f, int64_t grain = 4096)
{
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int64_t nt = std::min<int64_t>(std::min<int64_t>(hw, 16), (n + grain - 1) / grain);
    if (nt <= 1) {
        f(int64_t(0), n);
        return;
    }
    std::vector<std::thread> th;
    const int64_t chunk = (n + nt - 1) / nt;
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t b = t * chunk, e = std::min(n, b + chunk);
        if (b < e) th.emplace_back([&, b, e] { f(b, e); });
    }
    for (auto& x : th) x.join();
}

struct ReadView {
    int32_t len;
    const uint8_t *bases, *q, *i, *d, *c;
};
struct HapView {
    int32_t len;
    const uint8_t* bases;
};

}  // namespace

// --------------------------------------------------------------------------
// Prepared batch: every device array of one batch lives in one allocation,
// filled by one H2D copy from one pinned staging buffer.
struct hc_phmm_batch {
    int64_t n = 0;          // pairs
    int64_t cells = 0;
    int Hmax = 0;
    struct Cls {
        int W = 16;
        int n = 0;
        int ring_len = 0;
        int* d_order = nullptr;
    } cls[2];
    // Lane-per-pair class (large batches).
    int n_lane = 0;
    int n_seg_waves = 0;
    int lane_waves = 0;
    int lane_variant = 0;   // lane kernel variant (kernels.hpp LaneVariant)
    int* d_lane_order = nullptr;
    LaneWave* d_lane_waves = nullptr;
    float2* d_carry = nullptr;
    PairDesc* d_pairs = nullptr;
    uint32_t* d_rows = nullptr;
    uint32_t* d_hapw = nullptr;
    float* d_raw32 = nullptr;     // current output targets (own or bound)
    double* d_raw64 = nullptr;
    uint8_t* d_flag = nullptr;
    float* own_raw32 = nullptr;   // library-owned output buffers
    double* own_raw64 = nullptr;
    uint8_t* own_flag = nullptr;
    int* d_list = nullptr;
    int* d_sorted = nullptr;      // fp64 pass: rescue list in class order (device-planned)
    int* d_big = nullptr;         // fp64 pass: pairs too wide for the segmented kernel
    int* d_big_count = nullptr;
    Seg64Plan* d_plan = nullptr;
    int64_t n_wide = 0;           // pairs with H > 64 * 32 (may need the anti-diagonal fp64 kernel)
    int* d_count = nullptr;       // rescue counters, one per run parity
    int parity = 0;               // run parity: which counter this run appends to
    char* dev_base = nullptr;     // the batch's device allocation
    bool owns_dev = true;         // false: borrowed from the engine workspace
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};   // current run's triple (from ev_pool)
    // Event triples of every run since the last stats() call (reused pool), so
    // stats() reports the average kernel time over a whole timed region.
    std::vector<std::array<hipEvent_t, 3>> ev_pool;
    size_t ev_used = 0;
    hipStream_t last_stream = nullptr;
    int64_t launch_waves = 0;
    bool ran = false;
};

namespace {

constexpr int kW64Threshold = 768;   // H above this -> one pair per wave (W = 64)
constexpr int kLaneMaxH = 4096;            // longer haps stay on the anti-diagonal kernel
constexpr int kSegWavesPerSimd = 3;        // resident seg waves per SIMD (phmm_seg_kernel occupancy)
constexpr int kSegMinWavesPerSimd = 2;     // small batches: narrower seg blocks until this many waves

// Lane kernel variant (kernels.hpp LaneVariant): HC_PHMM_LANE_VARIANT=<id>,
// default 0 = {1 pair per lane, 64-column blocks, 3 waves per SIMD}.
int lane_variant_id()
{
    const char* e = std::getenv("HC_PHMM_LANE_VARIANT");
    return (e && *e) ? std::atoi(e) : 0;
}

// Column-segmented lane waves (lane_kernel.hip run_seg): HC_PHMM_LANE_SEG=
// auto = all (default: every lane pair up to 64 * kSegMaxBC columns) | off
// (one lane per pair with the carry buffer). Returns -1 auto, 0 off, 1 all.
int lane_seg_policy()
{
    const char* e = std::getenv("HC_PHMM_LANE_SEG");
    if (!e || !*e || !std::strcmp(e, "auto")) return -1;
    return std::strcmp(e, "all") ? 0 : 1;
}

// Kernel selection: HC_PHMM_KERNEL=auto (default: lane kernels for H <= kLaneMaxH,
// anti-diagonal above) | lane (lane kernels for every pair) | diag.
int kernel_policy()
{
    const char* e = std::getenv("HC_PHMM_KERNEL");
    if (!e || !*e || !std::strcmp(e, "auto")) return 0;
    if (!std::strcmp(e, "lane")) return 1;
    return 2;
}

// HC_PHMM_TRACE=1: per-phase host timings of plan/results on stderr.
struct PhaseTimer {
    bool on;
    std::chrono::steady_clock::time_point t0;
    PhaseTimer() : on(std::getenv("HC_PHMM_TRACE") != nullptr), t0(std::chrono::steady_clock::now()) {}
    void mark(const char* what)
    {
        if (!on) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[hc_phmm] %-18s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    }
};

// Grow-only buffers reused by the synchronous entry points (no per-call
// hipMalloc / hipHostMalloc once warm).
struct Workspace {
    char* dev = nullptr;
    size_t dev_cap = 0;
    char* host = nullptr;   // pinned
    size_t host_cap = 0;
    hc_phmm_batch* batch = nullptr;   // batch shell reused for its event pool
};
Workspace g_ws;

int ws_dev(size_t bytes, char** out)
{
    if (bytes > g_ws.dev_cap) {
        if (g_ws.dev) HIP_TRY(hipFree(g_ws.dev));
        g_ws.dev = nullptr;
        g_ws.dev_cap = 0;
        const size_t cap = std::max(bytes + bytes / 4, size_t(64) << 20);
        if (hipMalloc(&g_ws.dev, cap) != hipSuccess) return fail(HC_PHMM_ENOMEM, "device workspace");
        g_ws.dev_cap = cap;
    }
    *out = g_ws.dev;
    return HC_PHMM_OK;
}

int ws_host(size_t bytes, char** out)
{
    if (bytes > g_ws.host_cap) {
        if (g_ws.host) HIP_TRY(hipHostFree(g_ws.host));
        g_ws.host = nullptr;
        g_ws.host_cap = 0;
        const size_t cap = std::max(bytes + bytes / 4, size_t(16) << 20);
        if (hipHostMalloc(&g_ws.host, cap, hipHostMallocDefault) != hipSuccess)
            return fail(HC_PHMM_ENOMEM, "pinned staging buffer");
        g_ws.host_cap = cap;
    }
    *out = g_ws.host;
    return HC_PHMM_OK;
}

void release_batch_memory(hc_phmm_batch* b)
{
    if (b->owns_dev) (void)hipFree(b->dev_base);
    b->dev_base = nullptr;
}

void free_batch(hc_phmm_batch* b)
{
    if (!b) return;
    release_batch_memory(b);
    for (auto& t : b->ev_pool)
        for (auto& e : t) (void)hipEventDestroy(e);
    delete b;
}

// LSD radix sort of `idx` by a 32-bit key, DESCENDING, stable: the keys are
// gathered once next to the indices ((~key << 32) | index, sorted ascending on
// the high word), so every pass streams one contiguous array; 11-bit digits
// (cache-resident counters), passes above the largest key's top bit skipped.
void sort_desc(std::vector<int>& idx, const std::vector<uint32_t>& key)
{
    if (idx.size() < 2) return;
    uint32_t kmax = 0;
    for (int p : idx) kmax = std::max(kmax, key[p]);
    const size_t n = idx.size();
    std::vector<uint64_t> v(n), tmp(n);
    for (size_t k = 0; k < n; ++k) v[k] = (uint64_t(kmax - key[idx[k]]) << 32) | uint32_t(idx[k]);
    constexpr int kBits = 11, kBuckets = 1 << kBits;
    for (int shift = 0; shift < 32 && (kmax >> shift) != 0; shift += kBits) {
        size_t cnt[kBuckets + 1] = {};
        for (uint64_t x : v) ++cnt[((x >> (32 + shift)) & (kBuckets - 1)) + 1];
        for (int k = 1; k <= kBuckets; ++k) cnt[k] += cnt[k - 1];
        for (uint64_t x : v) tmp[cnt[(x >> (32 + shift)) & (kBuckets - 1)]++] = x;
        v.swap(tmp);
    }
    for (size_t k = 0; k < n; ++k) idx[k] = int(uint32_t(v[k]));
}

// Bump allocator over one device region: 256-B aligned segments.
struct Layout {
    size_t off = 0;
    size_t take(size_t bytes)
    {
        const size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    }
};

// Pack reads/haps once each, pairs refer to them (cross product reuses both).
// borrow_ws: place the device arrays in the engine workspace (synchronous
// calls) instead of a batch-owned allocation.
int plan(const std::vector<ReadView>& reads, const std::vector<HapView>& haps,
         int64_t npairs, const int32_t* pr, const int32_t* ph, bool borrow_ws,
         hc_phmm_batch** out)
{
    for (const auto& r : reads)
        if (r.len <= 0 || r.len > HC_PHMM_MAX_READ_LEN || !r.bases || !r.q || !r.i || !r.d || !r.c)
            return fail(HC_PHMM_EINVAL, "read with invalid length or null array");
    for (const auto& h : haps)
        if (h.len <= 0 || h.len > HC_PHMM_MAX_HAP_LEN || !h.bases)
            return fail(HC_PHMM_EINVAL, "haplotype with invalid length (1.." +
                                            std::to_string(HC_PHMM_MAX_HAP_LEN) + ") or null bases");
    if (npairs > (int64_t(1) << 31) - 1) return fail(HC_PHMM_EINVAL, "too many pairs for one batch");

    PhaseTimer tm;
    const int64_t nr = reads.size(), nh = haps.size();
    std::vector<int64_t> row_off(nr + 1, 0), hap_off(nh + 1, 0);
    for (int64_t r = 0; r < nr; ++r) row_off[r + 1] = row_off[r] + reads[r].len;
    for (int64_t h = 0; h < nh; ++h) hap_off[h + 1] = hap_off[h] + hap_table_words(haps[h].len);
    if (row_off[nr] > INT32_MAX || hap_off[nh] > INT32_MAX)
        return fail(HC_PHMM_EINVAL, "batch too large (row or hap pool exceeds 2^31 words)");

    tm.mark("offsets");
    // Descriptors and length binning.
    std::vector<PairDesc> pd(npairs);
    int64_t cells = 0;
    int Hmax = 0;
    int64_t n_wide = 0;
    {
        std::mutex mu;
        parallel_for(npairs, [&](int64_t lo, int64_t hi) {
            int64_t c = 0, w = 0;
            int hm = 0;
            for (int64_t p = lo; p < hi; ++p) {
                const int r = pr[p], h = ph[p];
                pd[p] = PairDesc{int(row_off[r]), reads[r].len, int(hap_off[h]), haps[h].len};
                c += int64_t(reads[r].len) * haps[h].len;
                hm = std::max(hm, haps[h].len);
                w += haps[h].len > 64 * 32;
            }
            std::lock_guard<std::mutex> lk(mu);
            cells += c;
            Hmax = std::max(Hmax, hm);
            n_wide += w;
        }, 1 << 16);
    }
    tm.mark("bin: descriptors");
    std::vector<int> ord[2], lane_ord;
    lane_ord.reserve(npairs);
    const int pol = kernel_policy();
    const bool use_lane = pol != 2;
    for (int64_t p = 0; p < npairs; ++p) {
        if (use_lane && (pol == 1 || pd[p].w <= kLaneMaxH))
            lane_ord.push_back(int(p));
        else
            ord[pd[p].w > kW64Threshold ? 1 : 0].push_back(int(p));
    }
    std::vector<uint32_t> key(npairs);
    // Lane class. Column-segmented waves (lane_kernel.hip run_seg) take every
    // lane pair with H <= 64 * kSegMaxBC (policy "off": none): a pair gets nb
    // lanes of BC columns, BC from the compiled widths, choosing between
    // nb0 = ceil(H/cap) and nb0 + 1 lanes by modelled cost nb*BC*(R + nb - 1).
    // The width cap is 64 unless the batch is too small to give every SIMD
    // kSegMinWavesPerSimd waves at that width (a lone wave issues at half
    // rate): then the widest cap that does, down to 16, so small batches are
    // spread over more, shorter waves. Pairs are binned by (BC, R) descending
    // and packed greedily into waves of up to 64 lanes (a short look-ahead
    // fills a wave's last lanes). Longer haps (or policy "off") take one lane
    // per pair with the carry buffer, binned by (H rounded up to 16, R).
    std::vector<LaneWave> lw;
    int64_t carry_rows = 0;
    const int lane_var = lane_variant_id();
    const LaneVariant& LV = lane_variant(lane_var);
    const int lane_p = LV.P;
    const int seg_max_h = lane_seg_policy() == 0 ? 0 : 64 * kSegMaxBC;
    std::vector<int> seg_in, one_ord;
    std::vector<uint8_t> seg_bc(npairs, 0), seg_nb(npairs, 0);
    for (int p : lane_ord) (pd[p].w > seg_max_h ? one_ord : seg_in).push_back(p);
    auto choose = [&](int p, int cap) {
        const int H = pd[p].w, R = pd[p].y;
        const int nb0 = std::min(64, (H + cap - 1) / cap);
        int64_t best = INT64_MAX;
        for (int nb = nb0; nb <= std::min(nb0 + 1, 64); ++nb) {
            int bc = std::max(16, ((H + nb - 1) / nb + 3) / 4 * 4);
            while (!seg_width_ok(bc)) bc += 4;
            const int n = (H + bc - 1) / bc;
            const int64_t cost = int64_t(n) * bc * (R + n - 1);
            if (cost < best) {
                best = cost;
                seg_bc[p] = uint8_t(bc);
                seg_nb[p] = uint8_t(n);
            }
        }
    };
    int cap = kSegMaxBC;
    {
        const int64_t want = int64_t(kSegMinWavesPerSimd) * 4 * g_eng.n_cu * 64;   // lanes
        const char* e = std::getenv("HC_PHMM_SEG_CAP");
        if (e && *e) {
            cap = std::max(16, std::min(kSegMaxBC, std::atoi(e)));
        } else {
            constexpr int kCaps[5] = {64, 48, 32, 24, 16};
            int64_t lanes[5] = {};
            std::mutex mu;
            parallel_for(int64_t(seg_in.size()), [&](int64_t lo, int64_t hi) {
                int64_t part[5] = {};
                for (int64_t k = lo; k < hi; ++k) {
                    const int w = pd[seg_in[k]].w;
                    for (int c = 0; c < 5; ++c) part[c] += std::min(64, (w + kCaps[c] - 1) / kCaps[c]);
                }
                std::lock_guard<std::mutex> lk(mu);
                for (int c = 0; c < 5; ++c) lanes[c] += part[c];
            }, 1 << 16);
            for (int c = 0; c < 5; ++c) {
                cap = kCaps[c];
                if (lanes[c] >= want) break;
            }
        }
    }
    tm.mark("bin: classify + cap");
    parallel_for(int64_t(seg_in.size()), [&](int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; ++k) {
            const int p = seg_in[k];
            choose(p, cap);
            key[p] = (uint32_t(seg_bc[p]) << 16) | uint32_t(std::min(pd[p].y, 65535));
        }
    }, 1 << 15);
    tm.mark("bin: choose");
    sort_desc(seg_in, key);
    tm.mark("bin: seg sort");
    std::vector<int> seg_ord;
    seg_ord.reserve(seg_in.size());
    {
        // The packer walks the sorted list; gather what it reads per pair.
        const size_t ns = seg_in.size();
        std::vector<uint8_t> bcs(ns), nbs(ns), used(ns, 0);
        std::vector<int> ys(ns);
        parallel_for(int64_t(ns), [&](int64_t lo, int64_t hi) {
            for (int64_t k = lo; k < hi; ++k) {
                const int p = seg_in[k];
                bcs[k] = seg_bc[p];
                nbs[k] = seg_nb[p];
                ys[k] = pd[p].y;
            }
        }, 1 << 16);
        size_t i = 0;
        constexpr size_t kLook = 64;
        while (i < ns) {
            if (used[i]) {
                ++i;
                continue;
            }
            const int bc = bcs[i];
            LaneWave w{};
            w.slot0 = int(seg_ord.size());
            w.ncols = bc;
            w.rmin = INT32_MAX;
            int free = 64;
            for (size_t j = i; j < ns && j < i + kLook && free > 0; ++j) {
                if (used[j] || bcs[j] != bc) {
                    if (!used[j]) break;
                    continue;
                }
                if (nbs[j] > free) continue;
                used[j] = 1;
                free -= nbs[j];
                seg_ord.push_back(seg_in[j]);
                ++w.npairs;
                w.rmax = std::max(w.rmax, ys[j]);
                w.rmin = std::min(w.rmin, ys[j]);
                w.nsteps = std::max(w.nsteps, ys[j] + nbs[j] - 1);
            }
            lw.push_back(w);
        }
    }
    // Dispatch order. Packing walks pairs by (BC, R), so a short BC=64 wave
    // precedes a long BC=60 one. The bulk keeps that order (co-resident waves
    // share one width's code: measured 2 % faster on S2 than a global sort);
    // the shortest waves filling the last tail_rounds rounds of wave slots go
    // last, longest first (LPT, duration ~ BC * nsteps), so the chip drains
    // evenly. Waves address their pairs through slot0: no pair moves.
    {
        int tail_rounds = 2;
        if (const char* e = std::getenv("HC_PHMM_TAIL_ROUNDS")) tail_rounds = std::max(0, std::atoi(e));   // A/B
        const size_t nw = lw.size();
        const size_t K = std::min(nw, size_t(tail_rounds) * 4 * g_eng.n_cu * kSegWavesPerSimd);
        auto cost = [&](size_t k) { return int64_t(lw[k].ncols) * lw[k].nsteps; };
        std::vector<uint32_t> id(nw);
        for (size_t k = 0; k < nw; ++k) id[k] = uint32_t(k);
        if (K < nw)
            std::nth_element(id.begin(), id.begin() + K, id.end(), [&](uint32_t x, uint32_t y) {
                return cost(x) != cost(y) ? cost(x) < cost(y) : x < y;
            });
        std::vector<uint8_t> in_tail(nw, 0);
        for (size_t k = 0; k < K; ++k) in_tail[id[k]] = 1;
        std::vector<LaneWave> ordered;
        ordered.reserve(nw);
        for (size_t k = 0; k < nw; ++k)
            if (!in_tail[k]) ordered.push_back(lw[k]);
        const size_t t0 = ordered.size();
        for (size_t k = 0; k < nw; ++k)
            if (in_tail[k]) ordered.push_back(lw[k]);
        std::stable_sort(ordered.begin() + t0, ordered.end(), [](const LaneWave& x, const LaneWave& y) {
            return int64_t(x.ncols) * x.nsteps > int64_t(y.ncols) * y.nsteps;
        });
        lw.swap(ordered);
    }
    tm.mark("bin: seg pack");
    const int n_seg_waves = int(lw.size());
    const int n_seg_slots = int(seg_ord.size());
    auto cols16 = [&](int p) { return (pd[p].w + 15) / 16 * 16; };
    for (int p : one_ord) key[p] = (uint32_t(cols16(p)) << 16) | uint32_t(std::min(pd[p].y, 65535));
    sort_desc(one_ord, key);
    const size_t per_wave = size_t(64) * lane_p;
    for (size_t s0 = 0; s0 < one_ord.size(); s0 += per_wave) {
        LaneWave w{};
        w.slot0 = n_seg_slots + int(s0);
        w.rmin = INT32_MAX;
        for (size_t k = s0; k < std::min(one_ord.size(), s0 + per_wave); ++k) {
            const int p = one_ord[k];
            w.rmax = std::max(w.rmax, pd[p].y);
            w.rmin = std::min(w.rmin, pd[p].y);
            w.ncols = std::max(w.ncols, cols16(p));
        }
        w.carry_row = carry_rows;
        if (w.ncols > LV.BC) carry_rows += w.rmax + 1;
        lw.push_back(w);
    }
    lane_ord = std::move(seg_ord);
    lane_ord.insert(lane_ord.end(), one_ord.begin(), one_ord.end());
    // Anti-diagonal classes: W by H; (stripes, H) descending so the G pairs
    // sharing a wave have equal stripe counts and similar H, heaviest first.
    const int Wc[2] = {16, 64};
    int ring_len[2];
    for (int c = 0; c < 2; ++c) {
        const int W = Wc[c];
        int hm = 0;
        for (int p : ord[c]) {
            key[p] = (uint32_t((pd[p].y + W - 1) / W) << 16) | uint32_t(pd[p].w);
            hm = std::max(hm, pd[p].w);
        }
        sort_desc(ord[c], key);
        ring_len[c] = hm + 2 * W + 16;
    }

    tm.mark("binning");
    // One device region: uploaded arrays first, then outputs and scratch.
    // Host uploads raw bytes; the device packs rows and hap tables
    // (pack_kernels.hip), so the host work is memcpy.
    std::vector<int64_t> hb_off(nh + 1, 0);
    for (int64_t h = 0; h < nh; ++h) hb_off[h + 1] = hb_off[h] + haps[h].len;
    const size_t nrows = size_t(row_off[nr]);
    const size_t stride = (nrows + 16 + 15) & ~size_t(15);   // one byte plane, padded
    Layout L;
    const size_t o_pairs = L.take(sizeof(PairDesc) * npairs);
    const size_t o_raw = L.take(5 * stride);
    const size_t o_hb = L.take(size_t(hb_off[nh]) + 16);
    const size_t o_hd = L.take(sizeof(int4) * nh);
    const size_t o_t0 = L.take(sizeof(long long) * nh);
    const size_t o_rd = L.take(sizeof(int2) * nr);
    const size_t o_ord0 = L.take(sizeof(int) * ord[0].size());
    const size_t o_ord1 = L.take(sizeof(int) * ord[1].size());
    const size_t o_lord = L.take(sizeof(int) * lane_ord.size());
    const size_t o_lw = L.take(sizeof(LaneWave) * lw.size());
    const size_t upload = L.off;
    const size_t o_rows = L.take(sizeof(uint32_t) * (nrows + 16));
    const size_t o_hapw = L.take(sizeof(uint32_t) * (hap_off[nh] + 1));
    const size_t n1 = size_t(std::max<int64_t>(npairs, 1));
    const size_t o_raw32 = L.take(sizeof(float) * n1);
    const size_t o_raw64 = L.take(sizeof(double) * n1);
    const size_t o_flag = L.take(n1);
    const size_t o_list = L.take(sizeof(int) * n1);
    const size_t o_count = L.take(2 * sizeof(int));
    const size_t o_sorted = L.take(sizeof(int) * n1);
    const size_t o_big = L.take(sizeof(int) * n1);
    const size_t o_bigc = L.take(sizeof(int));
    const size_t o_plan = L.take(sizeof(Seg64Plan));
    const size_t o_carry = L.take(sizeof(float2) * size_t(carry_rows) * 64 * lane_p);
    const size_t total = L.off;

    char* host = nullptr;
    bool own_host = false;
    int rc = HC_PHMM_OK;
    if (borrow_ws) {
        rc = ws_host(upload, &host);
    } else {
        if (hipHostMalloc(&host, std::max<size_t>(upload, 1), hipHostMallocDefault) != hipSuccess)
            rc = fail(HC_PHMM_ENOMEM, "pinned staging buffer");
        own_host = true;
    }
    if (rc) return rc;
    tm.mark("staging alloc");

    // Fill the staging image (parallel over reads and haps).
    std::memcpy(host + o_pairs, pd.data(), sizeof(PairDesc) * npairs);
    uint8_t* raw = reinterpret_cast<uint8_t*>(host + o_raw);
    int2* rdesc = reinterpret_cast<int2*>(host + o_rd);
    parallel_for(nr, [&](int64_t b, int64_t e) {
        for (int64_t r = b; r < e; ++r) {
            const ReadView& v = reads[r];
            const size_t o = size_t(row_off[r]);
            std::memcpy(raw + o, v.bases, v.len);
            std::memcpy(raw + stride + o, v.q, v.len);
            std::memcpy(raw + 2 * stride + o, v.i, v.len);
            std::memcpy(raw + 3 * stride + o, v.d, v.len);
            std::memcpy(raw + 4 * stride + o, v.c, v.len);
            rdesc[r] = make_int2(int(o), v.len);
        }
    }, 1024);
    uint8_t* hb = reinterpret_cast<uint8_t*>(host + o_hb);
    int4* hd = reinterpret_cast<int4*>(host + o_hd);
    long long* t0 = reinterpret_cast<long long*>(host + o_t0);
    parallel_for(nh, [&](int64_t b, int64_t e) {
        for (int64_t h = b; h < e; ++h) {
            std::memcpy(hb + hb_off[h], haps[h].bases, haps[h].len);
            hd[h] = make_int4(int(hb_off[h]), haps[h].len, int(hap_off[h]), 0);
            t0[h] = hap_off[h] / 5;
        }
    }, 1024);
    std::memcpy(host + o_ord0, ord[0].data(), sizeof(int) * ord[0].size());
    std::memcpy(host + o_ord1, ord[1].data(), sizeof(int) * ord[1].size());
    std::memcpy(host + o_lord, lane_ord.data(), sizeof(int) * lane_ord.size());
    std::memcpy(host + o_lw, lw.data(), sizeof(LaneWave) * lw.size());

    tm.mark("pack");
    auto* b = new hc_phmm_batch();
    char* dev = nullptr;
    if (borrow_ws) {
        rc = ws_dev(total, &dev);
        b->owns_dev = false;
    } else if (hipMalloc(&dev, total) != hipSuccess) {
        rc = fail(HC_PHMM_ENOMEM, "device allocation failed (" + std::to_string(total >> 20) + " MiB)");
    }
    if (rc == HC_PHMM_OK) {
        b->dev_base = dev;
        // The workspace staging stays valid until the call returns, so only a
        // batch-owned staging buffer needs the copy to finish here.
        hipError_t e1 = hipMemcpyAsync(dev, host, upload, hipMemcpyHostToDevice, g_eng.stream);
        if (e1 == hipSuccess) e1 = hipMemsetAsync(dev + o_count, 0, 2 * sizeof(int), g_eng.stream);
        if (e1 == hipSuccess)
            e1 = launch_pack_rows(reinterpret_cast<const uint8_t*>(dev + o_raw), (long long)nrows,
                                  (long long)stride, reinterpret_cast<uint32_t*>(dev + o_rows), g_eng.stream);
        if (e1 == hipSuccess && !std::getenv("HC_PHMM_NO_CG"))   // A/B switch for the CG path
            e1 = launch_mark_cg(reinterpret_cast<uint32_t*>(dev + o_rows), reinterpret_cast<const int2*>(dev + o_rd),
                                int(nr), g_eng.stream);
        if (e1 == hipSuccess)
            e1 = launch_hap_tables(reinterpret_cast<const uint8_t*>(dev + o_hb),
                                   reinterpret_cast<const int4*>(dev + o_hd), int(nh),
                                   reinterpret_cast<const long long*>(dev + o_t0), hap_off[nh] / 5,
                                   reinterpret_cast<uint32_t*>(dev + o_hapw), g_eng.stream);
        const hipError_t e2 = (e1 == hipSuccess && own_host) ? hipStreamSynchronize(g_eng.stream) : e1;
        if (e2 != hipSuccess) rc = fail(HC_PHMM_EHIP, std::string("H2D: ") + hipGetErrorString(e2));
    }
    if (own_host) (void)hipHostFree(host);
    tm.mark("device alloc+H2D");
    if (rc != HC_PHMM_OK) {
        free_batch(b);
        return rc;
    }
    b->n = npairs;
    b->cells = cells;
    b->Hmax = Hmax;
    b->n_lane = int(lane_ord.size());
    b->n_seg_waves = n_seg_waves;
    b->lane_variant = lane_var;
    b->lane_waves = int(lw.size());
    b->d_pairs = reinterpret_cast<PairDesc*>(dev + o_pairs);
    b->d_rows = reinterpret_cast<uint32_t*>(dev + o_rows);
    b->d_hapw = reinterpret_cast<uint32_t*>(dev + o_hapw);
    for (int c = 0; c < 2; ++c) {
        b->cls[c].W = Wc[c];
        b->cls[c].n = int(ord[c].size());
        b->cls[c].ring_len = ring_len[c];
    }
    b->cls[0].d_order = reinterpret_cast<int*>(dev + o_ord0);
    b->cls[1].d_order = reinterpret_cast<int*>(dev + o_ord1);
    b->d_lane_order = reinterpret_cast<int*>(dev + o_lord);
    b->d_lane_waves = reinterpret_cast<LaneWave*>(dev + o_lw);
    b->own_raw32 = b->d_raw32 = reinterpret_cast<float*>(dev + o_raw32);
    b->own_raw64 = b->d_raw64 = reinterpret_cast<double*>(dev + o_raw64);
    b->own_flag = b->d_flag = reinterpret_cast<uint8_t*>(dev + o_flag);
    b->d_list = reinterpret_cast<int*>(dev + o_list);
    b->d_count = reinterpret_cast<int*>(dev + o_count);
    b->d_sorted = reinterpret_cast<int*>(dev + o_sorted);
    b->d_big = reinterpret_cast<int*>(dev + o_big);
    b->d_big_count = reinterpret_cast<int*>(dev + o_bigc);
    b->d_plan = reinterpret_cast<Seg64Plan*>(dev + o_plan);
    b->n_wide = n_wide;
    b->d_carry = carry_rows ? reinterpret_cast<float2*>(dev + o_carry) : nullptr;
    *out = b;
    return HC_PHMM_OK;
}

int run(hc_phmm_batch* b, hipStream_t s)
{
    if (!s) s = g_eng.stream;
    b->last_stream = s;
    b->launch_waves = 0;
    if (b->ev_used == b->ev_pool.size()) {
        std::array<hipEvent_t, 3> t{};
        for (auto& e : t) HIP_TRY(hipEventCreate(&e));
        b->ev_pool.push_back(t);
    }
    const auto& ev = b->ev_pool[b->ev_used++];
    for (int k = 0; k < 3; ++k) b->ev[k] = ev[k];
    HIP_TRY(hipEventRecord(b->ev[0], s));
    // No memsets: the fp32 kernels zero each pair's raw f64 slot as they emit,
    // and the rescue kernel zeroes the other parity's counter for the next run.
    const int par = b->parity;
    b->parity ^= 1;
    int* count = b->d_count + par;
    if (b->n_lane > 0) {
        LaneArgs a{};
        a.pairs = b->d_pairs;
        a.order = b->d_lane_order;
        a.n_slots = b->n_lane;
        a.carry = b->d_carry;
        a.rows = b->d_rows;
        a.hapw = b->d_hapw;
        a.lut = g_eng.lut_f;
        a.raw_out = b->d_raw32;
        a.rescue_flag = b->d_flag;
        a.rescue_list = b->d_list;
        a.rescue_count = count;
        a.raw64_zero = b->d_raw64;
        b->launch_waves += b->lane_waves;
        const int n_one = b->lane_waves - b->n_seg_waves;
        const bool fork = b->n_seg_waves > 0 && n_one > 0;
        if (b->n_seg_waves > 0) {
            // Segmented waves; beside one-lane waves (long haps) they go on the
            // side stream, launched first so they are dispatched first.
            LaneArgs g = a;
            g.waves = b->d_lane_waves;
            g.n_waves = b->n_seg_waves;
            if (fork) {
                HIP_TRY(hipEventRecord(g_eng.fork, s));
                HIP_TRY(hipStreamWaitEvent(g_eng.side, g_eng.fork, 0));
            }
            HIP_TRY(launch_lane_seg_f32(g, fork ? g_eng.side : s));
            if (fork) HIP_TRY(hipEventRecord(g_eng.join, g_eng.side));
        }
        if (n_one > 0) {
            a.waves = b->d_lane_waves + b->n_seg_waves;
            a.n_waves = n_one;
            HIP_TRY(launch_lane_f32(b->lane_variant, a, s));
        }
        if (fork) HIP_TRY(hipStreamWaitEvent(s, g_eng.join, 0));
    }
    for (auto& c : b->cls) {
        if (c.n == 0) continue;
        DiagArgs a{};
        a.pairs = b->d_pairs;
        a.order = c.d_order;
        a.n_slots = c.n;
        a.rows = b->d_rows;
        a.hapw = b->d_hapw;
        a.lut = g_eng.lut_f;
        a.ring_len = c.ring_len;
        a.raw_out = b->d_raw32;
        a.rescue_flag = b->d_flag;
        a.rescue_list = b->d_list;
        a.rescue_count = count;
        a.raw64_zero = b->d_raw64;
        const int G = 64 / c.W;
        const int grid = (c.n + G - 1) / G;
        b->launch_waves += grid;
        HIP_TRY(launch_diag_f32(c.W, a, grid, s));
    }
    HIP_TRY(hipEventRecord(b->ev[1], s));
    if (b->n > 0) {
        // fp64 rescue (intel_pairhmm.hpp:137-139) over the device-built list, no
        // host round trip for its length: device planning + column-segmented
        // fp64 waves (grid-stride), then the anti-diagonal fp64 kernel for haps
        // wider than 64 blocks of 32 (only launched if the batch has any).
        Seg64Args r{};
        r.pairs = b->d_pairs;
        r.rows = b->d_rows;
        r.hapw = b->d_hapw;
        r.lut = g_eng.lut_d;
        r.list = b->d_list;
        r.count = count;
        r.count_reset = b->d_count + (par ^ 1);
        r.sorted = b->d_sorted;
        r.big = b->d_big;
        r.big_count = b->d_big_count;
        r.plan = b->d_plan;
        r.raw_out = b->d_raw64;
        r.min_lanes = int64_t(2) * 4 * g_eng.n_cu * 64;
        const int grid = int(std::min<int64_t>((b->n + 3) / 4, int64_t(2) * g_eng.n_cu));
        HIP_TRY(launch_rescue_seg64(r, grid, s));
        if (b->n_wide > 0) {
            DiagArgs a{};
            a.pairs = b->d_pairs;
            a.order = b->d_big;
            a.n_slots_dev = b->d_big_count;
            a.rows = b->d_rows;
            a.hapw = b->d_hapw;
            a.lut = g_eng.lut_d;
            a.ring_len = b->Hmax + 2 * 64 + 16;
            a.raw_out = b->d_raw64;
            HIP_TRY(launch_diag_f64(64, a, int(std::min<int64_t>(b->n_wide, 2048)), s));
        }
    }
    HIP_TRY(hipEventRecord(b->ev[2], s));
    b->ran = true;
    return HC_PHMM_OK;
}

int results(hc_phmm_batch* b, double* loglik, float* raw32, double* raw64, uint8_t* resc)
{
    if (!b->ran) return fail(HC_PHMM_EINVAL, "batch has not been run");
    const int64_t n = b->n;
    if (n == 0) return HC_PHMM_OK;
    // D2H into the pinned workspace: [raw32 | raw64 | flags]. Drain the stream
    // first: growing the workspace frees the staging an earlier H2D read.
    HIP_TRY(hipStreamSynchronize(b->last_stream));
    char* host = nullptr;
    const size_t o64 = (sizeof(float) * n + 15) & ~size_t(15);
    const size_t ofl = o64 + sizeof(double) * n;
    int rc = ws_host(ofl + n, &host);
    if (rc) return rc;
    hipStream_t s = b->last_stream;
    HIP_TRY(hipMemcpyAsync(host, b->d_raw32, sizeof(float) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(host + o64, b->d_raw64, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(host + ofl, b->d_flag, n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const float* f = reinterpret_cast<const float*>(host);
    const double* d = reinterpret_cast<const double*>(host + o64);
    const uint8_t* fl = reinterpret_cast<const uint8_t*>(host + ofl);
    if (raw32) std::memcpy(raw32, f, sizeof(float) * n);
    if (raw64) std::memcpy(raw64, d, sizeof(double) * n);
    if (resc) std::memcpy(resc, fl, n);
    if (loglik) {
        // intel_pairhmm.hpp:137-143, glibc log10 / log10f as in the reference.
        const Luts& L = luts();
        const float l10f = L.log10_init_f;
        const double l10d = L.log10_init_d;
        parallel_for(n, [&](int64_t lo, int64_t hi) {
            for (int64_t p = lo; p < hi; ++p)
                loglik[p] = fl[p] ? std::log10(d[p]) - l10d : double(std::log10(f[p]) - l10f);
        }, 1 << 15);
    }
    return HC_PHMM_OK;
}

int run_sync(hc_phmm_batch* b, double* loglik, float* raw32, double* raw64, uint8_t* resc)
{
    PhaseTimer tm;
    int rc = run(b, nullptr);
    tm.mark("run (launch)");
    if (rc == HC_PHMM_OK) rc = results(b, loglik, raw32, raw64, resc);
    tm.mark("results+finish");
    return rc;
}

int flat_views(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
               const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
               const uint8_t* del, const uint8_t* gcp, const uint8_t* hap,
               std::vector<ReadView>& rv, std::vector<HapView>& hv, std::vector<int32_t>& idx)
{
    if (n < 0) return fail(HC_PHMM_EINVAL, "negative pair count");
    if (n > 0 && (!read_off || !R || !hap_off || !H || !rs || !q || !ins || !del || !gcp || !hap))
        return fail(HC_PHMM_EINVAL, "null input array");
    rv.resize(n);
    hv.resize(n);
    idx.resize(n);
    for (int64_t p = 0; p < n; ++p) {
        const int64_t o = read_off[p];
        rv[p] = ReadView{R[p], rs + o, q + o, ins + o, del + o, gcp + o};
        hv[p] = HapView{H[p], hap + hap_off[p]};
        idx[p] = int32_t(p);
    }
    return HC_PHMM_OK;
}

}  // namespace

// --------------------------------------------------------------------------
// C ABI
namespace hcphmm {
// Shared with sw_engine.cpp: one last-error slot per thread for the library.
void set_last_error(const std::string& msg) { g_err = msg; }
}  // namespace hcphmm

extern "C" {

int hc_phmm_version(void) { return 100; }

const char* hc_phmm_last_error(void) { return g_err.c_str(); }

int hc_phmm_init(uint32_t /*flags*/, int device)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return ensure_init(device);
}

int hc_phmm_shutdown(void)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_eng.ready) return HC_PHMM_OK;
    (void)hipFree(g_eng.lut_f);
    (void)hipFree(g_eng.lut_d);
    (void)hipFree(g_ws.dev);
    (void)hipHostFree(g_ws.host);
    free_batch(g_ws.batch);
    g_ws = Workspace{};
    (void)hipEventDestroy(g_eng.fork);
    (void)hipEventDestroy(g_eng.join);
    (void)hipStreamDestroy(g_eng.side);
    (void)hipStreamDestroy(g_eng.stream);
    g_eng = Engine{};
    return HC_PHMM_OK;
}

int hc_phmm_get_luts(float* pf, double* pd, float* mf, double* md)
{
    const Luts& L = luts();
    if (pf) std::memcpy(pf, L.ph2pr_f, sizeof(L.ph2pr_f));
    if (pd) std::memcpy(pd, L.ph2pr_d, sizeof(L.ph2pr_d));
    if (mf) std::memcpy(mf, L.mm_f.data(), sizeof(float) * kMMEntries);
    if (md) std::memcpy(md, L.mm_d.data(), sizeof(double) * kMMEntries);
    return HC_PHMM_OK;
}

int hc_phmm_pairs_flat(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                       const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                       const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, double* loglik,
                       float* raw_f32, double* raw_f64, uint8_t* rescued)
{
    std::lock_guard<std::mutex> lk(g_mu);
    int rc = ensure_init(-1);
    if (rc) return rc;
    if (n == 0) return HC_PHMM_OK;
    std::vector<ReadView> rv;
    std::vector<HapView> hv;
    std::vector<int32_t> idx;
    rc = flat_views(n, read_off, R, hap_off, H, rs, q, ins, del, gcp, hap, rv, hv, idx);
    if (rc) return rc;
    hc_phmm_batch* b = nullptr;
    rc = plan(rv, hv, n, idx.data(), idx.data(), true, &b);
    if (rc) return rc;
    rc = run_sync(b, loglik, raw_f32, raw_f64, rescued);
    free_batch(b);
    return rc;
}

int hc_phmm_cross(const hc_phmm_read* reads, int32_t n_reads, const hc_phmm_hap* haps,
                  int32_t n_haps, double* out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (n_reads < 0 || n_haps < 0) return fail(HC_PHMM_EINVAL, "negative count");
    if (n_reads == 0 || n_haps == 0) return HC_PHMM_OK;
    if (!reads || !haps || !out) return fail(HC_PHMM_EINVAL, "null argument");
    int rc = ensure_init(-1);
    if (rc) return rc;
    std::vector<ReadView> rv(n_reads);
    std::vector<HapView> hv(n_haps);
    for (int r = 0; r < n_reads; ++r)
        rv[r] = ReadView{reads[r].length, (const uint8_t*)reads[r].bases, (const uint8_t*)reads[r].q,
                         (const uint8_t*)reads[r].i, (const uint8_t*)reads[r].d, (const uint8_t*)reads[r].c};
    for (int h = 0; h < n_haps; ++h) hv[h] = HapView{haps[h].length, (const uint8_t*)haps[h].bases};
    const int64_t np = int64_t(n_reads) * n_haps;
    std::vector<int32_t> pr(np), ph(np);
    for (int64_t p = 0; p < np; ++p) {
        pr[p] = int32_t(p / n_haps);   // read-major, intel_pairhmm.hpp:131-132
        ph[p] = int32_t(p % n_haps);
    }
    hc_phmm_batch* b = nullptr;
    rc = plan(rv, hv, np, pr.data(), ph.data(), true, &b);
    if (rc) return rc;
    rc = run_sync(b, out, nullptr, nullptr, nullptr);
    free_batch(b);
    return rc;
}

int hc_phmm_cross_regions(const hc_phmm_region* regions, int32_t n_regions)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (n_regions < 0 || (n_regions > 0 && !regions)) return fail(HC_PHMM_EINVAL, "bad region list");
    int rc = ensure_init(-1);
    if (rc) return rc;
    std::vector<ReadView> rv;
    std::vector<HapView> hv;
    std::vector<int32_t> pr, ph;
    std::vector<int64_t> out_base;   // first pair of each region
    for (int k = 0; k < n_regions; ++k) {
        const hc_phmm_region& g = regions[k];
        if (g.n_reads < 0 || g.n_haps < 0) return fail(HC_PHMM_EINVAL, "negative count in region");
        out_base.push_back(int64_t(pr.size()));
        if (g.n_reads == 0 || g.n_haps == 0) continue;
        if (!g.reads || !g.haps || !g.out) return fail(HC_PHMM_EINVAL, "null pointer in region");
        const int32_t r0 = int32_t(rv.size()), h0 = int32_t(hv.size());
        for (int r = 0; r < g.n_reads; ++r)
            rv.push_back(ReadView{g.reads[r].length, (const uint8_t*)g.reads[r].bases, (const uint8_t*)g.reads[r].q,
                                  (const uint8_t*)g.reads[r].i, (const uint8_t*)g.reads[r].d,
                                  (const uint8_t*)g.reads[r].c});
        for (int h = 0; h < g.n_haps; ++h) hv.push_back(HapView{g.haps[h].length, (const uint8_t*)g.haps[h].bases});
        for (int r = 0; r < g.n_reads; ++r)
            for (int h = 0; h < g.n_haps; ++h) {
                pr.push_back(r0 + r);
                ph.push_back(h0 + h);
            }
    }
    const int64_t np = int64_t(pr.size());
    if (np == 0) return HC_PHMM_OK;
    hc_phmm_batch* b = nullptr;
    rc = plan(rv, hv, np, pr.data(), ph.data(), true, &b);
    if (rc) return rc;
    std::vector<double> all(np);
    rc = run_sync(b, all.data(), nullptr, nullptr, nullptr);
    free_batch(b);
    if (rc) return rc;
    for (int k = 0; k < n_regions; ++k) {
        const hc_phmm_region& g = regions[k];
        if (g.n_reads == 0 || g.n_haps == 0) continue;
        std::memcpy(g.out, all.data() + out_base[k], sizeof(double) * size_t(g.n_reads) * g.n_haps);
    }
    return HC_PHMM_OK;
}

int hc_phmm_compute_likelihoods(const hc_phmm_read* reads, int32_t n_reads, const hc_phmm_hap* haps,
                                int32_t n_haps, double* out, uint8_t* keep, int32_t* n_kept)
{
    int rc = hc_phmm_cross(reads, n_reads, haps, n_haps, out);
    if (rc) return rc;
    if (n_reads > 0 && (!keep || !n_kept)) return fail(HC_PHMM_EINVAL, "null keep/n_kept");
    int kept = 0;
    // normalize_likelihoods_and_filter_poorly_modeled_reads, intel_pairhmm.hpp:24-46
    for (int r = 0; r < n_reads; ++r) {
        double* row = out + size_t(r) * n_haps;
        double best = n_haps ? row[0] : -INFINITY;
        for (int h = 1; h < n_haps; ++h)
            if (best < row[h]) best = row[h];
        const double cap = best + -4.5;
        for (int h = 0; h < n_haps; ++h)
            if (row[h] < cap) row[h] = cap;
        const double thr = std::min(2.0, std::ceil(double(reads[r].length) * 0.02)) * -4.0;
        keep[r] = !(best < thr);
        kept += keep[r];
    }
    if (n_kept) *n_kept = kept;
    return HC_PHMM_OK;
}

int hc_phmm_batch_create(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                         const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                         const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, hc_phmm_batch** out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!out) return fail(HC_PHMM_EINVAL, "null out");
    int rc = ensure_init(-1);
    if (rc) return rc;
    std::vector<ReadView> rv;
    std::vector<HapView> hv;
    std::vector<int32_t> idx;
    rc = flat_views(n, read_off, R, hap_off, H, rs, q, ins, del, gcp, hap, rv, hv, idx);
    if (rc) return rc;
    return plan(rv, hv, n, idx.data(), idx.data(), false, out);
}

int hc_phmm_batch_run(hc_phmm_batch* b, void* stream)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    if (!g_eng.ready) return fail(HC_PHMM_ENODEV, "not initialised");
    return run(b, static_cast<hipStream_t>(stream));
}

int hc_phmm_batch_results(hc_phmm_batch* b, double* loglik, float* raw_f32, double* raw_f64,
                          uint8_t* rescued)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    return results(b, loglik, raw_f32, raw_f64, rescued);
}

int hc_phmm_batch_device_results(hc_phmm_batch* b, void** raw_f32, void** raw_f64, void** rescued)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    if (raw_f32) *raw_f32 = b->d_raw32;
    if (raw_f64) *raw_f64 = b->d_raw64;
    if (rescued) *rescued = b->d_flag;
    return HC_PHMM_OK;
}

int hc_phmm_batch_bind_outputs(hc_phmm_batch* b, void* raw_f32, void* raw_f64, void* rescued)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    b->d_raw32 = raw_f32 ? static_cast<float*>(raw_f32) : b->own_raw32;
    b->d_raw64 = raw_f64 ? static_cast<double*>(raw_f64) : b->own_raw64;
    b->d_flag = rescued ? static_cast<uint8_t*>(rescued) : b->own_flag;
    return HC_PHMM_OK;
}

int hc_phmm_batch_stats(hc_phmm_batch* b, hc_phmm_stats* st)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!b || !st) return fail(HC_PHMM_EINVAL, "null argument");
    std::memset(st, 0, sizeof(*st));
    st->n_pairs = b->n;
    st->cells = b->cells;
    st->n_launch_waves = b->launch_waves;
    st->n_lane_pairs = b->n_lane;
    st->n_seg_waves = b->n_seg_waves;
    if (b->ran && b->ev_used > 0) {
        HIP_TRY(hipStreamSynchronize(b->last_stream));
        double sa = 0, sc = 0;
        for (size_t k = 0; k < b->ev_used; ++k) {
            float a = 0, c = 0;
            HIP_TRY(hipEventSynchronize(b->ev_pool[k][2]));
            HIP_TRY(hipEventElapsedTime(&a, b->ev_pool[k][0], b->ev_pool[k][1]));
            HIP_TRY(hipEventElapsedTime(&c, b->ev_pool[k][1], b->ev_pool[k][2]));
            sa += a;
            sc += c;
        }
        st->n_runs = int64_t(b->ev_used);
        st->kernel_ms_f32 = sa / double(b->ev_used);
        st->kernel_ms_f64 = sc / double(b->ev_used);
        st->run_ms = st->kernel_ms_f32 + st->kernel_ms_f64;
        b->ev_used = 0;
        int cnt = 0;
        HIP_TRY(hipMemcpy(&cnt, b->d_count + (b->parity ^ 1), sizeof(int), hipMemcpyDeviceToHost));
        st->n_rescued = cnt;
    }
    return HC_PHMM_OK;
}

int hc_phmm_batch_destroy(hc_phmm_batch* b)
{
    std::lock_guard<std::mutex> lk(g_mu);
    free_batch(b);
    return HC_PHMM_OK;
}

}  // extern "C"

// --------------------------------------------------------------------------
// The reference's own accelerator slot: a strong definition of the weak
// `bool shacc_pairhmm::calculate(Batch&)` declared in
// pairhmm/native/shacc_pairhmm.h:10-36. The structs below are layout- and
// name-compatible declarations (same namespace, same member order) so the
// mangled symbol matches; results[r * num_haps + h] receives the fp32 cast of
// the log10 likelihood (the slot's `float* results`; hc_phmm_cross gives the
// full double).
namespace shacc_pairhmm {
struct Read {
    int length;
    const char* bases;
    const char* q;
    const char* i;
    const char* d;
    const char* c;
};
struct Haplotype {
    int length;
    const char* bases;
};
struct Batch {
    int num_reads;
    int num_haps;
    long num_cells;
    Read* reads;
    Haplotype* haps;
    float* results;
};
__attribute__((visibility("default"))) bool calculate(Batch& batch);
bool calculate(Batch& batch)
{
    static_assert(sizeof(Read) == sizeof(hc_phmm_read), "Read layout");
    static_assert(sizeof(Haplotype) == sizeof(hc_phmm_hap), "Haplotype layout");
    if (batch.num_reads < 0 || batch.num_haps < 0 || !batch.results) return false;
    std::vector<double> out(size_t(batch.num_reads) * size_t(batch.num_haps));
    const int rc = hc_phmm_cross(reinterpret_cast<const hc_phmm_read*>(batch.reads), batch.num_reads,
                                 reinterpret_cast<const hc_phmm_hap*>(batch.haps), batch.num_haps, out.data());
    if (rc != HC_PHMM_OK) return false;
    for (size_t k = 0; k < out.size(); ++k) batch.results[k] = float(out[k]);
    return true;
}
}  // namespace shacc_pairhmm
