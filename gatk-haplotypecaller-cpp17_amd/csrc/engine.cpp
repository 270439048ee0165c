// Host engine + C ABI of libhcpairhmm.so (include/hc_pairhmm.h).
//
// The reference's computeLikelihoodsNative (intel_pairhmm.hpp:115-152) split
// into plan / execute / finish over one or more device slots:
//   plan     (host) length-bin the pairs and pack them into waves; stage the
//            raw inputs in pinned memory, 2 bytes per read base (+3 only for
//            reads whose gap qualities vary) and 1 per hap base
//   execute  (device) H2D, pack rows + hap match tables, fp32 kernels ->
//            raw f32 + rescue list, fp64 rescue over the list, D2H of results
//   finish   (host) glibc log10f / log10 exactly as intel_pairhmm.hpp:137-143,
//            scattered into the caller's outputs
// A call is cut into parts: contiguous pair ranges (or region blocks) of equal
// cells, dealt round-robin over the device slots and, for large calls, over
// several chunks per slot, so the host planning of part k+1 overlaps the
// device work of part k. Each part in flight holds a grow-only workspace
// (device + pinned host), reused across calls.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/hc_pairhmm.h"
#include "kernels.hpp"
#include "luts.hpp"
#include "pool.hpp"

using namespace hcphmm;

namespace hcphmm {
// Shared with sw_engine.cpp / gt_engine.cpp.
void set_last_error(const std::string& msg);
int primary_device();   // HIP ordinal of the first device slot, -1 if not initialised
void sw_release();      // sw_engine.cpp: drop the aligner's stream and workspace
void gt_release();      // gt_engine.cpp: drop the genotyper's stream and buffers
}  // namespace hcphmm

namespace {

thread_local std::string g_err;

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

// ---------------------------------------------------------------------------
// Device slots.

// Grow-only workspace of one part in flight: device memory (upload image,
// packed rows and tables, outputs, scratch) and pinned host memory (upload
// image, then the D2H'd results).
struct Slot {
    char* dev = nullptr;
    size_t dev_cap = 0;
    char* host = nullptr;
    size_t host_cap = 0;
    bool busy = false;
    // Streams of the part in this slot: parts in different slots of one device
    // run concurrently (a call cut into parts overlaps the planning of part
    // k + 1 and the kernels of part k, and its kernels fill the chip together).
    hipStream_t stream = nullptr, side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;   // side-stream fork / join (timing disabled)
    hipEvent_t ev[6] = {};   // pack [2], fp32 / fp64 pass [3], done: reused by every part in the slot
};

struct Device {
    int ordinal = 0;
    int n_cu = 256;   // compute units (4 SIMDs each): sizes the lane-wave latency ceiling
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;                  // segmented waves beside one-lane waves
    hipEvent_t fork = nullptr, join = nullptr;   // side-stream fork / join (timing disabled)
    float* lut_f = nullptr;
    double* lut_d = nullptr;
    std::vector<Slot*> slots;
    double outstanding = 0;   // cells submitted and not yet collected
};

std::mutex g_mu;   // device list, slot pools, outstanding counters
std::vector<Device*> g_devs;

void release_device(Device* d)
{
    if (!d) return;
    (void)hipSetDevice(d->ordinal);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    for (Slot* s : d->slots) {
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        if (s->side) (void)hipStreamSynchronize(s->side);
        if (s->dev) (void)hipFree(s->dev);
        if (s->host) (void)hipHostFree(s->host);
        for (auto& e : s->ev)
            if (e) (void)hipEventDestroy(e);
        if (s->fork) (void)hipEventDestroy(s->fork);
        if (s->join) (void)hipEventDestroy(s->join);
        if (s->side) (void)hipStreamDestroy(s->side);
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
    }
    if (d->lut_f) (void)hipFree(d->lut_f);
    if (d->lut_d) (void)hipFree(d->lut_d);
    if (d->fork) (void)hipEventDestroy(d->fork);
    if (d->join) (void)hipEventDestroy(d->join);
    if (d->side) (void)hipStreamDestroy(d->side);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

int init_device(Device& d)
{
    HIP_TRY(hipSetDevice(d.ordinal));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, d.ordinal));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(HC_PHMM_ENODEV, std::string("device ") + std::to_string(d.ordinal) + " is " +
                                        prop.gcnArchName + ", need gfx950");
    HIP_TRY(configure_kernels());
    d.n_cu = std::max(1, prop.multiProcessorCount);
    HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&d.side, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&d.fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.join, hipEventDisableTiming));
    const Luts& L = luts();
    HIP_TRY(hipMalloc(&d.lut_f, sizeof(float) * kTableLen));
    HIP_TRY(hipMalloc(&d.lut_d, sizeof(double) * kTableLen));
    HIP_TRY(hipMemcpy(d.lut_f, L.dev_f.data(), sizeof(float) * kTableLen, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d.lut_d, L.dev_d.data(), sizeof(double) * kTableLen, hipMemcpyHostToDevice));
    return HC_PHMM_OK;
}

// Resolve a device list (-1 = current device; empty = every visible device).
int resolve_devices(const int32_t* devices, int32_t n, std::vector<int>& out)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(HC_PHMM_ENODEV, "no HIP device visible");
    out.clear();
    if (!devices || n <= 0) {
        for (int k = 0; k < count; ++k) out.push_back(k);
        return HC_PHMM_OK;
    }
    for (int32_t k = 0; k < n; ++k) {
        int dev = devices[k];
        if (dev < 0) HIP_TRY(hipGetDevice(&dev));
        if (dev >= count) return fail(HC_PHMM_ENODEV, "device ordinal " + std::to_string(dev) + " out of range");
        out.push_back(dev);
    }
    return HC_PHMM_OK;
}

// Under g_mu.
int init_devices_locked(const int32_t* devices, int32_t n, bool any_ok)
{
    if (!g_devs.empty()) {
        if (any_ok) return HC_PHMM_OK;
        std::vector<int> want;
        const int rc = resolve_devices(devices, n, want);
        if (rc) return rc;
        bool same = want.size() == g_devs.size();
        for (size_t k = 0; same && k < want.size(); ++k) same = want[k] == g_devs[k]->ordinal;
        if (same) return HC_PHMM_OK;
        std::string have;
        for (const Device* d : g_devs) have += (have.empty() ? "" : ",") + std::to_string(d->ordinal);
        return fail(HC_PHMM_EINVAL, "engine already initialised on device(s) " + have +
                                        "; call hc_phmm_shutdown() before selecting others");
    }
    std::vector<int> want;
    int rc = resolve_devices(devices, n, want);
    if (rc) return rc;
    std::vector<Device*> made;
    for (int o : want) {
        auto* d = new Device();
        d->ordinal = o;
        made.push_back(d);
        rc = init_device(*d);
        if (rc) {
            for (Device* x : made) release_device(x);
            return rc;
        }
    }
    g_devs = made;
    (void)hipSetDevice(g_devs[0]->ordinal);
    return HC_PHMM_OK;
}

int ensure_init()
{
    std::lock_guard<std::mutex> lk(g_mu);
    const int32_t cur = -1;
    return init_devices_locked(&cur, 1, true);
}

// A free slot of device d (d current on the calling thread), its streams and
// events created on first use; nullptr if they cannot be created.
Slot* take_slot(Device& d)
{
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (Slot* s : d.slots)
            if (!s->busy) {
                s->busy = true;
                return s;
            }
    }
    auto* s = new Slot();
    bool ok = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&s->fork, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&s->join, hipEventDisableTiming) == hipSuccess;
    for (int k = 0; ok && k < 6; ++k)
        ok = hipEventCreateWithFlags(&s->ev[k], k == 5 ? hipEventDisableTiming : 0) == hipSuccess;
    if (!ok) {
        for (auto& e : s->ev)
            if (e) (void)hipEventDestroy(e);
        if (s->fork) (void)hipEventDestroy(s->fork);
        if (s->join) (void)hipEventDestroy(s->join);
        if (s->side) (void)hipStreamDestroy(s->side);
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
        fail(HC_PHMM_EHIP, "slot stream / event creation");
        return nullptr;
    }
    s->busy = true;
    std::lock_guard<std::mutex> lk(g_mu);
    d.slots.push_back(s);
    return s;
}

void give_slot(Slot* s)
{
    std::lock_guard<std::mutex> lk(g_mu);
    s->busy = false;
}

// Grow a slot (caller's device current). Growing drops the old contents.
int slot_reserve(Slot& s, size_t dev_bytes, size_t host_bytes)
{
    if (dev_bytes > s.dev_cap) {
        if (s.dev) HIP_TRY(hipFree(s.dev));
        s.dev = nullptr;
        s.dev_cap = 0;
        const size_t cap = std::max(dev_bytes + dev_bytes / 4, size_t(16) << 20);
        if (hipMalloc(&s.dev, cap) != hipSuccess) return fail(HC_PHMM_ENOMEM, "device workspace");
        s.dev_cap = cap;
    }
    if (host_bytes > s.host_cap) {
        if (s.host) HIP_TRY(hipHostFree(s.host));
        s.host = nullptr;
        s.host_cap = 0;
        const size_t cap = std::max(host_bytes + host_bytes / 4, size_t(4) << 20);
        if (hipHostMalloc(&s.host, cap, hipHostMallocPortable) != hipSuccess)
            return fail(HC_PHMM_ENOMEM, "pinned staging buffer");
        s.host_cap = cap;
    }
    return HC_PHMM_OK;
}

// ---------------------------------------------------------------------------
// Inputs.

struct ReadView {
    int32_t len;
    const uint8_t *bases, *q, *i, *d, *c;
};
struct HapView {
    int32_t len;
    const uint8_t* bases;
};

// Where a call's reads and haps live: flat pools (pair p = read p x hap p) or
// struct arrays (hc_phmm_read / hc_phmm_hap).
struct Src {
    const int64_t* read_off = nullptr;
    const int32_t* R = nullptr;
    const int64_t* hap_off = nullptr;
    const int32_t* H = nullptr;
    const uint8_t *rs = nullptr, *q = nullptr, *ins = nullptr, *del = nullptr, *gcp = nullptr, *hap = nullptr;
    const hc_phmm_read* reads = nullptr;
    const hc_phmm_hap* haps = nullptr;

    ReadView read(int64_t k) const
    {
        if (reads) {
            const hc_phmm_read& r = reads[k];
            return ReadView{r.length, (const uint8_t*)r.bases, (const uint8_t*)r.q, (const uint8_t*)r.i,
                            (const uint8_t*)r.d, (const uint8_t*)r.c};
        }
        const int64_t o = read_off[k];
        return ReadView{R[k], rs + o, q + o, ins + o, del + o, gcp + o};
    }
    HapView hapv(int64_t k) const
    {
        if (haps) return HapView{haps[k].length, (const uint8_t*)haps[k].bases};
        return HapView{H[k], hap + hap_off[k]};
    }
    int32_t read_len(int64_t k) const { return reads ? reads[k].length : R[k]; }
    int32_t hap_len(int64_t k) const { return haps ? haps[k].length : H[k]; }
};

// Cross-product block: reads [r0, r0+nr) x haps [h0, h0+nh) of the Src, results
// to out[r * ostride + h] (read-major, as hc_phmm_cross / a region).
struct Block {
    int64_t r0;
    int32_t nr;
    int64_t h0;
    int32_t nh;
    double* out;
    int64_t ostride;
};

// Caller outputs of flat (pair) calls; any may be null.
struct Outputs {
    double* loglik = nullptr;
    float* raw32 = nullptr;
    double* raw64 = nullptr;
    uint8_t* resc = nullptr;
};

// What one part computes: flat pairs [lo, hi) (read p x hap p), or blocks.
struct PartSpec {
    bool flat = true;
    int64_t lo = 0, hi = 0;
    std::vector<Block> blocks;
};

// HC_PHMM_TRACE=1: per-phase host timings on stderr.
struct PhaseTimer {
    bool on;
    std::chrono::steady_clock::time_point t0;
    PhaseTimer() : on(std::getenv("HC_PHMM_TRACE") != nullptr), t0(std::chrono::steady_clock::now()) {}
    void mark(const char* what)
    {
        if (!on) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[hc_phmm] %-22s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    }
};

// Host-only planning (no device calls): hcx_plan_* below time the host side
// of plan_part in a container without a GPU.
bool g_dry = false;

// The last dry-run plan (hcx_dump_sizes / hcx_dump_plan).
struct DryDump {
    std::mutex mu;
    std::vector<int4> pairs;
    std::vector<int> order;
    std::vector<LaneWave> waves;
    int n_seg_slots = 0;
    bool grid = false;
} g_dump;

int64_t env_i64(const char* name, int64_t dflt)
{
    const char* e = std::getenv(name);
    return (e && *e) ? std::atoll(e) : dflt;
}

}  // namespace

// ---------------------------------------------------------------------------
// A part prepared on one device: every device array lives in one allocation,
// filled by one H2D from one pinned staging image.
struct Part {
    Device* dev = nullptr;
    PartSpec spec;
    int64_t n = 0;          // pairs
    int64_t cells = 0;
    int Hmax = 0;
    struct Cls {
        int W = 16;
        int n = 0;
        int ring_len = 0;
        int* d_order = nullptr;
    } cls[2];
    int n_lane = 0;
    int n_seg_waves = 0;
    int lane_waves = 0;
    int lane_variant = 0;
    int* d_lane_order = nullptr;
    LaneWave* d_lane_waves = nullptr;
    float2* d_carry = nullptr;
    PairDesc* d_pairs = nullptr;
    uint32_t* d_rows = nullptr;
    uint32_t* d_hapw = nullptr;
    float* d_raw32 = nullptr;     // current output targets (own or bound)
    double* d_raw64 = nullptr;
    uint8_t* d_flag = nullptr;
    float* own_raw32 = nullptr;   // outputs in the part's allocation: [raw32 | raw64 | flag]
    double* own_raw64 = nullptr;
    uint8_t* own_flag = nullptr;
    size_t res_bytes = 0;         // bytes of that contiguous output block
    size_t res_o64 = 0, res_ofl = 0;
    int* d_list = nullptr;
    int* d_sorted = nullptr;
    int* d_big = nullptr;
    int* d_big_count = nullptr;
    Seg64Plan* d_plan = nullptr;
    int64_t n_wide = 0;
    int* d_count = nullptr;
    int inker_limit = 0;   // in-wave rescues allowed in the last run
    int parity = 0;
    char* dev_base = nullptr;
    Slot* slot = nullptr;         // borrowed workspace (jobs), else dev_base is owned
    char* host_res = nullptr;     // pinned results image (slot) after the D2H
    size_t upload_bytes = 0;
    hipEvent_t pack_ev[2] = {nullptr, nullptr};
    hipEvent_t done = nullptr;    // jobs: D2H complete
    std::vector<std::array<hipEvent_t, 3>> ev_pool;
    size_t ev_used = 0;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool slot_ev = false;         // pack_ev / ev / done are the slot's (not destroyed here)
    hipStream_t stream = nullptr;             // the part's stream: its slot's, else its device's
    hipStream_t side = nullptr;               // segmented waves beside one-lane waves
    hipEvent_t fork = nullptr, join = nullptr;
    hipStream_t last_stream = nullptr;
    int64_t launch_waves = 0;
    bool ran = false;
};

struct hc_phmm_batch {
    std::vector<Part*> parts;   // one per device slot
    int64_t n = 0;
};

struct hc_phmm_job {
    std::vector<Part*> parts;
    Outputs out;
    std::vector<double> cells_per_part;
};

namespace {

constexpr int kW64Threshold = 768;     // anti-diagonal kernel: H above this -> one pair per wave
constexpr int kLaneMaxH = 4096;        // longer haps stay on the anti-diagonal kernel (policy "auto")
constexpr size_t kRowPadBefore = 256;     // words of slack before the packed rows (run_seg prefetch)
constexpr int kSegWavesPerSimd = 3;    // resident seg waves per SIMD (phmm_seg_kernel occupancy)

int lane_variant_id() { return int(env_i64("HC_PHMM_LANE_VARIANT", 0)); }

// HC_PHMM_LANE_SEG = auto (default) | all | off. Returns -1 auto, 0 off, 1 all.
int lane_seg_policy()
{
    const char* e = std::getenv("HC_PHMM_LANE_SEG");
    if (!e || !*e || !std::strcmp(e, "auto")) return -1;
    return std::strcmp(e, "all") ? 0 : 1;
}

// HC_PHMM_KERNEL = auto (lane kernels for H <= kLaneMaxH) | lane | diag.
int kernel_policy()
{
    const char* e = std::getenv("HC_PHMM_KERNEL");
    if (!e || !*e || !std::strcmp(e, "auto")) return 0;
    if (!std::strcmp(e, "lane")) return 1;
    return 2;
}

void free_part(Part* p)
{
    if (!p) return;
    if (p->dev) (void)hipSetDevice(p->dev->ordinal);
    if (p->slot) give_slot(p->slot);
    else if (p->dev_base) (void)hipFree(p->dev_base);
    if (!p->slot_ev) {
        for (auto& t : p->ev_pool)
            for (auto& e : t) (void)hipEventDestroy(e);
        for (auto& e : p->pack_ev)
            if (e) (void)hipEventDestroy(e);
        if (p->done) (void)hipEventDestroy(p->done);
    }
    delete p;
}

// LSD radix sort of `idx` by a 32-bit key, DESCENDING, stable (fallback of
// the counting sort when the key range is wide).
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

// Stable parallel counting sort of `idx` by bucket(p) DESCENDING, buckets < nb.
template <typename B>
void counting_sort_desc(std::vector<int>& idx, std::vector<int>& out, std::vector<int64_t>& hist, int nb, B bucket)
{
    const int64_t n = int64_t(idx.size());
    if (n < 2) return;
    const int T = int(std::min<int64_t>(64, std::max<int64_t>(1, n / 8192)));
    const int64_t chunk = (n + T - 1) / T;
    hist.assign(size_t(T) * nb, 0);
    WorkerPool::get().run(T, [&](int t) {
        int64_t* h = hist.data() + size_t(t) * nb;
        for (int64_t k = t * chunk, e = std::min(n, k + chunk); k < e; ++k) ++h[bucket(idx[k])];
    });
    int64_t run = 0;
    for (int b = nb - 1; b >= 0; --b)
        for (int t = 0; t < T; ++t) {
            int64_t& h = hist[size_t(t) * nb + b];
            const int64_t c = h;
            h = run;
            run += c;
        }
    out.resize(size_t(n));
    WorkerPool::get().run(T, [&](int t) {
        int64_t* h = hist.data() + size_t(t) * nb;
        for (int64_t k = t * chunk, e = std::min(n, k + chunk); k < e; ++k) out[h[bucket(idx[k])]++] = idx[k];
    });
    idx.swap(out);
}

// Parallel exclusive prefix sum of f(k), k in [0, n), into out[0..n].
template <typename F>
void prefix_sum(int64_t n, std::vector<int64_t>& out, F f)
{
    out.assign(size_t(n) + 1, 0);
    if (n <= 0) return;
    const int T = int(std::min<int64_t>(32, std::max<int64_t>(1, n / 16384)));
    const int64_t chunk = (n + T - 1) / T;
    std::vector<int64_t> part(static_cast<size_t>(T) + 1, 0);
    WorkerPool::get().run(T, [&](int t) {
        int64_t s = 0;
        for (int64_t k = t * chunk, e = std::min(n, k + chunk); k < e; ++k) {
            out[size_t(k) + 1] = s += f(k);
        }
        part[size_t(t) + 1] = s;
    });
    for (int t = 1; t <= T; ++t) part[size_t(t)] += part[size_t(t) - 1];
    WorkerPool::get().run(T, [&](int t) {
        const int64_t add = part[size_t(t)];
        if (add)
            for (int64_t k = t * chunk, e = std::min(n, k + chunk); k < e; ++k) out[size_t(k) + 1] += add;
    });
}

// Bump allocator over one region: 256-B aligned segments.
struct Layout {
    size_t off = 0;
    size_t take(size_t bytes)
    {
        const size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    }
};

// Whether a read's (i, d, c) gap qualities are the same on every row (then
// they travel once, in its descriptor). Blocks of 64 rows without early exit
// inside a block, so the compiler vectorises the compare.
bool constant_gaps(const ReadView& v)
{
    const uint8_t i0 = v.i[0], d0 = v.d[0], c0 = v.c[0];
    int k = 0;
    for (; k + 64 <= v.len; k += 64) {
        uint8_t a = 0;
        for (int j = 0; j < 64; ++j) a |= uint8_t((v.i[k + j] ^ i0) | (v.d[k + j] ^ d0) | (v.c[k + j] ^ c0));
        if (a) return false;
    }
    uint8_t a = 0;
    for (; k < v.len; ++k) a |= uint8_t((v.i[k] ^ i0) | (v.d[k] ^ d0) | (v.c[k] ^ c0));
    return a == 0;
}

// The part's reads / haps in part-local order, and the (read, hap) of each
// part-local pair.
struct Local {
    const Src* src;
    const PartSpec* spec;
    int64_t nr = 0, nh = 0, np = 0;
    std::vector<int64_t> blk_r, blk_h, blk_p;   // per block: first local read / hap / pair

    Local(const Src& s, const PartSpec& p) : src(&s), spec(&p)
    {
        if (p.flat) {
            nr = nh = np = p.hi - p.lo;
            return;
        }
        for (const Block& b : p.blocks) {
            blk_r.push_back(nr);
            blk_h.push_back(nh);
            blk_p.push_back(np);
            nr += b.nr;
            nh += b.nh;
            np += int64_t(b.nr) * b.nh;
        }
        blk_p.push_back(np);
    }
    int64_t read_id(int64_t lr) const   // Src read index of local read lr
    {
        if (spec->flat) return spec->lo + lr;
        const size_t b = size_t(std::upper_bound(blk_r.begin(), blk_r.end(), lr) - blk_r.begin()) - 1;
        return spec->blocks[b].r0 + (lr - blk_r[b]);
    }
    int64_t hap_mult(int64_t lh) const   // reads paired with local hap lh
    {
        if (spec->flat) return 1;
        const size_t b = size_t(std::upper_bound(blk_h.begin(), blk_h.end(), lh) - blk_h.begin()) - 1;
        return spec->blocks[b].nr;
    }
    int64_t hap_id(int64_t lh) const
    {
        if (spec->flat) return spec->lo + lh;
        const size_t b = size_t(std::upper_bound(blk_h.begin(), blk_h.end(), lh) - blk_h.begin()) - 1;
        return spec->blocks[b].h0 + (lh - blk_h[b]);
    }
    // f(k, local read, local hap) for pairs k in [lo, hi).
    template <typename F>
    void pairs(int64_t lo, int64_t hi, F&& f) const
    {
        if (lo >= hi) return;
        if (spec->flat) {
            for (int64_t k = lo; k < hi; ++k) f(k, k, k);
            return;
        }
        size_t b = size_t(std::upper_bound(blk_p.begin(), blk_p.end(), lo) - blk_p.begin()) - 1;
        int64_t k = lo;
        while (k < hi) {
            const Block& B = spec->blocks[b];
            const int64_t base = blk_p[b], end = std::min(hi, blk_p[b + 1]);
            int64_t r = (k - base) / B.nh, h = (k - base) % B.nh;
            for (; k < end; ++k) {
                f(k, blk_r[b] + r, blk_h[b] + h);
                if (++h == B.nh) {
                    h = 0;
                    ++r;
                }
            }
            ++b;
        }
    }
};

// A hap's two segmented-wave candidates: nb0 = ceil(H / cap) lanes or one more,
// each with the narrowest compiled width covering H.
struct Cand {
    uint8_t bc[2], nb[2];
};
static_assert(sizeof(Cand) == sizeof(uint32_t), "Cand packs into a word");

// A structured plan's segment tables for the device (launch_grid_waves).
struct GridDev {
    std::vector<GridSeg> segs;
    std::vector<int> rord, hord;
    int64_t slots = 0, waves = 0;
};

// Grow-only per-thread scratch of the planner: fresh large vectors would be
// fresh mmap'd pages, zero-filled by the kernel on first touch, every call.
struct PlanScratch {
    std::vector<int32_t> rlen, gapw, hlen;
    std::vector<int64_t> row_off, gap_off, hap_w, hap_b;
    std::vector<uint8_t> hcls, cls, seg_bc, seg_nb, used, in_tail;
    std::vector<uint32_t> srec;   // (BC, nb, R) of the segmented pairs in sorted order
    std::vector<uint32_t> hcand, key;
    std::vector<Cand> ctab;
    GridDev gdev;
    std::vector<int> seg_in, one_ord, ord2[2], seg_ord, sort_tmp;
    std::vector<LaneWave> lw, ordered;
    std::vector<int64_t> wcost;
    std::vector<uint64_t> wkey;
    std::vector<std::vector<LaneWave>> part_w;
    std::vector<int64_t> hist;
};
thread_local PlanScratch t_scr;

template <typename T>
void grow(std::vector<T>& v, size_t n)
{
    if (v.size() < n) v.resize(n);
}


// Modelled wave instructions of nb lanes of bc columns over R rows: 13 per
// column + 26 per step, R + nb - 1 steps, times the lane-waste weight.
inline float seg_cost(int nb, int bc, int R, const float* waste)
{
    return float(nb * (13 * bc + 26) * (R + nb - 1)) * waste[nb];
}

// Cross-product fast path of the planner (regions: hc_phmm_cross,
// cross_regions, submit_regions) when every hap takes segmented waves. The
// pairs of a block are reads x haps, so their sorted order need not be found
// by sorting pairs: each hap takes one (BC, nb) candidate (chosen at its
// block's mean read length), the block's haps are grouped by (BC, nb) and its
// reads sorted by R, and a group's pairs in (read by R descending) x (hap)
// order fill waves of floor(64 / nb) pairs — the order the general planner's
// sort + greedy packing reaches on such a batch, built in one parallel pass
// over segments (one per block and group; a segment's last wave may be
// partial). Segments run widest block first, so co-resident waves share a
// width's code. Writes every pair's descriptor, the slot order and the waves;
// returns the batch's cells.
int64_t plan_grid(const Local& loc, const int32_t* rlen, const int32_t* hlen, const int64_t* row_off,
                  const int64_t* hap_w, const Cand* hcand, const float* waste, int qforce, PairDesc* pd,
                  bool write_pairs, std::vector<int>& seg_ord, std::vector<LaneWave>& lw, PhaseTimer& tm,
                  GridDev* gd)
{
    const PartSpec& spec = *loc.spec;
    const size_t nblk = spec.blocks.size();
    // Per block: reads by R descending, haps grouped by their (BC, nb) key.
    std::vector<int> rord(size_t(loc.nr)), hord(size_t(loc.nh));
    std::vector<uint16_t> hkey(size_t(loc.nh));
    struct Seg {
        uint32_t key;   // bc << 8 | nb
        int blk;
        int g0, G;      // haps hord[g0 .. g0 + G) (local ids)
        int64_t n, slot0, w0;
    };
    std::vector<std::vector<Seg>> bsegs(nblk);
    parallel_for(int64_t(nblk), [&](int64_t lo, int64_t hi) {
        for (int64_t b = lo; b < hi; ++b) {
            const Block& B = spec.blocks[size_t(b)];
            const int64_t r0 = loc.blk_r[size_t(b)], h0 = loc.blk_h[size_t(b)];
            int64_t rs = 0;
            for (int r = 0; r < B.nr; ++r) {
                rord[size_t(r0 + r)] = int(r0 + r);
                rs += rlen[r0 + r];
            }
            std::stable_sort(rord.begin() + r0, rord.begin() + r0 + B.nr,
                             [&](int x, int y) { return rlen[x] > rlen[y]; });
            const int Rm = int((rs + B.nr / 2) / std::max(1, B.nr));
            for (int h = 0; h < B.nh; ++h) {
                const int lh = int(h0 + h);
                const Cand cd = hcand[lh];
                const int q = qforce >= 0 ? qforce
                              : seg_cost(cd.nb[1], cd.bc[1], Rm, waste) < seg_cost(cd.nb[0], cd.bc[0], Rm, waste) ? 1
                                                                                                                 : 0;
                hkey[size_t(lh)] = uint16_t(cd.bc[q] << 8 | cd.nb[q]);
                hord[size_t(lh)] = lh;
            }
            std::stable_sort(hord.begin() + h0, hord.begin() + h0 + B.nh,
                             [&](int x, int y) { return hkey[size_t(x)] > hkey[size_t(y)]; });
            auto& out = bsegs[size_t(b)];
            out.clear();
            for (int g = 0; g < B.nh;) {
                const uint16_t k = hkey[size_t(hord[size_t(h0 + g)])];
                int e = g;
                while (e < B.nh && hkey[size_t(hord[size_t(h0 + e)])] == k) ++e;
                out.push_back(Seg{k, int(b), int(h0 + g), e - g, int64_t(B.nr) * (e - g), 0, 0});
                g = e;
            }
        }
    }, 1);
    tm.mark("grid: blocks");
    std::vector<Seg> segs;
    for (auto& v : bsegs) segs.insert(segs.end(), v.begin(), v.end());
    std::stable_sort(segs.begin(), segs.end(), [](const Seg& x, const Seg& y) { return x.key > y.key; });
    int64_t slots = 0, waves = 0;
    for (Seg& g : segs) {
        g.slot0 = slots;
        g.w0 = waves;
        slots += g.n;
        waves += (g.n + 64 / int(g.key & 0xff) - 1) / (64 / int(g.key & 0xff));
    }
    if (gd) {   // order and waves built on the device from the segments (launch_grid_waves)
        gd->slots = slots;
        gd->waves = waves;
        gd->segs.resize(segs.size());
        for (size_t k = 0; k < segs.size(); ++k) {
            const Seg& g = segs[k];
            const Block& B = spec.blocks[size_t(g.blk)];
            gd->segs[k] = GridSeg{g.slot0, loc.blk_p[size_t(g.blk)], int(g.w0), int(loc.blk_r[size_t(g.blk)]), B.nr,
                                  B.nh, int(loc.blk_h[size_t(g.blk)]), g.g0, g.G, int(g.key >> 8),
                                  int(g.key & 0xff), 0};
        }
        gd->rord.swap(rord);
        gd->hord.swap(hord);
        seg_ord.clear();
        lw.clear();
    } else {
    seg_ord.resize(size_t(slots));
    lw.resize(size_t(waves));
    parallel_for(int64_t(segs.size()), [&](int64_t lo, int64_t hi) {
        for (int64_t t = lo; t < hi; ++t) {
            const Seg& g = segs[size_t(t)];
            const Block& B = spec.blocks[size_t(g.blk)];
            const int64_t r0 = loc.blk_r[size_t(g.blk)], h0 = loc.blk_h[size_t(g.blk)], p0 = loc.blk_p[size_t(g.blk)];
            const int bc = int(g.key >> 8), nb = int(g.key & 0xff), per = 64 / nb;
            int* o = seg_ord.data() + g.slot0;
            int64_t i = 0;
            for (int rr = 0; rr < B.nr; ++rr) {
                const int64_t rowbase = p0 + (rord[size_t(r0 + rr)] - r0) * int64_t(B.nh) - h0;
                for (int hh = 0; hh < g.G; ++hh) o[i++] = int(rowbase + hord[size_t(g.g0 + hh)]);
            }
            for (int64_t w = 0; w * per < g.n; ++w) {
                const int64_t a = w * per, e = std::min(g.n, a + per);
                const int Rmax = rlen[rord[size_t(r0 + a / g.G)]];
                const int Rmin = rlen[rord[size_t(r0 + (e - 1) / g.G)]];
                LaneWave v{};
                v.slot0 = int(g.slot0 + a);
                v.ncols = bc;
                v.npairs = int(e - a);
                v.rmax = Rmax;
                v.rmin = Rmin;
                v.nsteps = Rmax + nb - 1;
                lw[size_t(g.w0 + w)] = v;
            }
        }
    }, 1);
    }   // host order and waves
    tm.mark("grid: slots + waves");
    if (!write_pairs) {   // descriptors built on the device (launch_grid_pairs): cells from block sums
        int64_t cells = 0;
        for (size_t b = 0; b < nblk; ++b) {
            const Block& B = spec.blocks[b];
            int64_t sr = 0, sh = 0;
            for (int r = 0; r < B.nr; ++r) sr += rlen[loc.blk_r[b] + r];
            for (int h = 0; h < B.nh; ++h) sh += hlen[loc.blk_h[b] + h];
            cells += sr * sh;
        }
        return cells;
    }
    // Pair descriptors (read-major within each block, as Local::pairs).
    std::atomic<int64_t> cells{0};
    parallel_for(loc.np, [&](int64_t lo, int64_t hi) {
        int64_t c = 0;
        loc.pairs(lo, hi, [&](int64_t k, int64_t r, int64_t h) {
            const int R = rlen[r], H = hlen[h];
            pd[k] = PairDesc{int(row_off[r]), R, int(hap_w[h]), H};
            c += int64_t(R) * H;
        });
        cells += c;
    }, 16384);
    return cells.load();
}

// Plan one part on device d: host binning + staging, then the H2D, device
// packing and (with_run) the device pass and the D2H of the results, all
// enqueued on d's stream. slot == nullptr: the part owns its memory (batches).
int plan_part(Device& d, const Src& src, const PartSpec& spec, Slot* slot, bool with_run, Part** out);
int run_part(Part* b, hipStream_t s);

int plan_part(Device& dv, const Src& src, const PartSpec& spec, Slot* slot, bool with_run, Part** out)
{
    PhaseTimer tm;
    Local loc(src, spec);
    const int64_t nr = loc.nr, nh = loc.nh, npairs = loc.np;
    if (npairs > (int64_t(1) << 31) - 1) return fail(HC_PHMM_EINVAL, "too many pairs for one batch");

    // Reads: validate, lengths, gap-quality constancy; haps: validate, lengths.
    PlanScratch& S = t_scr;
    grow(S.rlen, size_t(nr));
    grow(S.gapw, size_t(nr));
    grow(S.hlen, size_t(nh));
    int32_t* rlen = S.rlen.data();
    int32_t* gapw = S.gapw.data();
    int32_t* hlen = S.hlen.data();
    std::atomic<int> bad_read{0}, bad_hap{0}, rlen_max{0};
    parallel_for(nr, [&](int64_t lo, int64_t hi) {
        int rm = 0;
        for (int64_t r = lo; r < hi; ++r) {
            const ReadView v = src.read(loc.read_id(r));
            if (v.len <= 0 || v.len > HC_PHMM_MAX_READ_LEN || !v.bases || !v.q || !v.i || !v.d || !v.c) {
                bad_read.store(1);
                rlen[size_t(r)] = 0;
                gapw[size_t(r)] = 0;
                continue;
            }
            rlen[size_t(r)] = v.len;
            rm = std::max(rm, v.len);
            gapw[size_t(r)] = constant_gaps(v) ? int32_t((v.i[0] & 127) | ((v.d[0] & 127) << 7) | ((v.c[0] & 127) << 14))
                                               : -1;
        }
        int cur = rlen_max.load();
        while (rm > cur && !rlen_max.compare_exchange_weak(cur, rm)) {
        }
    }, 2048);
    if (bad_read.load()) return fail(HC_PHMM_EINVAL, "read with invalid length or null array");
    parallel_for(nh, [&](int64_t lo, int64_t hi) {
        for (int64_t h = lo; h < hi; ++h) {
            const HapView v = src.hapv(loc.hap_id(h));
            const bool ok = v.len > 0 && v.len <= HC_PHMM_MAX_HAP_LEN && v.bases;
            if (!ok) bad_hap.store(1);
            hlen[size_t(h)] = ok ? v.len : 0;
        }
    }, 8192);
    if (bad_hap.load())
        return fail(HC_PHMM_EINVAL, "haplotype with invalid length (1.." + std::to_string(HC_PHMM_MAX_HAP_LEN) +
                                        ") or null bases");
    // rows / irregular gap rows / table words / hap bytes
    std::vector<int64_t>&row_off = S.row_off, &gap_off = S.gap_off, &hap_w = S.hap_w, &hap_b = S.hap_b;
    prefix_sum(nr, row_off, [&](int64_t r) -> int64_t { return rlen[size_t(r)]; });
    prefix_sum(nr, gap_off, [&](int64_t r) -> int64_t { return gapw[size_t(r)] < 0 ? rlen[size_t(r)] : 0; });
    prefix_sum(nh, hap_w, [&](int64_t h) -> int64_t { return hap_table_words(hlen[size_t(h)]); });
    prefix_sum(nh, hap_b, [&](int64_t h) -> int64_t { return hlen[size_t(h)]; });
    const int64_t nrows = row_off[size_t(nr)], ngap = gap_off[size_t(nr)];
    if (nrows > INT32_MAX || hap_w[size_t(nh)] > INT32_MAX || hap_b[size_t(nh)] > INT32_MAX || ngap > INT32_MAX)
        return fail(HC_PHMM_EINVAL, "batch too large (row or hap pool exceeds 2^31)");
    tm.mark("reads/haps scan");

    // Staging layout (upload part first; waves last, their count is known later).
    Layout U;
    const size_t o_pairs = U.take(sizeof(PairDesc) * size_t(npairs));
    const size_t o_rd = U.take(sizeof(int4) * size_t(nr));
    const size_t o_hd = U.take(sizeof(int4) * size_t(nh));
    const size_t o_ord = U.take(sizeof(int) * size_t(npairs));
    const size_t o_bases = U.take(size_t(nrows) + 16);
    const size_t o_quals = U.take(size_t(nrows) + 16);
    const size_t gap_stride = (size_t(ngap) + 16 + 15) & ~size_t(15);
    const size_t o_gaps = U.take(ngap ? 3 * gap_stride : 0);
    const size_t o_hb = U.take(size_t(hap_b[size_t(nh)]) + 16);
    const size_t o_lw = U.off;   // LaneWave array, sized after packing

    // Pinned staging: upper bound for the waves (one per seg pair at most, plus
    // one-lane waves) and the results image after the upload.
    const size_t waves_max = sizeof(LaneWave) * (size_t(npairs) + 1) + sizeof(GridBlock) * spec.blocks.size() +
                             sizeof(GridSeg) * size_t(nh) + sizeof(int) * size_t(nr + nh) + 1024;
    const size_t n1 = size_t(std::max<int64_t>(npairs, 1));
    const size_t res_o64 = (sizeof(float) * n1 + 255) & ~size_t(255);
    const size_t res_ofl = res_o64 + ((sizeof(double) * n1 + 255) & ~size_t(255));
    const size_t res_bytes = res_ofl + n1;
    const size_t host_upload_cap = o_lw + waves_max;
    const size_t host_res_off = (host_upload_cap + 255) & ~size_t(255);
    char* host = nullptr;
    bool own_host = false;
    static std::vector<char> dry_host;   // g_dry: plain memory, one planner at a time
    if (g_dry) {
        if (dry_host.size() < host_res_off + res_bytes) dry_host.resize(host_res_off + res_bytes);
        host = dry_host.data();
    } else if (slot) {
        const int rc = slot_reserve(*slot, 0, host_res_off + res_bytes);
        if (rc) return rc;
        host = slot->host;
    } else {
        if (hipHostMalloc(&host, std::max<size_t>(host_upload_cap, 1), hipHostMallocPortable) != hipSuccess)
            return fail(HC_PHMM_ENOMEM, "pinned staging buffer");
        own_host = true;
    }
    struct HostGuard {
        char* p;
        bool own;
        ~HostGuard()
        {
            if (own && p) (void)hipHostFree(p);
        }
    } hguard{host, own_host};
    tm.mark("staging alloc");

    // Per hap: kernel class, lanes at each width cap (times the reads it pairs
    // with), then the pass's cap and the hap's two (BC, nb) candidates.
    PairDesc* pd = reinterpret_cast<PairDesc*>(host + o_pairs);
    const int pol = kernel_policy();
    const bool use_lane = pol != 2;
    const int seg_max_h = lane_seg_policy() == 0 ? 0 : 64 * kSegMaxBC;
    constexpr int kNCaps = 7;
    constexpr int kCaps[kNCaps] = {64, 48, 32, 24, 16, 12, 8};
    // class: 0 seg, 1 one-lane, 2 diag W16, 3 diag W64
    grow(S.hcls, size_t(nh));
    uint8_t* hcls = S.hcls.data();
    std::array<std::atomic<int64_t>, kNCaps> lanes_at{};
    for (auto& x : lanes_at) x = 0;
    std::atomic<int64_t> wide_a{0};
    std::atomic<int> hmax_a{0};
    // seg_width_ceil as a table (the planner calls it per hap and cap).
    static const std::array<int8_t, kSegMaxBC + 1> kWidthCeil = [] {
        std::array<int8_t, kSegMaxBC + 1> t{};
        for (int x = 0; x <= kSegMaxBC; ++x) t[size_t(x)] = int8_t(seg_width_ceil(x));
        return t;
    }();
    // Modelled wave instructions at each cap (13 per column + ~30 per step,
    // R + nb - 1 steps at the batch's mean read length), for the cap choice.
    const double ravg = double(nrows) / double(std::max<int64_t>(nr, 1));
    std::mutex work_mu;
    std::array<double, kNCaps> work_at{};
    // The cap model needs only totals: past 8k haps it prices every stride-th
    // hap (weighted by the stride), which is all the cap choice can resolve.
    const int64_t cap_stride = std::max<int64_t>(1, nh / 8192);
    parallel_for(nh, [&](int64_t lo, int64_t hi) {
        int64_t w = 0;
        int hm = 0;
        const int32_t* __restrict hl = hlen;
        uint8_t* __restrict hc = hcls;
        for (int64_t h = lo; h < hi; ++h) {
            const int H = hl[h];
            int cl;
            if (use_lane && (pol == 1 || H <= kLaneMaxH))
                cl = H > seg_max_h ? 1 : 0;
            else
                cl = H > kW64Threshold ? 3 : 2;
            hc[h] = uint8_t(cl);
            hm = std::max(hm, H);
            w += H > 64 * 32 ? loc.hap_mult(h) : 0;
        }
        wide_a += w;
        int cur = hmax_a.load();
        while (hm > cur && !hmax_a.compare_exchange_weak(cur, hm)) {
        }
    }, 1 << 14);
    parallel_for((nh + cap_stride - 1) / cap_stride, [&](int64_t lo, int64_t hi) {
        int64_t lanes[kNCaps] = {};
        double work[kNCaps] = {};
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t h = i * cap_stride;
            if (hcls[size_t(h)] != 0) continue;
            const int H = hlen[size_t(h)];
            const int64_t m = cap_stride * loc.hap_mult(h);
            for (int q = 0; q < kNCaps; ++q) {
                const int nbq = std::min(64, (H + kCaps[q] - 1) / kCaps[q]);
                const int bc = kWidthCeil[size_t(std::min(kSegMaxBC, (H + nbq - 1) / nbq))];
                const int nb = (H + bc - 1) / bc;
                lanes[q] += m * nb;
                work[q] += double(m) * nb * (ravg + nb - 1) * (13.0 * bc + 30.0);
            }
        }
        for (int q = 0; q < kNCaps; ++q) lanes_at[q] += lanes[q];
        std::lock_guard<std::mutex> lk(work_mu);
        for (int q = 0; q < kNCaps; ++q) work_at[size_t(q)] += work[q];
    }, 4096);
    tm.mark("hap classes: cost");
    int cap = kSegMaxBC;
    bool few_waves = false;   // the pass gives each SIMD at most ~3 waves: latency-bound, prefer more lanes
    {
        const int64_t forced = env_i64("HC_PHMM_SEG_CAP", 0);
        if (forced > 0) {
            cap = int(std::max<int64_t>(kSegMinBC, std::min<int64_t>(kSegMaxBC, forced)));
        } else if (lanes_at[0].load() > 0) {
            const double simds = 4.0 * dv.n_cu;
            double best = 0;
            for (int c = 0; c < kNCaps; ++c) {
                const double waves = double(lanes_at[c].load()) / 60.0;   // ~60 of 64 lanes filled
                // Up to two rounds of resident waves (3 per SIMD): the SIMD with
                // the most waves sets the time, its last round issuing at half
                // rate if it holds one wave (n waves: 3 floor(n/3) + {0, 2, 2}).
                // More rounds: waves start as slots free up, so the pass time
                // follows the total work (a ceil() there once picked cap 48 for
                // a 415 x 128 region: 1.05 ms vs 0.94 at cap 64).
                const double per_simd = waves / simds;
                double rounds = per_simd;
                if (per_simd <= 6.0) {
                    const int n = std::max(1, int(std::ceil(per_simd - 1e-9)));
                    rounds = 3.0 * (n / 3) + (n % 3 ? 2.0 : 0.0);
                }
                const double est = rounds * work_at[size_t(c)] / 60.0 / waves;
                if (c == 0 || est < best * 0.98) {
                    best = est;
                    cap = kCaps[c];
                    few_waves = waves <= 3.0 * simds;
                }
            }
        }
    }
    static const std::array<float, 65> kHalfWaste = [] {
        std::array<float, 65> f{};
        for (int nb = 1; nb <= 64; ++nb) f[size_t(nb)] = std::sqrt(64.f / float((64 / nb) * nb));
        return f;
    }();
    // A pass with few waves per SIMD is latency-bound: its time is one wave's,
    // so the candidate with the shorter wave wins there (S1: 11 lanes of 14
    // columns beat 10 of 16; S1w: 12 of 22 beat 11 of 24).
    static const std::array<float, 65> kPerLane = [] {
        std::array<float, 65> f{};
        for (int nb = 1; nb <= 64; ++nb) f[size_t(nb)] = 1.f / float(nb);
        return f;
    }();
    const float* waste = few_waves ? kPerLane.data() : kHalfWaste.data();
    grow(S.hcand, size_t(nh));
    Cand* hcand = reinterpret_cast<Cand*>(S.hcand.data());
    auto cand_of = [&](int H) {
        const int nb0 = std::min(64, (H + cap - 1) / cap);
        Cand c{};
        for (int q = 0; q < 2; ++q) {
            const int nb = std::min(nb0 + q, 64);
            const int bc = kWidthCeil[size_t(std::min(kSegMaxBC, (H + nb - 1) / nb))];
            c.bc[q] = uint8_t(bc);
            c.nb[q] = uint8_t((H + bc - 1) / bc);
        }
        return c;
    };
    // Many haps (flat batches: one per pair): the candidates by H from a table
    // (divisions once per length, not per hap).
    const int hmax_seg = std::min(hmax_a.load(), seg_max_h);
    std::vector<Cand>& ctab = S.ctab;
    const bool by_table = nh > 4 * int64_t(hmax_seg + 1);
    if (by_table) {
        ctab.resize(size_t(hmax_seg) + 1);
        for (int H = 1; H <= hmax_seg; ++H) ctab[size_t(H)] = cand_of(H);
    }
    parallel_for(nh, [&](int64_t lo, int64_t hi) {
        for (int64_t h = lo; h < hi; ++h) {
            if (hcls[size_t(h)] != 0) continue;
            const int H = hlen[size_t(h)];
            hcand[size_t(h)] = by_table ? ctab[size_t(H)] : cand_of(H);
        }
    }, 1 << 14);
    tm.mark("hap classes");

    std::atomic<int64_t> cells_a{0};
    std::vector<int>&one_ord = S.one_ord, (&ord2)[2] = S.ord2;
    std::vector<int>& seg_ord = S.seg_ord;
    std::vector<LaneWave>& lw = S.lw;
    lw.clear();
    const int qforce = int(env_i64("HC_PHMM_SEG_Q", -1));   // sweeps: force the nb0 (0) or nb0 + 1 (1) candidate
    // Cross products whose haps all take segmented waves (every region call):
    // the structured planner (plan_grid); HC_PHMM_GRID_PLAN=0 forces the
    // general one (A/B, tests).
    bool grid = !spec.flat && env_i64("HC_PHMM_GRID_PLAN", 1) != 0;
    for (int64_t h = 0; grid && h < nh; ++h) grid = hcls[size_t(h)] == 0;
    // Structured plans outside dry runs: pair descriptors, slot order and waves
    // are built on the device from the block and segment tables.
    const bool dev_plan = grid && !g_dry;
    GridDev& gd = S.gdev;
    if (grid) {
        one_ord.clear();
        ord2[0].clear();
        ord2[1].clear();
        cells_a = plan_grid(loc, rlen, hlen, row_off.data(), hap_w.data(), hcand, waste, qforce, pd, !dev_plan, seg_ord, lw, tm,
                            dev_plan ? &gd : nullptr);
        tm.mark("grid: pairs");
    } else {
        // Per pair: descriptor straight into the staging image, class, and for
        // segmented pairs the cheaper candidate for its R.
        grow(S.cls, size_t(npairs));
        grow(S.seg_bc, size_t(npairs));
        grow(S.seg_nb, size_t(npairs));
        uint8_t *cls = S.cls.data(), *seg_bc = S.seg_bc.data(), *seg_nb = S.seg_nb.data();
        std::atomic<int> rmin_a{INT32_MAX}, rmax_a{0};
        // Pairs per planning task (a 415 x 128 region call on the GPU box: 2.0 ms
        // at 8192, 2.96 ms on one task; tools/region_ab.py).
        const int64_t task_pairs = std::max<int64_t>(1024, env_i64("HC_PHMM_TASK_PAIRS", 8192));
        const int T = int(std::min<int64_t>(64, std::max<int64_t>(1, npairs / task_pairs)));
        const int64_t pchunk = (npairs + T - 1) / T;
        std::vector<std::array<int64_t, 4>> tcnt(size_t(T) + 1);
        WorkerPool::get().run(T, [&](int t) {
            const int64_t lo = t * pchunk, hi = std::min(npairs, lo + pchunk);
            // Plain restrict locals: the uint8_t stores below may alias anything,
            // so anything reached through a capture would be reloaded per pair.
            const int32_t* __restrict rl = rlen;
            const int32_t* __restrict hl = hlen;
            const int64_t* __restrict ro = row_off.data();
            const int64_t* __restrict hw = hap_w.data();
            const uint8_t* __restrict hc = hcls;
            const Cand* __restrict cand = hcand;
            PairDesc* __restrict pdo = pd;
            uint8_t* __restrict clo = cls;
            uint8_t* __restrict bco = seg_bc;
            uint8_t* __restrict nbo = seg_nb;
            int64_t c = 0, cn0 = 0, cn1 = 0, cn2 = 0, cn3 = 0;
            int rlo = INT32_MAX, rhi = 0;
            auto one = [=, &c, &cn0, &cn1, &cn2, &cn3, &rlo, &rhi](int64_t k, int64_t r, int64_t h) {
                const int R = rl[r], H = hl[h];
                pdo[k] = PairDesc{int(ro[r]), R, int(hw[h]), H};
                c += int64_t(R) * H;
                const int cl = hc[h];
                clo[k] = uint8_t(cl);
                if (cl == 0) {
                    ++cn0;
                    const Cand cd = cand[h];
                    // modelled wave instructions: nb lanes x (13 per column + 26 per
                    // step) x (R + nb - 1) steps, times half the lane waste of a
                    // wave of such pairs alone (floor(64 / nb) groups): uniform
                    // batches pack like that, mixed ones fill the gaps with others;
                    // with few waves, the wave's own time (per lane)
                    auto cost = [&](int q) {
                        const int nb = cd.nb[q];
                        return float(nb * (13 * cd.bc[q] + 26) * (R + nb - 1)) * waste[nb];
                    };
                    const int q = qforce >= 0 ? qforce : cost(1) < cost(0) ? 1 : 0;
                    bco[k] = cd.bc[q];
                    nbo[k] = cd.nb[q];
                    rlo = R < rlo ? R : rlo;
                    rhi = R > rhi ? R : rhi;
                } else {
                    cn1 += cl == 1;
                    cn2 += cl == 2;
                    cn3 += cl == 3;
                }
            };
            if (spec.flat) {
                for (int64_t k = lo; k < hi; ++k) one(k, k, k);
            } else {
                loc.pairs(lo, hi, one);
            }
            cells_a += c;
            tcnt[size_t(t) + 1] = {cn0, cn1, cn2, cn3};
            int cur = rmin_a.load();
            while (rlo < cur && !rmin_a.compare_exchange_weak(cur, rlo)) {
            }
            cur = rmax_a.load();
            while (rhi > cur && !rmax_a.compare_exchange_weak(cur, rhi)) {
            }
        });
        // Stable split of the pairs by class (per-task offsets, parallel scatter).
        std::array<int64_t, 4> cls_tot{};
        for (int t = 1; t <= T; ++t)
            for (int q = 0; q < 4; ++q) {
                const int64_t v = tcnt[size_t(t)][size_t(q)];
                tcnt[size_t(t)][size_t(q)] = cls_tot[size_t(q)];
                cls_tot[size_t(q)] += v;
            }
        std::vector<int>& seg_in = S.seg_in;
        seg_in.resize(size_t(cls_tot[0]));
        one_ord.resize(size_t(cls_tot[1]));
        ord2[0].resize(size_t(cls_tot[2]));
        ord2[1].resize(size_t(cls_tot[3]));
        WorkerPool::get().run(T, [&](int t) {
            int* dst[4] = {seg_in.data(), one_ord.data(), ord2[0].data(), ord2[1].data()};
            int64_t pos[4];
            for (int q = 0; q < 4; ++q) pos[q] = tcnt[size_t(t) + 1][size_t(q)];
            for (int64_t k = t * pchunk, e = std::min(npairs, k + pchunk); k < e; ++k) {
                const int q = cls[size_t(k)];
                dst[q][pos[q]++] = int(k);
            }
        });
        tm.mark("pairs");
        if (!seg_in.empty()) {
            const int rlo = rmin_a.load(), rspan = rmax_a.load() - rlo + 1;
            const int nbk = (kSegMaxBC / 2 + 1) * rspan;
            if (nbk <= (1 << 18)) {
                counting_sort_desc(seg_in, S.sort_tmp, S.hist, nbk,
                                   [&](int p) { return (seg_bc[size_t(p)] / 2) * rspan + (pd[p].y - rlo); });
            } else {
                std::vector<uint32_t>& key = S.key;
                grow(key, size_t(npairs));
                for (int p : seg_in) key[size_t(p)] = (uint32_t(seg_bc[size_t(p)]) << 16) | uint32_t(std::min(pd[p].y, 65535));
                sort_desc(seg_in, key);
            }
        }
        tm.mark("seg sort");
        // Greedy packing in independent segments of the sorted list (one per task;
        // a segment boundary costs at most one partly filled wave).
        const int64_t ns = int64_t(seg_in.size());
        seg_ord.resize(size_t(ns));
        {
            const int T = int(std::min<int64_t>(64, std::max<int64_t>(1, ns / task_pairs)));
            const int64_t chunk = (ns + T - 1) / T;
            std::vector<std::vector<LaneWave>>& part_w = S.part_w;
            if (part_w.size() < size_t(T)) part_w.resize(size_t(T));
            for (auto& W : part_w) W.clear();
            S.used.assign(size_t(ns), 0);
            // The packing reads (BC, nb, R) of the pairs in sorted order: gather
            // them once into a sequential array (one parallel pass of random
            // reads, instead of three per look-ahead probe on one task per 16k
            // pairs: 0.3 ms of a 415 x 128 region's planning on the GPU box).
            std::vector<uint32_t>& srec = S.srec;
            grow(srec, size_t(ns));
            parallel_for(ns, [&](int64_t lo, int64_t hi) {
                for (int64_t k = lo; k < hi; ++k) {
                    const int p = seg_in[size_t(k)];
                    srec[size_t(k)] = uint32_t(seg_bc[size_t(p)]) | uint32_t(seg_nb[size_t(p)]) << 8 |
                                      uint32_t(std::min(pd[p].y, 65535)) << 16;
                }
            });
            // Smallest nb of each width in the part: a wave whose free lanes drop
            // below it cannot take another pair of its width, so its look-ahead
            // stops there (a uniform region once scanned all 64 entries per wave).
            std::array<uint8_t, kSegMaxBC + 1> minnb;
            minnb.fill(64);
            for (int64_t k = 0; k < ns; ++k) {
                uint8_t& m = minnb[srec[size_t(k)] & 0xff];
                m = std::min<uint8_t>(m, uint8_t(srec[size_t(k)] >> 8));
            }
            WorkerPool::get().run(T, [&](int t) {
                const int64_t b = t * chunk, e = std::min(ns, b + chunk);
                if (b >= e) return;
                const int64_t m = e - b;
                const int* __restrict in = seg_in.data() + b;
                const uint32_t* __restrict rec = srec.data() + b;
                int* __restrict ordo = seg_ord.data();
                uint8_t* __restrict used = S.used.data() + b;
                auto& W = part_w[size_t(t)];
                int64_t slot_n = b;
                constexpr int64_t kLook = 64;
                for (int64_t i = 0; i < m; ++i) {
                    if (used[i]) continue;
                    const int bc = int(rec[i] & 0xff);
                    LaneWave w{};
                    w.slot0 = int(slot_n);
                    w.ncols = bc;
                    int rmin = INT32_MAX, rmax = 0, nst = 0, np = 0;
                    int free = 64;
                    const int need = minnb[size_t(bc)];
                    const int64_t jend = std::min(m, i + kLook);
                    for (int64_t j = i; j < jend && free >= need; ++j) {
                        if (used[j]) continue;
                        const uint32_t r = rec[j];
                        if (int(r & 0xff) != bc) break;
                        const int nb = int((r >> 8) & 0xff);
                        if (nb > free) continue;
                        used[j] = 1;
                        free -= nb;
                        ordo[slot_n++] = in[j];
                        ++np;
                        const int R = int(r >> 16);
                        rmax = R > rmax ? R : rmax;
                        rmin = R < rmin ? R : rmin;
                        nst = R + nb - 1 > nst ? R + nb - 1 : nst;
                    }
                    w.npairs = np;
                    w.rmax = rmax;
                    w.rmin = rmin;
                    w.nsteps = nst;
                    W.push_back(w);
                }
            });
            size_t nw = 0;
            for (auto& W : part_w) nw += W.size();
            lw.reserve(nw);
            for (auto& W : part_w) lw.insert(lw.end(), W.begin(), W.end());
        }
    }
    tm.mark("seg pack: greedy");
    // Dispatch order: the bulk in packing order (co-resident waves share one
    // width's code), the shortest waves filling the last tail_rounds rounds of
    // wave slots last, longest first (LPT, duration ~ BC * nsteps), so the chip
    // drains evenly. Waves address their pairs through slot0: no pair moves.
    {
        // Structured (region) plans keep their order: their waves are in width
        // then read-length order already, and the reorder measured slower there
        // (415 x 128 region: fp32 0.937 -> 0.908 ms without it, call 1.43 -> 1.30 ms,
        // profiles/r02_region_dev_sweep.jsonl).
        const int64_t tail_rounds = std::max<int64_t>(0, env_i64("HC_PHMM_TAIL_ROUNDS", grid ? 0 : 2));
        const size_t nw = lw.size();
        const size_t K = std::min(nw, size_t(tail_rounds) * 4 * size_t(dv.n_cu) * kSegWavesPerSimd);
        std::vector<int64_t>& wc = S.wcost;
        wc.resize(nw);
        int64_t cmin = INT64_MAX, cmax = 0;
        for (size_t k = 0; k < nw; ++k) {
            wc[k] = int64_t(lw[k].ncols) * lw[k].nsteps;
            cmin = std::min(cmin, wc[k]);
            cmax = std::max(cmax, wc[k]);
        }
        // Waves of (nearly) equal length (one region's cross product) drain
        // evenly in any order: no reorder.
        if (K > 0 && K < nw && cmax * 20 > cmin * 21) {
            // Keys (cost, index) in one word each: the K shortest by one
            // nth_element, then those longest first, ties in packing order.
            std::vector<uint64_t>& key = S.wkey;
            key.resize(nw);
            for (size_t k = 0; k < nw; ++k) key[k] = uint64_t(wc[k]) << 32 | k;
            std::nth_element(key.begin(), key.begin() + long(K), key.end());
            for (size_t k = 0; k < K; ++k) key[k] = uint64_t(cmax - int64_t(key[k] >> 32)) << 32 | (key[k] & 0xffffffffu);
            std::sort(key.begin(), key.begin() + long(K));
            std::vector<uint8_t>& in_tail = S.in_tail;
            in_tail.assign(nw, 0);
            for (size_t k = 0; k < K; ++k) in_tail[key[k] & 0xffffffffu] = 1;
            std::vector<LaneWave>& ordered = S.ordered;
            ordered.clear();
            ordered.reserve(nw);
            for (size_t k = 0; k < nw; ++k)
                if (!in_tail[k]) ordered.push_back(lw[k]);
            for (size_t k = 0; k < K; ++k) ordered.push_back(lw[key[k] & 0xffffffffu]);
            lw.swap(ordered);
        }
    }
    tm.mark("seg pack");
    const int n_seg_waves = dev_plan ? int(gd.waves) : int(lw.size());
    const int n_seg_slots = dev_plan ? int(gd.slots) : int(seg_ord.size());
    // One lane per pair with the carry buffer (haps longer than the segmented
    // kernel's reach, or policy "off"): binned by (H rounded up to 16, R).
    const int lane_var = lane_variant_id();
    const LaneVariant& LV = lane_variant(lane_var);
    int64_t carry_rows = 0;
    {
        std::vector<uint32_t>& key = S.key;
        grow(key, size_t(npairs));
        auto cols16 = [&](int p) { return (pd[p].w + 15) / 16 * 16; };
        for (int p : one_ord) key[size_t(p)] = (uint32_t(cols16(p)) << 16) | uint32_t(std::min(pd[p].y, 65535));
        sort_desc(one_ord, key);
        const size_t per_wave = size_t(64) * LV.P;
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
        // Anti-diagonal classes: W by H; (stripes, H) descending so the G pairs
        // sharing a wave have equal stripe counts and similar H, heaviest first.
        const int Wc[2] = {16, 64};
        for (int c = 0; c < 2; ++c) {
            for (int p : ord2[c]) key[size_t(p)] = (uint32_t((pd[p].y + Wc[c] - 1) / Wc[c]) << 16) | uint32_t(pd[p].w);
            sort_desc(ord2[c], key);
        }
    }
    const int Hmax = hmax_a.load();
    tm.mark("one-lane/diag bins");

    // Staging fill: order, wave list, read descriptors + bytes, hap bytes.
    int* ordp = reinterpret_cast<int*>(host + o_ord);
    std::memcpy(ordp, seg_ord.data(), sizeof(int) * seg_ord.size());
    std::memcpy(ordp + n_seg_slots, one_ord.data(), sizeof(int) * one_ord.size());
    const size_t o_ord0 = size_t(n_seg_slots) + one_ord.size();
    std::memcpy(ordp + o_ord0, ord2[0].data(), sizeof(int) * ord2[0].size());
    std::memcpy(ordp + o_ord0 + ord2[0].size(), ord2[1].data(), sizeof(int) * ord2[1].size());
    std::memcpy(host + o_lw, lw.data(), sizeof(LaneWave) * lw.size());
    size_t upload = o_lw + sizeof(LaneWave) * (dev_plan ? size_t(n_seg_waves) : lw.size());
    // Structured plans: the pair descriptors, the slot order and the waves are
    // built on the device (launch_grid_pairs, launch_grid_waves), so the upload
    // skips them and carries the block and segment tables instead.
    const bool dev_pairs = dev_plan;
    const size_t up0 = dev_pairs ? o_rd : 0;
    const size_t up_mid = dev_plan ? o_ord : upload;   // [up0, up_mid) and [o_gb, upload) travel
    size_t o_gb = 0, o_gs = 0, o_gr = 0, o_gh = 0;
    if (dev_pairs) {
        o_gb = (upload + 15) & ~size_t(15);
        GridBlock* gb = reinterpret_cast<GridBlock*>(host + o_gb);
        for (size_t b = 0; b < spec.blocks.size(); ++b)
            gb[b] = GridBlock{loc.blk_p[b], spec.blocks[b].nr, spec.blocks[b].nh, int(loc.blk_r[b]), int(loc.blk_h[b])};
        o_gs = (o_gb + sizeof(GridBlock) * spec.blocks.size() + 15) & ~size_t(15);
        std::memcpy(host + o_gs, gd.segs.data(), sizeof(GridSeg) * gd.segs.size());
        o_gr = (o_gs + sizeof(GridSeg) * gd.segs.size() + 15) & ~size_t(15);
        std::memcpy(host + o_gr, gd.rord.data(), sizeof(int) * gd.rord.size());
        o_gh = (o_gr + sizeof(int) * gd.rord.size() + 15) & ~size_t(15);
        std::memcpy(host + o_gh, gd.hord.data(), sizeof(int) * gd.hord.size());
        upload = o_gh + sizeof(int) * gd.hord.size();
    }
    int4* rdesc = reinterpret_cast<int4*>(host + o_rd);
    uint8_t* hb = reinterpret_cast<uint8_t*>(host + o_bases);
    uint8_t* hq = reinterpret_cast<uint8_t*>(host + o_quals);
    uint8_t* hg = reinterpret_cast<uint8_t*>(host + o_gaps);
    parallel_for(nr, [&](int64_t b, int64_t e) {
        for (int64_t r = b; r < e; ++r) {
            const ReadView v = src.read(loc.read_id(r));
            const size_t o = size_t(row_off[size_t(r)]);
            std::memcpy(hb + o, v.bases, size_t(v.len));
            std::memcpy(hq + o, v.q, size_t(v.len));
            const int32_t g = gapw[size_t(r)];
            int go = 0;
            if (g < 0) {
                go = int(gap_off[size_t(r)]);
                std::memcpy(hg + go, v.i, size_t(v.len));
                std::memcpy(hg + gap_stride + size_t(go), v.d, size_t(v.len));
                std::memcpy(hg + 2 * gap_stride + size_t(go), v.c, size_t(v.len));
            }
            rdesc[r] = make_int4(int(o), v.len, g, go);
        }
    }, 256);
    int4* hdesc = reinterpret_cast<int4*>(host + o_hd);
    uint8_t* hbytes = reinterpret_cast<uint8_t*>(host + o_hb);
    parallel_for(nh, [&](int64_t b, int64_t e) {
        for (int64_t h = b; h < e; ++h) {
            const HapView v = src.hapv(loc.hap_id(h));
            std::memcpy(hbytes + hap_b[size_t(h)], v.bases, size_t(v.len));
            hdesc[h] = make_int4(int(hap_b[size_t(h)]), v.len, int(hap_w[size_t(h)]), 0);
        }
    }, 256);
    tm.mark("staging fill");
    if (g_dry) {
        // Dry runs keep the last part's plan for the host-logic tests
        // (hcx_dump_*): pair descriptors, slot order, segmented waves.
        std::lock_guard<std::mutex> lk(g_dump.mu);
        g_dump.pairs.assign(pd, pd + npairs);
        g_dump.order.assign(seg_ord.begin(), seg_ord.end());
        g_dump.order.insert(g_dump.order.end(), one_ord.begin(), one_ord.end());
        g_dump.waves.assign(lw.begin(), lw.begin() + n_seg_waves);
        g_dump.n_seg_slots = n_seg_slots;
        g_dump.grid = grid;
        *out = nullptr;
        return HC_PHMM_OK;
    }

    // Device region: the upload image, then packed rows / tables, outputs, scratch.
    Layout L;
    L.off = (upload + 255) & ~size_t(255);
    // Packed rows with slack on both sides: the segmented kernels prefetch
    // read words PD steps ahead without clamping to the read (run_seg), so a
    // lane in pipeline fill reads up to 64 words before its read and a pair
    // shorter than its wave's longest read up to that length + 64 past it;
    // those words only feed rows that are never used.
    const size_t row_pad = kRowPadBefore + size_t(rlen_max.load()) + 256;
    const size_t o_rows = L.take(sizeof(uint32_t) * (size_t(nrows) + row_pad));
    const size_t o_hapw = L.take(sizeof(uint32_t) * (size_t(hap_w[size_t(nh)]) + 16));
    const size_t o_res = L.take(res_bytes);
    const size_t o_list = L.take(sizeof(int) * n1);
    const size_t o_count = L.take(4 * sizeof(int));   // rescue list counters, in-wave rescue counters (by run parity)
    const size_t o_sorted = L.take(sizeof(int) * n1);
    const size_t o_big = L.take(sizeof(int) * n1);
    const size_t o_bigc = L.take(sizeof(int));
    const size_t o_plan = L.take(sizeof(Seg64Plan));
    const size_t o_carry = L.take(sizeof(float2) * size_t(carry_rows) * 64 * LV.P);
    const size_t total = L.off;

    auto* b = new Part();
    b->dev = &dv;
    b->spec = spec;
    b->slot = slot;
    char* dev = nullptr;
    int rc = HC_PHMM_OK;
    if (slot) {
        rc = slot_reserve(*slot, total, 0);
        dev = slot->dev;
    } else if (hipMalloc(&dev, total) != hipSuccess) {
        rc = fail(HC_PHMM_ENOMEM, "device allocation failed (" + std::to_string(total >> 20) + " MiB)");
    }
    if (rc) {
        b->slot = nullptr;   // the caller returns the slot
        free_part(b);
        return rc;
    }
    b->dev_base = dev;
    b->n = npairs;
    b->cells = cells_a.load();
    b->Hmax = Hmax;
    b->n_lane = int(size_t(n_seg_slots) + one_ord.size());
    b->n_seg_waves = n_seg_waves;
    b->lane_variant = lane_var;
    b->lane_waves = dev_plan ? n_seg_waves : int(lw.size());
    b->upload_bytes = dev_pairs ? (up_mid - up0) + (o_lw - o_bases) + (upload - o_gb) : upload - up0;
    b->d_pairs = reinterpret_cast<PairDesc*>(dev + o_pairs);
    b->d_rows = reinterpret_cast<uint32_t*>(dev + o_rows) + kRowPadBefore;
    b->d_hapw = reinterpret_cast<uint32_t*>(dev + o_hapw);
    const int Wc[2] = {16, 64};
    int* d_ord = reinterpret_cast<int*>(dev + o_ord);
    b->d_lane_order = d_ord;
    b->cls[0].d_order = d_ord + o_ord0;
    b->cls[1].d_order = d_ord + o_ord0 + ord2[0].size();
    for (int c = 0; c < 2; ++c) {
        b->cls[c].W = Wc[c];
        b->cls[c].n = int(ord2[c].size());
        int hm = 0;
        for (int p : ord2[c]) hm = std::max(hm, pd[p].w);
        b->cls[c].ring_len = hm + 2 * Wc[c] + 16;
    }
    b->d_lane_waves = reinterpret_cast<LaneWave*>(dev + o_lw);
    b->res_bytes = res_bytes;
    b->res_o64 = res_o64;
    b->res_ofl = res_ofl;
    b->own_raw32 = b->d_raw32 = reinterpret_cast<float*>(dev + o_res);
    b->own_raw64 = b->d_raw64 = reinterpret_cast<double*>(dev + o_res + res_o64);
    b->own_flag = b->d_flag = reinterpret_cast<uint8_t*>(dev + o_res + res_ofl);
    b->d_list = reinterpret_cast<int*>(dev + o_list);
    b->d_count = reinterpret_cast<int*>(dev + o_count);
    b->d_sorted = reinterpret_cast<int*>(dev + o_sorted);
    b->d_big = reinterpret_cast<int*>(dev + o_big);
    b->d_big_count = reinterpret_cast<int*>(dev + o_bigc);
    b->d_plan = reinterpret_cast<Seg64Plan*>(dev + o_plan);
    b->n_wide = wide_a.load();
    b->d_carry = carry_rows ? reinterpret_cast<float2*>(dev + o_carry) : nullptr;
    if (slot) b->host_res = host + host_res_off;

    if (slot) {
        b->stream = slot->stream;
        b->side = slot->side;
        b->fork = slot->fork;
        b->join = slot->join;
        b->slot_ev = true;
        b->pack_ev[0] = slot->ev[0];
        b->pack_ev[1] = slot->ev[1];
        b->ev_pool.push_back({slot->ev[2], slot->ev[3], slot->ev[4]});
        b->done = slot->ev[5];
    } else {
        b->stream = dv.stream;
        b->side = dv.side;
        b->fork = dv.fork;
        b->join = dv.join;
    }
    hipStream_t s = b->stream;
    auto enqueue = [&]() -> int {
        if (!b->slot_ev)
            for (auto& e : b->pack_ev) HIP_TRY(hipEventCreate(&e));
        if (dev_pairs) {
            // [o_rd, o_ord): read / hap descriptors; the order and waves between
            // are built on the device; then the read / hap bytes and the block
            // and segment tables. One fused launch prepares everything.
            HIP_TRY(hipMemcpyAsync(dev + up0, host + up0, up_mid - up0, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(dev + o_bases, host + o_bases, o_lw - o_bases, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(dev + o_gb, host + o_gb, upload - o_gb, hipMemcpyHostToDevice, s));
            HIP_TRY(hipEventRecord(b->pack_ev[0], s));
            GridPrepArgs g{};
            g.bases = reinterpret_cast<const uint8_t*>(dev + o_bases);
            g.quals = reinterpret_cast<const uint8_t*>(dev + o_quals);
            g.gaps = reinterpret_cast<const uint8_t*>(dev + o_gaps);
            g.gap_stride = (long long)gap_stride;
            g.rdesc = reinterpret_cast<const int4*>(dev + o_rd);
            g.nreads = int(nr);
            g.rows = b->d_rows;
            g.hap_bytes = reinterpret_cast<const uint8_t*>(dev + o_hb);
            g.hdesc = reinterpret_cast<const int4*>(dev + o_hd);
            g.nhaps = int(nh);
            g.hapw = b->d_hapw;
            g.blocks = reinterpret_cast<const GridBlock*>(dev + o_gb);
            g.nblocks = int(spec.blocks.size());
            g.npairs = (long long)npairs;
            g.pairs = b->d_pairs;
            g.segs = reinterpret_cast<const GridSeg*>(dev + o_gs);
            g.nsegs = int(gd.segs.size());
            g.nslots = (long long)n_seg_slots;
            g.nwaves = n_seg_waves;
            g.rord = reinterpret_cast<const int*>(dev + o_gr);
            g.hord = reinterpret_cast<const int*>(dev + o_gh);
            g.order = reinterpret_cast<int*>(dev + o_ord);
            g.waves = reinterpret_cast<LaneWave*>(dev + o_lw);
            g.counters = b->d_count;
            HIP_TRY(launch_prepare_grid(g, s));
            HIP_TRY(hipEventRecord(b->pack_ev[1], s));
        } else {
            HIP_TRY(hipMemcpyAsync(dev + up0, host + up0, upload - up0, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemsetAsync(b->d_count, 0, 4 * sizeof(int), s));
            HIP_TRY(hipEventRecord(b->pack_ev[0], s));
            HIP_TRY(launch_pack_reads(reinterpret_cast<const uint8_t*>(dev + o_bases),
                                      reinterpret_cast<const uint8_t*>(dev + o_quals),
                                      reinterpret_cast<const uint8_t*>(dev + o_gaps), (long long)gap_stride,
                                      reinterpret_cast<const int4*>(dev + o_rd), int(nr), b->d_rows, s));
            HIP_TRY(launch_hap_tables(reinterpret_cast<const uint8_t*>(dev + o_hb),
                                      reinterpret_cast<const int4*>(dev + o_hd), int(nh), b->d_hapw, s));
            HIP_TRY(hipEventRecord(b->pack_ev[1], s));
        }
        if (with_run) {
            const int r = run_part(b, s);
            if (r) return r;
            HIP_TRY(hipMemcpyAsync(b->host_res, dev + o_res, res_bytes, hipMemcpyDeviceToHost, s));
            if (!b->done) HIP_TRY(hipEventCreateWithFlags(&b->done, hipEventDisableTiming));
            HIP_TRY(hipEventRecord(b->done, s));
        }
        // A part-owned staging buffer is freed on return: the copy must be done.
        if (own_host) HIP_TRY(hipStreamSynchronize(s));
        return HC_PHMM_OK;
    };
    rc = enqueue();
    tm.mark("enqueue");
    if (rc) {
        (void)hipStreamSynchronize(s);
        b->slot = nullptr;
        free_part(b);
        return rc;
    }
    *out = b;
    return HC_PHMM_OK;
}

// HC_PHMM_TIMELINE=1: per-wave start / end / HW_ID of the last segmented fp32
// pass (diagnostics; read back by hcx_timeline).
struct Timeline {
    std::mutex mu;
    unsigned long long* buf = nullptr;
    size_t cap = 0;
    int n = 0;
    hipStream_t stream = nullptr;
} g_tl;

int run_part(Part* b, hipStream_t s)
{
    Device& dv = *b->dev;
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
    // and the rescue planner zeroes the other parity's counter for the next run.
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
        a.lut = dv.lut_f;
        a.raw_out = b->d_raw32;
        a.rescue_flag = b->d_flag;
        a.rescue_list = b->d_list;
        a.rescue_count = count;
        a.raw64_zero = b->d_raw64;
        a.lut64 = dv.lut_d;
        if (env_i64("HC_PHMM_RESCUE_IN_WAVE", 1) != 0) {
            a.inker_count = b->d_count + 2 + par;
            // A wave that rescues in place runs up to ~2.5x longer; a few such
            // waves hide inside the pass, hundreds of them (a region whose reads
            // miss some haps: ~440 rescues) drain late and cost more than the
            // separate fp64 pass they would save (415 x 128 region: fp32
            // 0.925 -> 0.80 ms at a cap of 32, S2's 19 rescues unchanged;
            // profiles/r02_in_wave_rescue_cap.jsonl). Past the cap, the list.
            a.inker_limit = int(std::max<int64_t>(0, env_i64("HC_PHMM_RESCUE_IN_WAVE_MAX", 32)));
        }
        b->inker_limit = a.inker_limit;
        if (env_i64("HC_PHMM_TIMELINE", 0) != 0 && b->n_seg_waves > 0) {
            std::lock_guard<std::mutex> lk(g_tl.mu);
            const size_t need = size_t(b->n_seg_waves) * 3;
            if (g_tl.cap < need) {
                if (g_tl.buf) (void)hipFree(g_tl.buf);
                g_tl.buf = nullptr;
                g_tl.cap = 0;
                HIP_TRY(hipMalloc(&g_tl.buf, need * sizeof(unsigned long long)));
                g_tl.cap = need;
            }
            g_tl.n = b->n_seg_waves;
            g_tl.stream = s;
            a.timeline = g_tl.buf;
        }
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
                HIP_TRY(hipEventRecord(b->fork, s));
                HIP_TRY(hipStreamWaitEvent(b->side, b->fork, 0));
            }
            HIP_TRY(launch_lane_seg_f32(g, fork ? b->side : s));
            if (fork) HIP_TRY(hipEventRecord(b->join, b->side));
        }
        if (n_one > 0) {
            a.waves = b->d_lane_waves + b->n_seg_waves;
            a.n_waves = n_one;
            HIP_TRY(launch_lane_f32(b->lane_variant, a, s));
        }
        if (fork) HIP_TRY(hipStreamWaitEvent(s, b->join, 0));
    }
    for (auto& c : b->cls) {
        if (c.n == 0) continue;
        DiagArgs a{};
        a.pairs = b->d_pairs;
        a.order = c.d_order;
        a.n_slots = c.n;
        a.rows = b->d_rows;
        a.hapw = b->d_hapw;
        a.lut = dv.lut_f;
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
        r.lut = dv.lut_d;
        r.list = b->d_list;
        r.count = count;
        r.count_reset = b->d_count + (par ^ 1);
        r.inker_reset = b->d_count + 2 + (par ^ 1);
        r.sorted = b->d_sorted;
        r.big = b->d_big;
        r.big_count = b->d_big_count;
        r.plan = b->d_plan;
        r.raw_out = b->d_raw64;
        r.min_lanes = int64_t(2) * 4 * dv.n_cu * 64;
        const int grid = int(std::min<int64_t>((b->n + 3) / 4, int64_t(2) * dv.n_cu));
        HIP_TRY(launch_rescue_seg64(r, grid, s));
        if (b->n_wide > 0) {
            DiagArgs a{};
            a.pairs = b->d_pairs;
            a.order = b->d_big;
            a.n_slots_dev = b->d_big_count;
            a.rows = b->d_rows;
            a.hapw = b->d_hapw;
            a.lut = dv.lut_d;
            a.ring_len = b->Hmax + 2 * 64 + 16;
            a.raw_out = b->d_raw64;
            HIP_TRY(launch_diag_f64(64, a, int(std::min<int64_t>(b->n_wide, 2048)), s));
        }
    }
    HIP_TRY(hipEventRecord(b->ev[2], s));
    b->ran = true;
    return HC_PHMM_OK;
}

// log10 finish (intel_pairhmm.hpp:137-143, glibc log10 / log10f as in the
// reference) of a part's results, scattered into the caller's outputs.
void finish_part(const Part& P, const float* f, const double* d, const uint8_t* fl, const Outputs& o)
{
    const Luts& L = luts();
    const float l10f = L.log10_init_f;
    const double l10d = L.log10_init_d;
    auto ll = [&](int64_t k) { return fl[k] ? std::log10(d[k]) - l10d : double(std::log10(f[k]) - l10f); };
    if (P.spec.flat) {
        const int64_t id0 = P.spec.lo;
        parallel_for(P.n, [&](int64_t lo, int64_t hi) {
            for (int64_t k = lo; k < hi; ++k) {
                if (o.loglik) o.loglik[id0 + k] = ll(k);
                if (o.raw32) o.raw32[id0 + k] = f[k];
                if (o.raw64) o.raw64[id0 + k] = d[k];
                if (o.resc) o.resc[id0 + k] = fl[k];
            }
        }, 1 << 13);
        return;
    }
    // Blocks: pair k of block b is (r, h) = divmod(k - base, nh).
    std::vector<int64_t> base(P.spec.blocks.size() + 1, 0);
    for (size_t b = 0; b < P.spec.blocks.size(); ++b)
        base[b + 1] = base[b] + int64_t(P.spec.blocks[b].nr) * P.spec.blocks[b].nh;
    parallel_for(P.n, [&](int64_t lo, int64_t hi) {
        size_t b = size_t(std::upper_bound(base.begin(), base.end(), lo) - base.begin()) - 1;
        int64_t k = lo;
        while (k < hi) {
            const Block& B = P.spec.blocks[b];
            const int64_t end = std::min(hi, base[b + 1]);
            int64_t r = (k - base[b]) / B.nh, h = (k - base[b]) % B.nh;
            for (; k < end; ++k) {
                B.out[r * B.ostride + h] = ll(k);
                if (++h == B.nh) {
                    h = 0;
                    ++r;
                }
            }
            ++b;
        }
    }, 1 << 13);
}

// ---------------------------------------------------------------------------
// Splitting a call into parts.

// Cut a sequence of units with weights into `nparts` contiguous ranges of
// (nearly) equal weight: returns nparts + 1 boundaries.
std::vector<int64_t> equal_cuts(const std::vector<int64_t>& prefix, int nparts)
{
    const int64_t n = int64_t(prefix.size()) - 1;
    const int64_t tot = prefix.back();
    std::vector<int64_t> cut(static_cast<size_t>(nparts) + 1, 0);
    cut[size_t(nparts)] = n;
    for (int j = 1; j < nparts; ++j) {
        const int64_t target = (tot * j + nparts / 2) / nparts;
        int64_t c = int64_t(std::lower_bound(prefix.begin(), prefix.end(), target) - prefix.begin());
        // the nearer of the boundaries either side of the target (two halves of
        // a region just under half each must not both land in the first part)
        if (c > 0 && c <= n && target - prefix[size_t(c) - 1] < prefix[size_t(c)] - target) --c;
        cut[size_t(j)] = std::max(cut[size_t(j) - 1], std::min(n, c));
    }
    return cut;
}

// How many parts for `cells` over the configured devices: one part below
// HC_PHMM_SHARD_MIN_CELLS; above, per device at least HC_PHMM_MIN_CHUNKS (1)
// and about one per HC_PHMM_CHUNK_CELLS, so the planning of part k + 1
// overlaps the device pass of part k (the parts of one device run on their
// slots' streams, concurrently). One 415 x 128 region (3.3e9 cells) stays
// whole: cut in 2 / 3 / 4 parts it took 2.23 / 1.99 / 1.84 ms vs 1.89 ms
// (tools/region_ab.py; each part pays its own planning fixed costs and fp64
// pass).
int part_count(int64_t cells, int ndev)
{
    const int64_t shard_min = env_i64("HC_PHMM_SHARD_MIN_CELLS", int64_t(2000000000));
    const int64_t chunk = std::max<int64_t>(1, env_i64("HC_PHMM_CHUNK_CELLS", int64_t(12000000000)));
    const int64_t min_chunks = std::max<int64_t>(1, env_i64("HC_PHMM_MIN_CHUNKS", 1));
    if (cells < shard_min) return 1;
    const int64_t per_dev = (cells + ndev - 1) / ndev;
    const int64_t chunks = std::max<int64_t>(min_chunks, (per_dev + chunk / 2) / chunk);
    return int(std::min<int64_t>(int64_t(ndev) * chunks, 4096));
}

Device* least_loaded()
{
    std::lock_guard<std::mutex> lk(g_mu);
    Device* best = g_devs[0];
    for (Device* d : g_devs)
        if (d->outstanding < best->outstanding) best = d;
    return best;
}

// Plan + enqueue every part of a call (device of part j = j mod #devices, or
// the least loaded device for a one-part call); returns the job.
int submit(const Src& src, const std::vector<PartSpec>& specs, const std::vector<double>& part_cells,
           const Outputs& out, hc_phmm_job** job)
{
    auto* J = new hc_phmm_job();
    J->out = out;
    const int G = int(g_devs.size());
    if (std::getenv("HC_PHMM_TRACE")) std::fprintf(stderr, "[hc_phmm] submit: %zu part(s)\n", specs.size());
    Device* solo = specs.size() == 1 ? least_loaded() : nullptr;
    for (size_t j = 0; j < specs.size(); ++j) {
        Device& d = solo ? *solo : *g_devs[j % size_t(G)];
        int rc = hipSetDevice(d.ordinal) == hipSuccess ? HC_PHMM_OK : fail(HC_PHMM_EHIP, "hipSetDevice");
        Slot* sl = rc ? nullptr : take_slot(d);
        Part* p = nullptr;
        if (!rc) rc = plan_part(d, src, specs[j], sl, true, &p);
        if (rc) {
            if (sl) give_slot(sl);
            for (Part* q : J->parts) {
                (void)hipSetDevice(q->dev->ordinal);
                (void)hipStreamSynchronize(q->stream);
                free_part(q);
            }
            delete J;
            return rc;
        }
        {
            std::lock_guard<std::mutex> lk(g_mu);
            d.outstanding += part_cells[j];
        }
        J->parts.push_back(p);
        J->cells_per_part.push_back(part_cells[j]);
    }
    *job = J;
    return HC_PHMM_OK;
}

int collect(hc_phmm_job* J)
{
    int rc = HC_PHMM_OK;
    PhaseTimer tm;
    for (size_t j = 0; j < J->parts.size(); ++j) {
        Part* p = J->parts[j];
        if (rc == HC_PHMM_OK) {
            (void)hipSetDevice(p->dev->ordinal);
            const hipError_t e = hipEventSynchronize(p->done);
            if (e != hipSuccess) {
                rc = fail(HC_PHMM_EHIP, std::string("device pass: ") + hipGetErrorString(e));
            } else {
                tm.mark("collect: wait");
                if (tm.on) {
                    float a = 0, f32 = 0, f64 = 0;
                    (void)hipEventElapsedTime(&a, p->pack_ev[0], p->pack_ev[1]);
                    (void)hipEventElapsedTime(&f32, p->ev[0], p->ev[1]);
                    (void)hipEventElapsedTime(&f64, p->ev[1], p->ev[2]);
                    std::fprintf(stderr, "[hc_phmm]   device: pack %.3f ms, fp32 %.3f ms, fp64 %.3f ms (%lld pairs)\n", a,
                                 f32, f64, (long long)p->n);
                }
                const char* h = p->host_res;
                finish_part(*p, reinterpret_cast<const float*>(h), reinterpret_cast<const double*>(h + p->res_o64),
                            reinterpret_cast<const uint8_t*>(h + p->res_ofl), J->out);
                tm.mark("collect: finish");
            }
        } else {
            (void)hipSetDevice(p->dev->ordinal);
            (void)hipEventSynchronize(p->done);
        }
        {
            std::lock_guard<std::mutex> lk(g_mu);
            p->dev->outstanding -= J->cells_per_part[j];
        }
        free_part(p);
    }
    delete J;
    return rc;
}

// Flat pairs [0, n): cut into parts of equal cells.
int submit_flat(const Src& src, int64_t n, const Outputs& out, hc_phmm_job** job)
{
    std::vector<int64_t> pre;
    prefix_sum(n, pre, [&](int64_t p) { return int64_t(src.R[p] > 0 ? src.R[p] : 0) * (src.H[p] > 0 ? src.H[p] : 0); });
    const int np = part_count(pre.back(), int(g_devs.size()));
    const std::vector<int64_t> cut = equal_cuts(pre, np);
    std::vector<PartSpec> specs;
    std::vector<double> pc;
    for (int j = 0; j < np; ++j) {
        if (cut[size_t(j)] == cut[size_t(j) + 1] && np > 1) continue;
        PartSpec s;
        s.flat = true;
        s.lo = cut[size_t(j)];
        s.hi = cut[size_t(j) + 1];
        specs.push_back(s);
        pc.push_back(double(pre[size_t(s.hi)] - pre[size_t(s.lo)]));
    }
    return submit(src, specs, pc, out, job);
}

// Cross-product blocks (regions): a block larger than one part's share is cut
// into read ranges; then contiguous runs of blocks form parts of equal cells.
int submit_blocks(const Src& src, std::vector<Block> blocks, hc_phmm_job** job)
{
    int64_t cells = 0;
    std::vector<int64_t> bc(blocks.size());
    for (size_t k = 0; k < blocks.size(); ++k) {
        int64_t rl = 0, hl = 0;
        for (int32_t r = 0; r < blocks[k].nr; ++r) rl += std::max(0, src.read_len(blocks[k].r0 + r));
        for (int32_t h = 0; h < blocks[k].nh; ++h) hl += std::max(0, src.hap_len(blocks[k].h0 + h));
        bc[k] = rl * hl;
        cells += bc[k];
    }
    const int np = part_count(cells, int(g_devs.size()));
    if (np > 1) {
        const int64_t share = (cells + np - 1) / np;
        std::vector<Block> split;
        for (size_t k = 0; k < blocks.size(); ++k) {
            const Block& B = blocks[k];
            const int pieces = int(std::min<int64_t>(B.nr, (bc[k] + share - 1) / std::max<int64_t>(share, 1)));
            if (pieces <= 1) {
                split.push_back(B);
                continue;
            }
            for (int q = 0; q < pieces; ++q) {
                const int32_t a = int32_t(int64_t(B.nr) * q / pieces), e = int32_t(int64_t(B.nr) * (q + 1) / pieces);
                if (a == e) continue;
                split.push_back(Block{B.r0 + a, e - a, B.h0, B.nh, B.out + int64_t(a) * B.ostride, B.ostride});
            }
        }
        blocks.swap(split);
    }
    std::vector<int64_t> pre(blocks.size() + 1, 0);
    for (size_t k = 0; k < blocks.size(); ++k) {
        int64_t rl = 0, hl = 0;
        for (int32_t r = 0; r < blocks[k].nr; ++r) rl += std::max(0, src.read_len(blocks[k].r0 + r));
        for (int32_t h = 0; h < blocks[k].nh; ++h) hl += std::max(0, src.hap_len(blocks[k].h0 + h));
        pre[k + 1] = pre[k] + rl * hl;
    }
    const int nparts = std::max(1, std::min<int>(np, int(blocks.size())));
    const std::vector<int64_t> cut = equal_cuts(pre, nparts);
    std::vector<PartSpec> specs;
    std::vector<double> pc;
    for (int j = 0; j < nparts; ++j) {
        if (cut[size_t(j)] == cut[size_t(j) + 1]) continue;
        PartSpec s;
        s.flat = false;
        s.blocks.assign(blocks.begin() + long(cut[size_t(j)]), blocks.begin() + long(cut[size_t(j) + 1]));
        specs.push_back(std::move(s));
        pc.push_back(double(pre[size_t(cut[size_t(j) + 1])] - pre[size_t(cut[size_t(j)])]));
    }
    if (specs.empty()) {
        *job = new hc_phmm_job();
        return HC_PHMM_OK;
    }
    return submit(src, specs, pc, Outputs{}, job);
}

Src flat_src(const int64_t* read_off, const int32_t* R, const int64_t* hap_off, const int32_t* H, const uint8_t* rs,
             const uint8_t* q, const uint8_t* ins, const uint8_t* del, const uint8_t* gcp, const uint8_t* hap)
{
    Src s;
    s.read_off = read_off;
    s.R = R;
    s.hap_off = hap_off;
    s.H = H;
    s.rs = rs;
    s.q = q;
    s.ins = ins;
    s.del = del;
    s.gcp = gcp;
    s.hap = hap;
    return s;
}

bool flat_args_ok(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off, const int32_t* H,
                  const uint8_t* rs, const uint8_t* q, const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
                  const uint8_t* hap)
{
    return n == 0 || (read_off && R && hap_off && H && rs && q && ins && del && gcp && hap);
}

// Regions -> one Src over concatenated read / hap structs + one block per region.
struct RegionSet {
    std::vector<hc_phmm_read> reads;
    std::vector<hc_phmm_hap> haps;
    std::vector<Block> blocks;
};

int gather_regions(const hc_phmm_region* regions, int32_t n_regions, RegionSet& rs)
{
    if (n_regions < 0 || (n_regions > 0 && !regions)) return fail(HC_PHMM_EINVAL, "bad region list");
    size_t tr = 0, th = 0;
    for (int k = 0; k < n_regions; ++k) {
        const hc_phmm_region& g = regions[k];
        if (g.n_reads < 0 || g.n_haps < 0) return fail(HC_PHMM_EINVAL, "negative count in region");
        if (g.n_reads == 0 || g.n_haps == 0) continue;
        if (!g.reads || !g.haps || !g.out) return fail(HC_PHMM_EINVAL, "null pointer in region");
        tr += size_t(g.n_reads);
        th += size_t(g.n_haps);
    }
    rs.reads.resize(tr);
    rs.haps.resize(th);
    size_t r0 = 0, h0 = 0;
    for (int k = 0; k < n_regions; ++k) {
        const hc_phmm_region& g = regions[k];
        if (g.n_reads == 0 || g.n_haps == 0) continue;
        std::memcpy(rs.reads.data() + r0, g.reads, sizeof(hc_phmm_read) * size_t(g.n_reads));
        std::memcpy(rs.haps.data() + h0, g.haps, sizeof(hc_phmm_hap) * size_t(g.n_haps));
        rs.blocks.push_back(Block{int64_t(r0), g.n_reads, int64_t(h0), g.n_haps, g.out, g.n_haps});
        r0 += size_t(g.n_reads);
        h0 += size_t(g.n_haps);
    }
    return HC_PHMM_OK;
}

}  // namespace

// --------------------------------------------------------------------------
// C ABI
namespace hcphmm {
void set_last_error(const std::string& msg) { g_err = msg; }
int primary_device()
{
    std::lock_guard<std::mutex> lk(g_mu);
    return g_devs.empty() ? -1 : g_devs[0]->ordinal;
}
}  // namespace hcphmm

extern "C" {

int hc_phmm_version(void) { return 200; }

const char* hc_phmm_last_error(void) { return g_err.c_str(); }

int hc_phmm_init(uint32_t /*flags*/, int device)
{
    std::lock_guard<std::mutex> lk(g_mu);
    const int32_t d = device;
    return init_devices_locked(&d, 1, device < 0);
}

int hc_phmm_init_devices(uint32_t /*flags*/, const int32_t* devices, int32_t n)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return init_devices_locked(devices, n, false);
}

int hc_phmm_device_count(void)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return int(g_devs.size());
}

int hc_phmm_shutdown(void)
{
    hcphmm::sw_release();
    hcphmm::gt_release();
    std::lock_guard<std::mutex> lk(g_mu);
    for (Device* d : g_devs) release_device(d);
    g_devs.clear();
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

int hc_phmm_submit_pairs(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                         const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                         const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, double* loglik,
                         float* raw_f32, double* raw_f64, uint8_t* rescued, hc_phmm_job** job)
{
    if (!job) return fail(HC_PHMM_EINVAL, "null job");
    *job = nullptr;
    if (n < 0) return fail(HC_PHMM_EINVAL, "negative pair count");
    if (!flat_args_ok(n, read_off, R, hap_off, H, rs, q, ins, del, gcp, hap))
        return fail(HC_PHMM_EINVAL, "null input array");
    int rc = ensure_init();
    if (rc) return rc;
    if (n == 0) {
        *job = new hc_phmm_job();
        return HC_PHMM_OK;
    }
    Outputs o{loglik, raw_f32, raw_f64, rescued};
    return submit_flat(flat_src(read_off, R, hap_off, H, rs, q, ins, del, gcp, hap), n, o, job);
}

int hc_phmm_submit_regions(const hc_phmm_region* regions, int32_t n_regions, hc_phmm_job** job)
{
    if (!job) return fail(HC_PHMM_EINVAL, "null job");
    *job = nullptr;
    RegionSet rs;
    int rc = gather_regions(regions, n_regions, rs);
    if (rc) return rc;
    rc = ensure_init();
    if (rc) return rc;
    Src src;
    src.reads = rs.reads.data();
    src.haps = rs.haps.data();
    return submit_blocks(src, rs.blocks, job);
}

int hc_phmm_job_ready(hc_phmm_job* job)
{
    if (!job) return fail(HC_PHMM_EINVAL, "null job");
    for (Part* p : job->parts) {
        (void)hipSetDevice(p->dev->ordinal);
        const hipError_t e = hipEventQuery(p->done);
        if (e == hipErrorNotReady) return 0;
        if (e != hipSuccess) return fail(HC_PHMM_EHIP, std::string("device pass: ") + hipGetErrorString(e));
    }
    return 1;
}

int hc_phmm_collect(hc_phmm_job* job)
{
    if (!job) return fail(HC_PHMM_EINVAL, "null job");
    return collect(job);
}

int hc_phmm_pairs_flat(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                       const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                       const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, double* loglik,
                       float* raw_f32, double* raw_f64, uint8_t* rescued)
{
    hc_phmm_job* job = nullptr;
    const int rc = hc_phmm_submit_pairs(n, read_off, R, hap_off, H, rs, q, ins, del, gcp, hap, loglik, raw_f32,
                                        raw_f64, rescued, &job);
    if (rc) return rc;
    return collect(job);
}

int hc_phmm_cross(const hc_phmm_read* reads, int32_t n_reads, const hc_phmm_hap* haps, int32_t n_haps, double* out)
{
    if (n_reads < 0 || n_haps < 0) return fail(HC_PHMM_EINVAL, "negative count");
    if (n_reads == 0 || n_haps == 0) return HC_PHMM_OK;
    if (!reads || !haps || !out) return fail(HC_PHMM_EINVAL, "null argument");
    hc_phmm_region g{reads, n_reads, haps, n_haps, out};
    hc_phmm_job* job = nullptr;
    const int rc = hc_phmm_submit_regions(&g, 1, &job);
    if (rc) return rc;
    return collect(job);
}

int hc_phmm_cross_regions(const hc_phmm_region* regions, int32_t n_regions)
{
    hc_phmm_job* job = nullptr;
    const int rc = hc_phmm_submit_regions(regions, n_regions, &job);
    if (rc) return rc;
    return collect(job);
}

int hc_phmm_compute_likelihoods(const hc_phmm_read* reads, int32_t n_reads, const hc_phmm_hap* haps,
                                int32_t n_haps, double* out, uint8_t* keep, int32_t* n_kept)
{
    if (n_reads > 0 && (!keep || !n_kept)) return fail(HC_PHMM_EINVAL, "null keep/n_kept");
    int rc = hc_phmm_cross(reads, n_reads, haps, n_haps, out);
    if (rc) return rc;
    int kept = 0;
    // normalize_likelihoods_and_filter_poorly_modeled_reads, intel_pairhmm.hpp:24-46
    for (int r = 0; r < n_reads; ++r) {
        double* row = out + size_t(r) * size_t(n_haps);
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

// ---- prepared batches (device-resident, one part per device slot)

int hc_phmm_batch_create(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                         const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                         const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, hc_phmm_batch** out)
{
    if (!out) return fail(HC_PHMM_EINVAL, "null out");
    *out = nullptr;
    if (n < 0) return fail(HC_PHMM_EINVAL, "negative pair count");
    if (!flat_args_ok(n, read_off, R, hap_off, H, rs, q, ins, del, gcp, hap))
        return fail(HC_PHMM_EINVAL, "null input array");
    int rc = ensure_init();
    if (rc) return rc;
    const Src src = flat_src(read_off, R, hap_off, H, rs, q, ins, del, gcp, hap);
    std::vector<int64_t> pre;
    prefix_sum(n, pre, [&](int64_t p) { return int64_t(std::max(0, R[p])) * std::max(0, H[p]); });
    const int G = int(g_devs.size());
    const std::vector<int64_t> cut = equal_cuts(pre, G);
    auto* B = new hc_phmm_batch();
    B->n = n;
    for (int j = 0; j < G; ++j) {
        if (j > 0 && cut[size_t(j)] == cut[size_t(j) + 1]) continue;
        PartSpec s;
        s.flat = true;
        s.lo = cut[size_t(j)];
        s.hi = cut[size_t(j) + 1];
        Device& d = *g_devs[size_t(j)];
        Part* p = nullptr;
        rc = hipSetDevice(d.ordinal) == hipSuccess ? plan_part(d, src, s, nullptr, false, &p)
                                                   : fail(HC_PHMM_EHIP, "hipSetDevice");
        if (rc) {
            for (Part* x : B->parts) free_part(x);
            delete B;
            return rc;
        }
        B->parts.push_back(p);
    }
    *out = B;
    return HC_PHMM_OK;
}

int hc_phmm_batch_run(hc_phmm_batch* b, void* stream)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    if (stream && b->parts.size() > 1)
        return fail(HC_PHMM_EINVAL, "a caller stream selects one device; this batch spans several");
    for (Part* p : b->parts) {
        HIP_TRY(hipSetDevice(p->dev->ordinal));
        const int rc = run_part(p, stream ? static_cast<hipStream_t>(stream) : p->stream);
        if (rc) return rc;
    }
    return HC_PHMM_OK;
}

int hc_phmm_batch_results(hc_phmm_batch* b, double* loglik, float* raw_f32, double* raw_f64, uint8_t* rescued)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    const Outputs o{loglik, raw_f32, raw_f64, rescued};
    for (Part* p : b->parts) {
        if (!p->ran) return fail(HC_PHMM_EINVAL, "batch has not been run");
        if (p->n == 0) continue;
        HIP_TRY(hipSetDevice(p->dev->ordinal));
        HIP_TRY(hipStreamSynchronize(p->last_stream));
        std::vector<char> host(p->res_bytes);
        const size_t n = size_t(p->n);
        HIP_TRY(hipMemcpy(host.data(), p->d_raw32, sizeof(float) * n, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(host.data() + p->res_o64, p->d_raw64, sizeof(double) * n, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(host.data() + p->res_ofl, p->d_flag, n, hipMemcpyDeviceToHost));
        finish_part(*p, reinterpret_cast<const float*>(host.data()),
                    reinterpret_cast<const double*>(host.data() + p->res_o64),
                    reinterpret_cast<const uint8_t*>(host.data() + p->res_ofl), o);
    }
    return HC_PHMM_OK;
}

int hc_phmm_batch_device_results(hc_phmm_batch* b, void** raw_f32, void** raw_f64, void** rescued)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    if (b->parts.size() != 1) return fail(HC_PHMM_EINVAL, "device results of a batch split over several devices");
    Part* p = b->parts[0];
    if (raw_f32) *raw_f32 = p->d_raw32;
    if (raw_f64) *raw_f64 = p->d_raw64;
    if (rescued) *rescued = p->d_flag;
    return HC_PHMM_OK;
}

int hc_phmm_batch_bind_outputs(hc_phmm_batch* b, void* raw_f32, void* raw_f64, void* rescued)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    if (b->parts.size() != 1) return fail(HC_PHMM_EINVAL, "bind_outputs on a batch split over several devices");
    Part* p = b->parts[0];
    p->d_raw32 = raw_f32 ? static_cast<float*>(raw_f32) : p->own_raw32;
    p->d_raw64 = raw_f64 ? static_cast<double*>(raw_f64) : p->own_raw64;
    p->d_flag = rescued ? static_cast<uint8_t*>(rescued) : p->own_flag;
    return HC_PHMM_OK;
}

int hc_phmm_batch_stats(hc_phmm_batch* b, hc_phmm_stats* st)
{
    if (!b || !st) return fail(HC_PHMM_EINVAL, "null argument");
    std::memset(st, 0, sizeof(*st));
    st->n_pairs = b->n;
    st->n_devices = int64_t(b->parts.size());
    for (Part* p : b->parts) {
        HIP_TRY(hipSetDevice(p->dev->ordinal));
        st->cells += p->cells;
        st->n_launch_waves += p->launch_waves;
        st->n_lane_pairs += p->n_lane;
        st->n_seg_waves += p->n_seg_waves;
        st->upload_bytes += int64_t(p->upload_bytes);
        if (p->pack_ev[0]) {
            float pk = 0;
            HIP_TRY(hipEventSynchronize(p->pack_ev[1]));
            HIP_TRY(hipEventElapsedTime(&pk, p->pack_ev[0], p->pack_ev[1]));
            st->pack_ms = std::max(st->pack_ms, double(pk));
        }
        if (p->ran && p->ev_used > 0) {
            HIP_TRY(hipStreamSynchronize(p->last_stream));
            double sa = 0, sc = 0;
            for (size_t k = 0; k < p->ev_used; ++k) {
                float a = 0, c = 0;
                HIP_TRY(hipEventSynchronize(p->ev_pool[k][2]));
                HIP_TRY(hipEventElapsedTime(&a, p->ev_pool[k][0], p->ev_pool[k][1]));
                HIP_TRY(hipEventElapsedTime(&c, p->ev_pool[k][1], p->ev_pool[k][2]));
                sa += a;
                sc += c;
            }
            st->n_runs = std::max(st->n_runs, int64_t(p->ev_used));
            st->kernel_ms_f32 = std::max(st->kernel_ms_f32, sa / double(p->ev_used));
            st->kernel_ms_f64 = std::max(st->kernel_ms_f64, sc / double(p->ev_used));
            st->run_ms = std::max(st->run_ms, (sa + sc) / double(p->ev_used));
            p->ev_used = 0;
            int cnt[4] = {};
            HIP_TRY(hipMemcpy(cnt, p->d_count, sizeof(cnt), hipMemcpyDeviceToHost));
            // in-wave attempts past the limit were appended to the list instead
            st->n_rescued += cnt[p->parity ^ 1] + std::min(cnt[2 + (p->parity ^ 1)], p->inker_limit);
        }
    }
    return HC_PHMM_OK;
}

int hc_phmm_batch_destroy(hc_phmm_batch* b)
{
    if (!b) return HC_PHMM_OK;
    for (Part* p : b->parts) {
        (void)hipSetDevice(p->dev->ordinal);
        if (p->last_stream) (void)hipStreamSynchronize(p->last_stream);
        free_part(p);
    }
    delete b;
    return HC_PHMM_OK;
}

// ---- host-planning timing hooks (not part of the ABI: tools/plan_bench.py)
// Plan a call's parts on the host only, as submit would on `n_dev` slots of
// `n_cu` compute units, `reps` times; HC_PHMM_TRACE=1 prints the phases.
// Returns the mean milliseconds per call.
double hcx_plan_pairs(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off, const int32_t* H,
                      const uint8_t* rs, const uint8_t* q, const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
                      const uint8_t* hap, int n_cu, int n_dev, int reps)
{
    const Src src = flat_src(read_off, R, hap_off, H, rs, q, ins, del, gcp, hap);
    Device fake;
    fake.n_cu = n_cu;
    g_dry = true;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < reps; ++k) {
        std::vector<int64_t> pre;
        prefix_sum(n, pre, [&](int64_t p) { return int64_t(std::max(0, R[p])) * std::max(0, H[p]); });
        const int np = part_count(pre.back(), n_dev);
        const std::vector<int64_t> cut = equal_cuts(pre, np);
        for (int j = 0; j < np; ++j) {
            PartSpec s;
            s.lo = cut[size_t(j)];
            s.hi = cut[size_t(j) + 1];
            Part* p = nullptr;
            (void)plan_part(fake, src, s, nullptr, false, &p);
        }
    }
    g_dry = false;
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / reps;
}

// The last traced segmented pass (HC_PHMM_TIMELINE=1): up to max_waves
// records of {start, end, HW_ID} into out; returns the record count.
int hcx_timeline(unsigned long long* out, int max_waves)
{
    std::lock_guard<std::mutex> lk(g_tl.mu);
    if (!g_tl.buf || g_tl.n == 0) return 0;
    const int n = std::min(max_waves, g_tl.n);
    if (hipStreamSynchronize(g_tl.stream) != hipSuccess) return -1;
    if (hipMemcpy(out, g_tl.buf, size_t(n) * 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return n;
}

// Sizes of the last dry-run plan: {pairs, order entries, segmented slots,
// segmented waves, structured (1) or general (0) planner}.
void hcx_dump_sizes(int64_t* out5)
{
    std::lock_guard<std::mutex> lk(g_dump.mu);
    out5[0] = int64_t(g_dump.pairs.size());
    out5[1] = int64_t(g_dump.order.size());
    out5[2] = g_dump.n_seg_slots;
    out5[3] = int64_t(g_dump.waves.size());
    out5[4] = g_dump.grid ? 1 : 0;
}

// The last dry-run plan: pairs as {row offset, R, table offset, H}, the slot
// order, and per segmented wave {slot0, rmax, rmin, ncols, npairs, nsteps}.
void hcx_dump_plan(int32_t* pairs4, int32_t* order, int32_t* waves6)
{
    std::lock_guard<std::mutex> lk(g_dump.mu);
    for (size_t k = 0; k < g_dump.pairs.size(); ++k) {
        const int4 p = g_dump.pairs[k];
        pairs4[4 * k] = p.x;
        pairs4[4 * k + 1] = p.y;
        pairs4[4 * k + 2] = p.z;
        pairs4[4 * k + 3] = p.w;
    }
    std::copy(g_dump.order.begin(), g_dump.order.end(), order);
    for (size_t w = 0; w < g_dump.waves.size(); ++w) {
        const LaneWave& v = g_dump.waves[w];
        const int32_t f[6] = {v.slot0, v.rmax, v.rmin, v.ncols, v.npairs, v.nsteps};
        std::copy(f, f + 6, waves6 + 6 * w);
    }
}

double hcx_plan_regions(const hc_phmm_region* regions, int32_t n_regions, int n_cu, int reps)
{
    RegionSet rs;
    if (gather_regions(regions, n_regions, rs)) return -1;
    Src src;
    src.reads = rs.reads.data();
    src.haps = rs.haps.data();
    Device fake;
    fake.n_cu = n_cu;
    PartSpec s;
    s.flat = false;
    s.blocks = rs.blocks;
    g_dry = true;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < reps; ++k) {
        Part* p = nullptr;
        (void)plan_part(fake, src, s, nullptr, false, &p);
    }
    g_dry = false;
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / reps;
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
    std::vector<double> out(static_cast<size_t>(batch.num_reads) * size_t(batch.num_haps));
    const int rc = hc_phmm_cross(reinterpret_cast<const hc_phmm_read*>(batch.reads), batch.num_reads,
                                 reinterpret_cast<const hc_phmm_hap*>(batch.haps), batch.num_haps, out.data());
    if (rc != HC_PHMM_OK) return false;
    for (size_t k = 0; k < out.size(); ++k) batch.results[k] = float(out[k]);
    return true;
}
}  // namespace shacc_pairhmm
