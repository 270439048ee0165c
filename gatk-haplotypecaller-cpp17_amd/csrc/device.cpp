// Device slots of the PairHMM engine: initialisation on one or several GPUs
// (initNative, intel_pairhmm.hpp:77-113: the LUTs and the FTZ environment,
// here the device tables and the kernels' denormal mode), per-slot streams
// and grow-only workspaces, and the lifetime rules that make shutdown safe.
#include <algorithm>
#include <cstring>

#include "engine_core.hpp"
#include "luts.hpp"

namespace hcphmm {
namespace eng {

namespace {
thread_local std::string g_err;
}

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

const char* last_error() { return g_err.c_str(); }

int64_t env_i64(const char* name, int64_t dflt)
{
    const char* e = std::getenv(name);
    return (e && *e) ? std::atoll(e) : dflt;
}

std::mutex g_mu;
std::vector<Device*> g_devs;
int64_t g_live_parts = 0;
int64_t g_active_calls = 0;
std::atomic<uint32_t> g_flags{0};
bool g_shutting = false;
DryDump g_dump;
TimelineRef g_tl;

namespace {
// Host copy of the last traced part's records once that part is freed.
std::vector<unsigned long long> g_tl_saved;
int g_tl_saved_n32 = 0;
}

void release_device(Device* d)
{
    if (!d) return;
    (void)hipSetDevice(d->ordinal);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    if (d->aux) (void)hipStreamSynchronize(d->aux);
    for (Slot* s : d->slots) {
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        if (s->side) (void)hipStreamSynchronize(s->side);
        if (s->dev) (void)hipFree(s->dev);
        if (s->host) (void)hipHostFree(s->host);
        for (auto& e : s->ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : s->up_ev)
            if (e) (void)hipEventDestroy(e);
        if (s->fork) (void)hipEventDestroy(s->fork);
        if (s->join) (void)hipEventDestroy(s->join);
        if (s->side) (void)hipStreamDestroy(s->side);
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
    }
    for (int k = 0; k < kRingN; ++k) {
        if (d->ring.ev[k]) (void)hipEventSynchronize(d->ring.ev[k]);
        if (d->ring.ev[k]) (void)hipEventDestroy(d->ring.ev[k]);
        if (d->ring.buf[k]) (void)hipHostFree(d->ring.buf[k]);
    }
    if (d->lut_f) (void)hipFree(d->lut_f);
    if (d->lut_d) (void)hipFree(d->lut_d);
    if (d->fork) (void)hipEventDestroy(d->fork);
    if (d->join) (void)hipEventDestroy(d->join);
    if (d->aux) (void)hipStreamDestroy(d->aux);
    if (d->side) (void)hipStreamDestroy(d->side);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

namespace {

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
    HIP_TRY(hipStreamCreateWithFlags(&d.aux, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&d.fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.join, hipEventDisableTiming));
    const Luts& L = luts();
    HIP_TRY(hipMalloc(&d.lut_f, sizeof(float) * kTableLen));
    HIP_TRY(hipMalloc(&d.lut_d, sizeof(double) * kTableLen));
    HIP_TRY(hipMemcpy(d.lut_f, L.dev_f.data(), sizeof(float) * kTableLen, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d.lut_d, L.dev_d.data(), sizeof(double) * kTableLen, hipMemcpyHostToDevice));
    for (int k = 0; k < kRingN; ++k) {
        if (hipHostMalloc(&d.ring.buf[k], kRingChunk, hipHostMallocPortable) != hipSuccess)
            return fail(HC_PHMM_ENOMEM, "pinned staging ring");
        HIP_TRY(hipEventCreateWithFlags(&d.ring.ev[k], hipEventDisableTiming));
    }
    // The slots (streams + events) of a call cut into the usual part count,
    // made here rather than by the first call that needs them: each slot's
    // streams and events cost the first call ~1 ms of its host pipeline
    // (verdict round 5, item 4). Their memory still grows on first use.
    // Their workspaces are sized here too (grow-only afterwards):
    // HC_PHMM_INIT_SLOT_MB of device memory each (default 320: a pipelined
    // S2 part of up to 250k pairs needs ~300 MB) and 8 MB of pinned host
    // memory for the results; each hipMalloc / pinned allocation took ~1.4 ms
    // of a first call's host pipeline, per part.
    const int64_t slot_mb = std::max<int64_t>(0, env_i64("HC_PHMM_INIT_SLOT_MB", 320));
    for (int k = 0; k < kInitSlots; ++k) {
        Slot* s = make_slot();
        if (!s) return HC_PHMM_EHIP;
        d.slots.push_back(s);   // (under g_mu: init_devices_locked)
        if (slot_mb > 0) {
            const int rc = slot_reserve(*s, size_t(slot_mb) << 20, size_t(8) << 20);
            if (rc) return rc;
        }
    }
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

}  // namespace

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

CallGuard::CallGuard()
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_shutting) {   // hc_phmm_shutdown has committed: no new work
        rc = fail(HC_PHMM_ENODEV, "the engine is shutting down");
        return;
    }
    const int32_t cur = -1;
    rc = init_devices_locked(&cur, 1, true);
    if (rc) return;
    devs = g_devs;
    ++g_active_calls;
}

CallGuard::~CallGuard()
{
    if (rc) return;
    std::lock_guard<std::mutex> lk(g_mu);
    --g_active_calls;
}

// A new idle slot of the current device: its streams and events (no memory
// yet); nullptr (and the engine error set) if they cannot be created.
Slot* make_slot()
{
    auto* s = new Slot();
    bool ok = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&s->fork, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&s->join, hipEventDisableTiming) == hipSuccess;
    for (int k = 0; ok && k < 7; ++k)
        ok = hipEventCreateWithFlags(&s->ev[k], k >= 5 ? hipEventDisableTiming : 0) == hipSuccess;
    for (int k = 0; ok && k < 2; ++k) ok = hipEventCreateWithFlags(&s->up_ev[k], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        for (auto& e : s->ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : s->up_ev)
            if (e) (void)hipEventDestroy(e);
        if (s->fork) (void)hipEventDestroy(s->fork);
        if (s->join) (void)hipEventDestroy(s->join);
        if (s->side) (void)hipStreamDestroy(s->side);
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
        fail(HC_PHMM_EHIP, "slot stream / event creation");
        return nullptr;
    }
    return s;
}

// A free slot of device d (d current on the calling thread); a new one if
// every slot is busy (hc_phmm_init creates kInitSlots).
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
    Slot* s = make_slot();
    if (!s) return nullptr;
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

Part* new_part(Device* d)
{
    auto* p = new Part();
    p->dev = d;
    std::lock_guard<std::mutex> lk(g_mu);
    ++g_live_parts;
    return p;
}

void free_part(Part* p)
{
    if (!p) return;
    if (p->dev) (void)hipSetDevice(p->dev->ordinal);
    if (p->timeline) {
        std::lock_guard<std::mutex> lk(g_tl.mu);
        if (p->last_stream) (void)hipStreamSynchronize(p->last_stream);
        if (g_tl.part == p) {
            g_tl_saved.assign(size_t(p->timeline_n) * 3, 0ull);
            (void)hipMemcpy(g_tl_saved.data(), p->timeline, g_tl_saved.size() * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost);
            g_tl_saved_n32 = p->timeline_n32;
            g_tl.part = nullptr;
        }
        (void)hipFree(p->timeline);
    }
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
    std::lock_guard<std::mutex> lk(g_mu);
    --g_live_parts;
}

// A part that failed before it was handed out: its slot stays with the
// caller (who returns it) and so does the slot's memory the part borrowed.
void discard_part(Part* p)
{
    if (!p) return;
    if (p->slot) {
        p->dev_base = nullptr;
        p->slot = nullptr;
    }
    free_part(p);
}

// Records of the last traced part (alive: read from the device; freed: the copy
// saved at free_part).
// fp64: the fp64 waves' records (after the fp32 seg waves').
int timeline_records(unsigned long long* out, int max_waves, bool fp64)
{
    std::lock_guard<std::mutex> lk(g_tl.mu);
    if (g_tl.part) {
        const Part* p = g_tl.part;
        const int off = fp64 ? p->timeline_n32 : 0;
        const int n = std::min(max_waves, fp64 ? p->timeline_n - p->timeline_n32 : p->timeline_n32);
        (void)hipSetDevice(p->dev->ordinal);
        if (hipStreamSynchronize(p->last_stream) != hipSuccess) return -1;
        if (hipMemcpy(out, p->timeline + 3 * size_t(off), size_t(n) * 3 * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
        return n;
    }
    const int tot = int(g_tl_saved.size() / 3);
    const int off = fp64 ? g_tl_saved_n32 : 0;
    const int n = std::min<int>(max_waves, fp64 ? tot - g_tl_saved_n32 : g_tl_saved_n32);
    std::copy(g_tl_saved.begin() + 3 * size_t(off), g_tl_saved.begin() + 3 * size_t(off + n), out);
    return n;
}

// hc_phmm_shutdown, in two steps so that the decision is taken once, under
// g_mu: begin_shutdown refuses while a call runs or a part (job / batch) is
// alive, else commits (new calls are refused from then on, so nothing can
// become live again); the caller then releases the aligner and genotyper, and
// finish_shutdown drops the devices.
int begin_shutdown()
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_shutting) return fail(HC_PHMM_EINVAL, "shutdown already in progress");
    if (g_active_calls > 0 || g_live_parts > 0)
        return fail(HC_PHMM_EINVAL, "shutdown while " + std::to_string(g_active_calls) + " call(s) run and " +
                                        std::to_string(g_live_parts) +
                                        " part(s) of uncollected jobs / live batches exist: collect and destroy "
                                        "them first");
    g_shutting = true;
    return HC_PHMM_OK;
}

int finish_shutdown()
{
    std::lock_guard<std::mutex> lk(g_mu);
    for (Device* d : g_devs) release_device(d);
    g_devs.clear();
    g_flags.store(0);
    g_shutting = false;
    return HC_PHMM_OK;
}

}  // namespace eng

void set_last_error(const std::string& msg) { eng::fail(0, msg); }
int primary_device()
{
    std::lock_guard<std::mutex> lk(eng::g_mu);
    return eng::g_devs.empty() ? -1 : eng::g_devs[0]->ordinal;
}

}  // namespace hcphmm
