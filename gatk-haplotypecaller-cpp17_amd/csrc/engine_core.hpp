// Internal interface of the PairHMM host engine (libhcpairhmm.so), shared by
//   device.cpp   device slots: init / shutdown, per-slot streams + workspaces
//   planner.cpp  host planning of a part: length binning, wave packing, staging
//   flat_plan.cpp  flat batches planned on the device (the real call path)
//   run.cpp      the device pass of a part and the host log10 finish
//   api.cpp      splitting calls into parts, submit / collect, the C ABI
//
// The reference's computeLikelihoodsNative (intel_pairhmm.hpp:115-152) split
// into plan / execute / finish over one or more device slots:
//   plan     (host) length-bin the pairs and pack them into waves, or (flat
//            calls) only stage the raw inputs and let the device plan them
//   execute  (device) H2D, pack rows + hap match tables, fp32 kernels ->
//            raw f32 + rescue list, fp64 rescue over the list, D2H of results
//   finish   (host) glibc log10f / log10 exactly as intel_pairhmm.hpp:137-143,
//            scattered into the caller's outputs
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hc_pairhmm.h"
#include "kernels.hpp"

namespace hcphmm {

// Shared with sw_engine.cpp / gt_engine.cpp.
void set_last_error(const std::string& msg);
int primary_device();   // HIP ordinal of the first device slot, -1 if not initialised
void sw_release();      // sw_engine.cpp: drop the aligner's stream and workspace
void gt_release();      // gt_engine.cpp: drop the genotyper's stream and buffers

namespace eng {

int fail(int code, const std::string& msg);

#define HIP_TRY(expr)                                                                                 \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return ::hcphmm::eng::fail(HC_PHMM_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int64_t env_i64(const char* name, int64_t dflt);
// Test hook (hcx_test_plan_timeout, api.cpp): the fp64 launch's non-planner
// workgroups give up waiting for the plan at once. Off unless a test sets it;
// no environment variable reaches it.
bool test_plan_timeout();

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

// ---------------------------------------------------------------------------
// Device slots (device.cpp).

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
    hipEvent_t ev[7] = {};   // pack [2], fp32 / fp64 pass [3], done, early results: reused by every part in the slot
    hipEvent_t up_ev[2] = {};   // staging halves: H2D of a half done (timing disabled)
};

// Pinned staging ring of a device: the flat call path streams its upload
// through these chunks (fill chunk k on the host while chunk k-1 is copied),
// so no call allocates pinned memory; allocated once at init.
constexpr int kRingN = 4;
constexpr size_t kRingChunk = size_t(32) << 20;
struct Ring {
    std::mutex mu;   // held by one part's fill at a time
    char* buf[kRingN] = {};
    hipEvent_t ev[kRingN] = {};   // the last H2D out of each chunk
    bool used[kRingN] = {};
    int next = 0;
};

struct Device {
    int ordinal = 0;
    int n_cu = 256;   // compute units (4 SIMDs each): sizes the latency models
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;                  // segmented waves beside one-lane waves
    hipStream_t aux = nullptr;                   // speculative fp64 beside the fp32 pass
    hipEvent_t fork = nullptr, join = nullptr;   // side-stream fork / join (timing disabled)
    float* lut_f = nullptr;
    double* lut_d = nullptr;
    std::vector<Slot*> slots;
    double outstanding = 0;   // cells submitted and not yet collected
    Ring ring;
    // Host staging time of flat parts (scan + fill), ps per cell, a running
    // mean over the calls so far (0: none yet): sizes a call's parts
    // (api.cpp submit_flat, HC_PHMM_PART_GROWTH_PCT).
    std::atomic<double> stage_ps_per_cell{0.0};
    // Flat parts left to start with the nibble records without trying the
    // compact ones: set when a part's compact attempt is refused in pass 2 (a
    // rare 'N' its sample missed), so data that carries them pays one refusal
    // per kNibbleParts parts, not one per part (flat_plan.cpp plan_flat_device).
    std::atomic<int> nibble_parts{0};
};
constexpr int kNibbleParts = 64;

// Engine state, guarded by g_mu: the device list, the slot pools, the
// outstanding counters, and the number of parts alive and calls running (a
// shutdown while either is non-zero is refused: parts hold Device / Slot
// pointers).
extern std::mutex g_mu;
extern std::vector<Device*> g_devs;
extern int64_t g_live_parts;
extern int64_t g_active_calls;
// hc_phmm_init flags of the most recent successful init (HC_PHMM_FLAG_*): the
// default mode of later calls and batches (HC_PHMM_FLAG_F64 = initNative(
// use_double = true)), captured into each PartSpec when the call is made.
extern std::atomic<uint32_t> g_flags;

int init_devices_locked(const int32_t* devices, int32_t n, bool any_ok);
// Slots made at hc_phmm_init per device (a flat call of S2's size runs 8
// parts; more are made on demand).
constexpr int kInitSlots = 8;
Slot* make_slot();   // a new idle slot of the current device (streams, events)
Slot* take_slot(Device& d);
void give_slot(Slot* s);
int slot_reserve(Slot& s, size_t dev_bytes, size_t host_bytes);
void release_device(Device* d);

// A call in progress: initialises the engine on first use and snapshots the
// device list; shutdown is refused while any call holds one.
class CallGuard {
public:
    CallGuard();
    ~CallGuard();
    CallGuard(const CallGuard&) = delete;
    CallGuard& operator=(const CallGuard&) = delete;
    int rc = HC_PHMM_OK;
    std::vector<Device*> devs;
};

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
    // hc_phmm_init flags of the call (HC_PHMM_FLAG_F64 = initNative's
    // use_double), fixed when the call is made: the reference's g_use_double
    // is per IntelPairHMM instance (intel_pairhmm.hpp:58,81), so a later init
    // from another thread must not switch the mode of work already submitted.
    uint32_t flags = 0;
    // Parts below this many pairs write results in place instead of per-slot
    // records (run.cpp); -1: HC_PHMM_REC_MIN_PAIRS (200 000). A part of a
    // pipelined call takes 40 000: its gather's latency is hidden behind the
    // next part's staging.
    int64_t rec_min = -1;
    double cells = 0;   // R x H summed over the part's pairs (flat parts)
};

// Planning modes: a real part (device calls), or a dry run that plans on the
// host only and keeps the plan for the host-logic tests (hcx_* hooks).
enum class PlanMode { Real, Dry };

// A part's results block, one contiguous device range returned to the host by
// one store (enqueue_results): [raw32 | raw64 | flag | run counters]. The run
// counters (kNumCounters ints, kernels.hpp) ride along so the host sees the
// device error word (kErrWord) with the results, at no extra transfer.
struct ResLayout {
    size_t o64, ofl, ocnt, bytes;
};
inline ResLayout res_layout(size_t n1)
{
    ResLayout r;
    r.o64 = (sizeof(float) * n1 + 255) & ~size_t(255);
    r.ofl = r.o64 + ((sizeof(double) * n1 + 255) & ~size_t(255));
    r.ocnt = (r.ofl + n1 + 255) & ~size_t(255);
    r.bytes = (r.ocnt + kNumCounters * sizeof(int) + 15) & ~size_t(15);   // whole 16-byte stores (launch_store_to_host)
    return r;
}

// ---------------------------------------------------------------------------
// A part prepared on one device: every device array lives in one allocation,
// filled by H2D copies from one pinned staging image.
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
    const int* d_nwaves = nullptr;   // device-planned parts: the wave count lives on the device
    int max_seg_waves = 0;           //   and this bounds it (the launch grid)
    int* d_lane_order = nullptr;
    LaneWave* d_lane_waves = nullptr;
    float2* d_carry = nullptr;
    void* d_ring = nullptr;        // anti-diagonal rings beyond the LDS (planner.cpp)
    PairDesc* d_pairs = nullptr;
    uint32_t* d_rows = nullptr;
    uint32_t* d_hapw = nullptr;
    float* d_raw32 = nullptr;     // current output targets (own or bound)
    double* d_raw64 = nullptr;
    uint8_t* d_flag = nullptr;
    float* own_raw32 = nullptr;   // outputs in the part's allocation: [raw32 | raw64 | flag]
    double* own_raw64 = nullptr;
    uint8_t* own_flag = nullptr;
    size_t res_bytes = 0;         // bytes of that contiguous output block (ResLayout)
    size_t res_o64 = 0, res_ofl = 0, res_ocnt = 0;
    uint4* d_rec = nullptr;       // seg slot result records (LaneArgs::rec), gathered by the fp64 launch
    int* d_slot_of = nullptr;     // pair -> seg slot (-1: one-lane / anti-diagonal pair)
    PairDesc* d_sdesc = nullptr;  // seg slot -> pair descriptor (pairs[order[slot]])
    int* d_list = nullptr;
    int* d_sorted = nullptr;
    int* d_worder = nullptr;      // fp64 pass: dispatch position -> wave
    int* d_big = nullptr;
    int* d_big_count = nullptr;
    Seg64Plan* d_plan = nullptr;
    int64_t n_wide = 0;
    int wide_ring_blocks = 0;     // fp64 wide pass: workgroups its global ring has room for (0: ring in LDS)
    int* d_count = nullptr;
    int inker_limit = 0;   // in-wave rescues allowed in the last run
    int parity = 0;
    char* dev_base = nullptr;
    Slot* slot = nullptr;         // borrowed workspace (jobs), else dev_base is owned
    char* host_res = nullptr;     // pinned results image (slot) after the D2H
    size_t upload_bytes = 0;
    hipEvent_t pack_ev[2] = {nullptr, nullptr};
    hipEvent_t done = nullptr;    // jobs: D2H complete
    // Jobs: the fp32 pass's raw sums and flags on the host while the fp64
    // launch runs (run_part), so collect() finishes the unflagged pairs early.
    hipEvent_t early = nullptr;   // the slot's; null: never
    bool early_used = false;      // the last run stored them early
    std::vector<std::array<hipEvent_t, 3>> ev_pool;
    std::vector<uint8_t> ev_solo;   // per pooled run: no fp64 launch, ev[2] not recorded (ev[1] ends the run)
    size_t ev_used = 0;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool slot_ev = false;         // pack_ev / ev / done are the slot's (not destroyed here)
    hipStream_t stream = nullptr;             // the part's stream: its slot's, else its device's
    hipStream_t side = nullptr;               // segmented waves beside one-lane waves
    hipEvent_t fork = nullptr, join = nullptr;
    hipStream_t last_stream = nullptr;
    int64_t launch_waves = 0;
    bool ran = false;
    unsigned long long* timeline = nullptr;   // HC_PHMM_TIMELINE=1: this part's wave records
    int timeline_n = 0;                       //   (allocated), of which the fp32 seg waves' first,
    int timeline_n32 = 0;                     //   then the fp64 waves' (Seg64Args::timeline)
};

Part* new_part(Device* d);   // counted in g_live_parts
void free_part(Part* p);
void discard_part(Part* p);  // failed before hand-out: the slot and its memory stay with the caller

// A part under construction: discarded (after its stream drains) when the
// planner leaves by an error return or an exception, unless handed out.
class PartGuard {
public:
    explicit PartGuard(Part* p) : p_(p) {}
    ~PartGuard()
    {
        if (!p_) return;
        if (p_->stream) (void)hipStreamSynchronize(p_->stream);
        discard_part(p_);
    }
    PartGuard(const PartGuard&) = delete;
    PartGuard& operator=(const PartGuard&) = delete;
    Part* release()
    {
        Part* q = p_;
        p_ = nullptr;
        return q;
    }

private:
    Part* p_;
};

// planner.cpp: plan one part on device d (host planning + staging, then the
// H2D, device packing and, with_run, the device pass and the D2H of the
// results, all enqueued on the part's stream). slot == nullptr: the part owns
// its memory (batches). Dry runs stop after planning (*out = nullptr).
int plan_part(Device& d, const Src& src, const PartSpec& spec, Slot* slot, bool with_run, PlanMode mode,
              Part** out);
// flat_plan.cpp: a flat part whose pairs are planned on the device; returns
// HC_PHMM_OK with *out = nullptr when the batch needs the host planner.
int plan_flat_device(Device& d, const Src& src, const PartSpec& spec, Slot* slot, bool with_run, Part** out);
// run.cpp
int run_part(Part* b, hipStream_t s);
// which: every pair; the unflagged ones only (their raw f64 is 0: d unread);
// the flagged ones only.
enum class Finish { All, Plain, Rescued };
void finish_part(const Part& P, const float* f, const double* d, const uint8_t* fl, const Outputs& o,
                 Finish which = Finish::All);
// Enqueue the results' return to the pinned host image and the part's done
// event (with_run parts). A kernel stores them into the mapped host memory
// rather than a DMA copy: DMA copies run in enqueue order, so a D2H enqueued
// behind its part's kernels held the next part's uploads until those kernels
// finished (the parts of a call ran one after another: S2 end to end 22 ms).
// ConvertChar codes (pairhmm_common.h:26-44: A0 C1 T2 G3 N4, other bytes 0) of n bases, two per byte,
// base k in the low nibble of byte k / 2 when k is even (AVX2 when the CPU
// has it; flat_plan.cpp).
void pack_nibbles(const uint8_t* s, int n, uint8_t* d);
int enqueue_results(Part* b, hipStream_t s);
int check_device_error(const int* counters);   // run.cpp: counters = a host copy of a part's run counters

// The last dry-run plan (hcx_dump_sizes / hcx_dump_plan).
struct DryDump {
    std::mutex mu;
    std::vector<int4> pairs;
    std::vector<int> order;
    std::vector<LaneWave> waves;
    int n_seg_slots = 0;
    bool grid = false;
};
extern DryDump g_dump;

// HC_PHMM_TIMELINE=1 diagnostics: the last traced part's records.
struct TimelineRef {
    std::mutex mu;
    const Part* part = nullptr;
    unsigned long long* buf = nullptr;
    int n = 0;
    hipStream_t stream = nullptr;
    int ordinal = 0;
};
extern TimelineRef g_tl;

}  // namespace eng
}  // namespace hcphmm

struct hc_phmm_batch {
    std::vector<hcphmm::eng::Part*> parts;   // one per device slot
    int64_t n = 0;
};

struct hc_phmm_job {
    std::vector<hcphmm::eng::Part*> parts;
    hcphmm::eng::Outputs out;
    std::vector<double> cells_per_part;
};
