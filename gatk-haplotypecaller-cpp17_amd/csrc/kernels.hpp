// Device-side layout shared by the HIP kernels and the host engine.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace hcphmm {

// One row of a read, packed into 32 bits (built on the device, pack_kernels.hip):
//   bits  0- 6  q  (base quality byte & 127)
//   bits  7-13  i  (insertion GOP byte & 127)
//   bits 14-20  d  (deletion GOP byte & 127)
//   bits 21-27  c  (gap continuation byte & 127)
//   bits 28-30  read base code, ConvertChar (pairhmm_common.h:26-44): A0 C1 T2 G3 N4
//   bit  31     first row of a read only: the read's gap qualities are constant
//               (found on the host while staging, set by the packer)
__host__ __device__ inline uint32_t pack_row(int q, int i, int d, int c, int code)
{
    return uint32_t(q & 127) | (uint32_t(i & 127) << 7) | (uint32_t(d & 127) << 14) |
           (uint32_t(c & 127) << 21) | (uint32_t(code) << 28);
}

// Haplotype match table: for hap of length H, nw = ceil(H/32) data words,
// stored as (nw + kHapPadWords) rows of 5 uint32 — row (w + kHapLead) holds,
// for each read code rc, the bits of columns 32w+1 .. 32w+32 (MSB first) whose
// hap base matches rc: equal code, or hap 'N' (matches every rc), or rc = 'N'
// (matches every column). This is the reference's precompute_masks
// (avx-pairhmm-template.h:3-35) laid out for per-lane windows. kHapLead zero
// rows precede the data (columns <= 0), one zero row follows.
constexpr int kHapLead = 2;
constexpr int kHapPadWords = 3;
inline int hap_table_words(int H) { return ((H + 31) / 32 + kHapPadWords) * 5; }

// Per pair descriptor: {row offset into rows[], R, word offset into hapw[], H}.
using PairDesc = int4;
// Words of slack before the packed rows (the column-segmented kernels
// prefetch read words ahead without clamping). The kernels address a row word
// as a 32-bit byte offset from rows - kRowPadBefore (one VGPR per lane, the
// base in SGPRs), so a part's rows + slack stay below kMaxRowWords.
constexpr long long kRowPadBefore = 256;
constexpr long long kMaxRowWords = (1ll << 30) - 1024;
// Hap match tables are addressed the same way (32-bit byte offsets from the
// part's table base, seg_common.hpp LaneCtx::hbyte): a part's tables stay
// below 2^30 words too (advisor round 4).
constexpr long long kMaxHapWords = (1ll << 30) - 1024;

// Run counters of a part (zeroed when the part is prepared): [0, 1] rescue
// list lengths and [2, 3] in-wave rescue counts, by run parity (a run zeroes
// the other parity's for the next run: no memset per run); [4] the fp64
// pass's wave counter (zeroed by its plan each run); [5..8] the fp64
// planner's ticket and flag, by parity likewise.
constexpr int kNextWave = 4;
constexpr int kPlanTicket = 5;   // [5, 6] fp64 planner ticket, [7, 8] plan-published flag, by run parity
constexpr int kPlanReady = 7;
// [12] device error word (sticky, not by parity): a kernel that cannot finish
// its share sets a bit here instead of leaving results silently undone; the
// host reads it with the results (the counters are the last field of a part's
// results block, so the D2H of a call brings them along) and fails the call
// with HC_PHMM_EHIP. Batches clear it when they report it.
constexpr int kErrWord = 12;
constexpr int kErrPlanWait = 1;   // fp64 pass: a workgroup gave up waiting for the rescue plan
constexpr int kNumCounters = 16;
static_assert(kNumCounters <= 256, "the prep kernels zero the counters with one 256-thread block");

struct DiagArgs {
    const PairDesc* pairs;
    const int* order;         // slot -> pair id (caller order)
    int n_slots;              // number of slots when n_slots_dev == nullptr
    const int* n_slots_dev;   // device-side slot count (rescue list)
    const uint32_t* rows;
    const uint32_t* hapw;
    const void* lut;          // float or double table, luts.hpp layout
    int ring_len;             // ring entries per pair group (LDS)
    void* raw_out;            // float[n_pairs] or double[n_pairs], by pair id
    uint8_t* rescue_flag;     // fp32 pass: 1 if raw < 1e-28f (by pair id)
    int* rescue_list;         // fp32 pass: appended pair ids
    int* rescue_rh;           // fp32 pass: each appended pair's pack_rh(R, H) (the fp64 plan reads it)
    int* rescue_count;        // fp32 pass: append counter
    double* raw64_zero;       // fp32 pass: raw f64 result slot of each pair, zeroed
                              // (the rescue pass overwrites the rescued ones)
    int* count_reset;         // fp64 pass: the other run parity's rescue counter,
                              // zeroed for the next run (no memset per run)
    void* ring_global;        // stripe hand-off ring in global memory (block b: entries
                              // [b * G * ring_len, ...)) when it exceeds the LDS; null = LDS
};

// fp64 rescue pass in column-segmented form, planned on the device
// (lane_kernel.hip rescue_plan_kernel). A pair takes a slot of 2^k lanes
// (64 >> k pairs per wave) and the narrowest fp64 block width that covers its
// hap on those lanes, so the slot's lanes are all used: (k, width) is its
// class. Classes are numbered widest slot and block first (the longest waves
// are dispatched first); the last class holds haps wider than 64 blocks of 32
// (anti-diagonal kernel, through `big`). In passes of many waves the 64-lane
// pairs (haps over 1 024 columns) are mostly chained: a chain class per width,
// numbered before the others, whose waves stream up to `chain` pairs through
// the same 64 lanes one after the other (lane_kernel.hip chain_run: the 63-step
// skew of a 64-lane pair paid once per chain instead of once per pair).
// A rescue list entry's R and H for the fp64 plan, written beside the pair id
// (each clamped to 16 bits: H only selects the class, past 2 048 columns the
// anti-diagonal one, and R only prices the wave).
__host__ __device__ inline int pack_rh(int R, int H)
{
    return ((R < 65535 ? R : 65535) << 16) | (H < 65535 ? H : 65535);
}
constexpr int kSeg64Widths = 7;   // fp64 block widths 8, 12, ..., 32
constexpr int kChainClasses = kSeg64Widths;
constexpr int kMaxChain = 4;
constexpr int kSeg64Classes = kChainClasses + 7 * kSeg64Widths + 1;
constexpr int kSeg64MaxH = 64 * 32;   // longer haps: anti-diagonal fp64 kernel (host n_wide)
__host__ __device__ constexpr int seg64_width(int wi) { return 8 + 4 * wi; }
struct Seg64Plan {
    int bc0;                        // block width bound of the pass (32, or 16 / 8 for short lists)
    int dynamic;                    // waves fetched from a counter (more than two per SIMD)
    int chain;                      // pairs per wave of the chain classes (1: none chained)
    int n_class[kSeg64Classes];
    int off_class[kSeg64Classes];   // class c's entries in `sorted` start here
    int wave_base[kSeg64Classes];   // first wave of class c; [last] = total waves
};
struct Seg64Args {
    const PairDesc* pairs;
    const uint32_t* rows;
    const uint32_t* hapw;
    const double* lut;
    int* list;                // rescue list (fp32 pass, arbitrary order)
    const int* list_rh;       // each entry's pack_rh(R, H): the plan's walks read it coalesced
    const int* count;         // its length
    int* count_reset;         // the other run parity's counter, zeroed for the next run
    int* inker_reset;         // the other run parity's in-wave rescue counter, likewise
    int* ticket;              // this run's planner ticket (the first workgroup to take it plans)
    int* ready;               // this run's plan-published flag
    int* ticket_reset;        // the other run parity's ticket and flag, zeroed for the next run
    int* ready_reset;
    int* sorted;              // list in class order (n entries)
    int* big;                 // last-class pairs (anti-diagonal fp64 kernel)
    int* big_count;
    Seg64Plan* plan;
    double* raw_out;          // raw f64 sums by pair id
    long long min_lanes;      // narrower blocks below this many lanes at bc = 32
    int* wave_order;          // dispatch position -> wave (n entries), see rescue_plan_kernel
    int* next_wave;           // dynamic wave counter (zeroed by the plan)
    int chain;                // longest chain of 64-lane pairs in one wave (1: no chains)
    int chain_tail;           // rounds of single 64-lane waves (two per SIMD) kept unchained at the end
    int n_simd;               // SIMDs of the device (4 per CU)
    // Gather of the seg slots' result records (LaneArgs::rec) into the
    // per-pair outputs, done by this launch before its rescue work: pair p's
    // slot is slot_of[p] (-1: computed by another kernel, already in place).
    const uint4* rec;         // null: nothing to gather
    const int* slot_of;
    int n_pairs;
    float* raw32;
    uint8_t* flag;
    int prio;   // as LaneArgs::prio
    int* err;                 // the part's error word (kErrWord): kErrPlanWait on a plan-wait timeout
    // Diagnostics (HC_PHMM_TIMELINE=1): per fp64 wave w (class order), record
    // timeline[3 * w] = {start, end, HW_ID | XCC_ID << 32 | first pair id << 40};
    // record n_pairs: {the planner workgroup's start, plan published, list
    // length}; null = off.
    unsigned long long* timeline;
    int force_plan_timeout;   // test hook (hcx_test_plan_timeout): non-planner workgroups time out at once
};
// Lane-per-pair kernel (large batches): one lane owns one pair and sweeps it
// row by row over register-resident blocks of kLaneBlock columns. A wave holds
// 64 length-binned pairs; wave_meta gives its rows (max R) and column coverage.
constexpr int kLaneBlock = 64;
struct LaneWave {
    int slot0;      // first slot of the wave in `order`
    int rmax;       // rows swept (max R of the wave's pairs)
    int rmin;       // min R of the wave's pairs (first row that may need the sum)
    int ncols;      // one-lane waves: columns swept (max H rounded up to 16);
                    // column-segmented waves: block width BC (seg_width_ok)
    int npairs;     // column-segmented waves: pairs in the wave (slot0 ..)
    int nsteps;     // column-segmented waves: steps = max over pairs of R + nb - 1
    long long carry_row;  // one-lane waves: first carry row in `carry` (units of 64 float2)
};
struct LaneArgs {
    const PairDesc* pairs;
    const int* order;
    int n_slots;
    int n_waves;              // waves launched (an upper bound when n_waves_dev is set)
    const int* n_waves_dev;   // device-planned parts: the wave count on the device
    const LaneWave* waves;
    float2* carry;            // block-to-block column carry {T, Y} per row and lane
    const uint32_t* rows;
    const uint32_t* hapw;
    const float* lut;
    float* raw_out;
    uint8_t* rescue_flag;
    int* rescue_list;
    int* rescue_rh;           // as DiagArgs::rescue_rh
    int* rescue_count;
    double* raw64_zero;       // as DiagArgs::raw64_zero
    // Rescue inside the fp32 pass (column-segmented waves): a wave with at most
    // two rescued pairs of H <= kInWaveRescueMaxH recomputes them in fp64 itself
    // (all 64 lanes on one pair) while the rest of the pass runs, instead of
    // appending them to rescue_list; at most inker_limit per run (counter
    // inker_count, null = off).
    const double* lut64;
    int* inker_count;
    int inker_limit;
    // Diagnostics (HC_PHMM_TIMELINE=1, seg waves only): per wave
    // {start, end} of s_memrealtime (100 MHz) and the HW_ID register; null = off.
    unsigned long long* timeline;
    // Column-segmented waves: per-slot result records instead of the per-pair
    // outputs (null: write raw_out / rescue_flag / raw64_zero by pair id). A
    // wave's pairs own consecutive slots, so its stores are contiguous; the
    // fp64 pass gathers the records into the per-pair outputs (Seg64Args).
    uint4* rec;
    int prio;   // 1: issue priority by remaining steps (seg_common.hpp set_prio_by_remaining)
    const PairDesc* sdesc;   // seg slots' pair descriptors in slot order (pairs[order[slot]])
    // No fp64 launch after this pass (run.cpp: small parts of seg waves only,
    // every hap within kInWaveRescueMaxH): each flagged pair is rescued in its
    // own wave, however many the wave has, and workgroup 0 zeroes the other
    // run parity's counters, which the fp64 launch zeroes otherwise. null = an
    // fp64 launch follows.
    int* solo_counters;   // the part's counter block
    int solo_other;       // the other run parity
};
// Result record of one seg slot: {raw f32 bits, state, raw f64 low word, high
// word}; state 0 = not rescued, 1 = rescued in the fp32 pass (raw f64 here),
// 2 = rescued by the fp64 pass (raw f64 written there, by pair id).
constexpr unsigned kRecPlain = 0, kRecInWave = 1, kRecListed = 2;

constexpr int kInWaveRescueMaxH = 512;   // one pair over 64 lanes of 8 columns
// Variants of the one-lane kernel (lane_kernel.hip kVariants): pairs per lane
// P (1), register block width in columns, and the waves per SIMD the register
// allocation targets. Variant 0 is the default.
struct LaneVariant {
    int P, BC, occ;
};
const LaneVariant& lane_variant(int id);
hipError_t launch_lane_f32(int variant, const LaneArgs& a, hipStream_t s);
// Column-segmented waves only (lane_kernel.hip run_seg): a pair of hap length H
// takes ceil(H / BC) lanes; BC per wave, one of the compiled block widths.
hipError_t launch_lane_seg_f32(const LaneArgs& a, hipStream_t s);
bool seg_width_ok(int bc);
int seg_width_ceil(int bc);   // narrowest compiled width >= bc (-1: none)
constexpr int kSegMaxBC = 64;
constexpr int kSegMinBC = 8;    // narrowest compiled fp32 block width

hipError_t launch_rescue_seg64(const Seg64Args& a, int grid, hipStream_t s);
// initNative(use_double = true) (intel_pairhmm.hpp:71,81,135): result_float is
// 0 for every pair, so every pair takes the fp64 path. The fp32 pass is
// replaced by this fill: raw_f32 = 0, rescued = 1 and the rescue list = all n
// pairs (pair ids 0 .. n-1), *count = n.
hipError_t launch_all_f64_list(int n, float* raw32, uint8_t* flag, int* list, int* count, const PairDesc* pairs,
                               int* list_rh, hipStream_t s);

// Launchers (kernels.hip). W = lanes per pair: 16, 32 or 64.
hipError_t launch_diag_f32(int W, const DiagArgs& a, int grid, hipStream_t s);
hipError_t launch_diag_f64(int W, const DiagArgs& a, int grid, hipStream_t s);
size_t diag_lds_bytes(int W, int ring_len, bool f64);
// The anti-diagonal kernel keeps a wave's stripe hand-off ring (H + 2W + 16
// entries per pair) in LDS up to this size, in global memory beyond (haps
// longer than ~9.9k bases in fp32, ~4.9k in fp64 at W = 64), with at most
// kDiagRingBlocks workgroups, each looping over its share of the pairs.
constexpr size_t kDiagLdsMax = size_t(152) * 1024;
constexpr int kDiagRingBlocks = 1024;
constexpr int kWideRing64Blocks = 64;   // the fp64 wide-hap rescue pass's global ring (planner.cpp)
inline bool diag_ring_in_lds(int W, int ring_len, bool f64) { return diag_lds_bytes(W, ring_len, f64) <= kDiagLdsMax; }
hipError_t configure_kernels();   // raise the dynamic-LDS limit once

// Device packing of a staged part (pack_kernels.hip), one launch. Reads:
// `quals` one byte per row, `bases` the ConvertChar codes two per byte (row k
// of read r: quality byte rdesc[r].x + k, code nibble rdesc[r].x + k, low
// nibble first; each read's start a multiple of 4); rdesc {row offset,
// length, constant gap triple i | d << 7 | c << 14 or -1, offset (a multiple
// of 4) into the i/d/c planes `gaps` (3 planes of gap_stride bytes) when the
// read's gap qualities vary}. Haps: codes two per byte, hdesc {byte offset (a
// multiple of 4), H, table word offset, 0}; tables as hap_table_words. Bytes
// past a read's or hap's end up to its alignment are read and ignored.
struct PackArgs {
    const uint8_t *bases, *quals, *gaps;
    long long gap_stride;
    const int4* rdesc;
    int nreads;
    uint32_t* rows;
    const uint8_t* hap_bytes;
    const int4* hdesc;
    int nhaps;
    uint32_t* hapw;
    // Host-planned parts: the seg slots' pair descriptors in slot order
    // (sdesc[s] = pairs[order[s]], s < nslots), so a seg wave reads its pairs
    // without the order indirection (one dependent load fewer per wave).
    const int4* pairs;
    const int* order;
    int nslots;
    int4* sdesc;
};
hipError_t launch_pack_batch(const PackArgs& a, hipStream_t s);
// Pair descriptors of a structured (cross-product) plan, built on the device
// instead of uploaded: block b's pairs [p0, p0 + nr * nh) are its reads
// [r0, r0 + nr) x haps [h0, h0 + nh) (part-local ids), read-major; blocks in
// ascending p0. pairs[k] = {rows offset, R, table offset, H} from the read and
// hap descriptors (rdesc .x/.y, hdesc .z/.y).
struct GridBlock {
    long long p0;
    int nr, nh, r0, h0;
};
// Slot order and segmented waves of a structured plan, built on the device
// from its segments (engine.cpp plan_grid): segment g holds the pairs of block
// reads rord[r0 .. r0 + nr) (by R descending) x haps hord[g0 .. g0 + G),
// read-major, in slots [slot0, slot0 + nr * G) and waves [w0, ...) of
// floor(64 / nb) pairs at block width bc. Segments in ascending slot0 / w0.
struct GridSeg {
    long long slot0, p0;   // first slot; the block's first pair
    int w0, r0, nr, nh, h0, g0, G, bc, nb, pad;
};
// A structured part's preparation in one launch: the run counters zeroed,
// the packing of launch_pack_batch, its pair descriptors (GridBlock) and its
// slot order and waves (GridSeg).
struct GridPrepArgs {
    PackArgs pack;
    const GridBlock* blocks;
    int nblocks;
    long long npairs;
    PairDesc* pairs;
    const GridSeg* segs;
    int nsegs;
    long long nslots;
    int nwaves;
    const int *rord, *hord;
    int* order;
    int* slot_of;    // pair -> its slot (inverse of order)
    int4* sdesc;     // the slots' pair descriptors, slot order
    LaneWave* waves;
    int* counters;   // kNumCounters ints zeroed (run counters)
};
hipError_t launch_prepare_grid(const GridPrepArgs& a, hipStream_t s);

// Flat batches planned on the device (flat_plan.cpp, pack_kernels.hip): the
// host uploads one record per pair — its base qualities, its base codes as
// nibbles, its gap planes only when they vary, its hap codes as nibbles, each
// field 4-byte aligned — and a descriptor; the device packs rows (4 per
// lane) and hap tables (8 columns per lane), picks each pair's
// column-segmented shape (the host planner's cost model, from per-length
// candidate tables), sorts the pairs by (block width, lanes, R) with a
// counting sort and cuts the sorted runs into waves of floor(64 / nb) pairs.
struct FlatDesc {
    long long rec;   // byte offset of the pair's record in the upload image (4-aligned)
    int row_off;     // first packed row of the read (a multiple of 4)
    int R, H;
    int hapw_off;    // first word of the hap's match table
    int gapw;        // constant gap qualities i | d << 7 | c << 14, or -1 (planes in the record)
    int fmt;         // record format: kFmt* bits, the read's quality base in bits 8-14
};
// Compact record fields (flat_plan.cpp): a read with no 'N' whose qualities
// (& 127) span less than 64 sends one byte per base, (q - qbase) << 2 | code
// (codes A0 C1 T2 G3, every other byte 0 as ConvertChar), instead of its
// quality byte and code nibble; a hap with no 'N' sends its codes 2 bits each
// (base k in bits 2(k % 4) of byte k / 4) instead of nibbles. The S2 batch
// uploads ~250 instead of ~416 bytes per pair.
constexpr int kFmtRead1B = 1;
constexpr int kFmtHap2b = 2;
struct FlatPlanArgs {
    const uint8_t* img;
    const FlatDesc* desc;
    int n;
    uint32_t* rows;
    uint32_t* hapw;
    PairDesc* pairs;
    const int2* ctab;      // [H]: the two candidates, bc | nb << 8 | group << 16
    const float* waste;    // [65]: lane-waste weight of nb lanes
    int rmax, rshift, rspan;   // bin = group * rspan + ((rmax - R) >> rshift)
    int* bin_of;           // per pair
    int* hist;             // nbins counters (zeroed by the launcher), then slot cursors
    int nbins;
    const int2* groups;    // per group: {bc, nb}, widest block first
    int ngroups;
    int* gtab;             // per group: {first slot, pairs, first wave}
    int* order;            // slot -> pair
    int* slot_of;          // pair -> slot
    int4* sdesc;           // slot -> pair descriptor
    LaneWave* waves;       // the plan's waves (packing order), then the dispatch order
    LaneWave* waves_tmp;   // max_waves entries: the packing order while the tail is reordered
    int* wcost;            // max_waves entries: each wave's modelled cost (with the tail)
    int max_waves;         // waves the launch covers (upper bound of the plan's)
    int* nwaves;           // the plan's wave count; [1]: its largest modelled wave cost (with the tail)
    int tail;              // waves dispatched last, longest first (0: packing order)
    int* counters;         // kNumCounters run counters, zeroed
    int prep_blocks;       // flat_prep_kernel's grid bound (0: a wave per pair, up to 65 536 blocks)
};
hipError_t launch_flat_plan(const FlatPlanArgs& a, hipStream_t s);
// bytes (a multiple of 16, both 16-byte aligned) from device memory to mapped
// pinned host memory, stored by a kernel (no DMA engine).
hipError_t launch_store_to_host(void* host, const void* dev, size_t bytes, hipStream_t s);

}  // namespace hcphmm
