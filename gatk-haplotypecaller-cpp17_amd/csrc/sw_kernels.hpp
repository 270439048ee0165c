// Smith-Waterman device layout shared by sw_kernels.hip and sw_engine.cpp.
//
// Reference: src/haplotypecaller/smithwaterman/native/PairWiseSW.h
// (smithWatermanBackTrack :41-238, getCIGAR :240-415). seq1 (ref window) is the
// row axis, seq2 (haplotype) the column axis, as there.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace hcsw {

constexpr int kLow = -1073741824;        // LOW_INIT_VALUE = INT32_MIN/2 (smithwaterman_common.h:51)
constexpr int kMinCutoff = -100000000;   // MATRIX_MIN_CUTOFF (:50)
constexpr int kStripe = 64;              // rows per stripe = lanes per wave
constexpr int kGroup = 8;                // steps per 32-bit backtrack word (4 bits per cell)

// Steps one stripe takes over n2 columns: n2 + 63 (the one-row skew) plus one
// (lane 63 hands column n2 on the step after it computed it), rounded up to
// whole backtrack words.
__host__ __device__ inline int stripe_steps(int n2) { return (n2 + kStripe + kGroup - 1) & ~(kGroup - 1); }
// Backtrack words of one pair: per stripe, one word per lane per 8 steps.
__host__ __device__ inline int64_t bt_words(int n1, int n2)
{
    return int64_t((n1 + kStripe - 1) / kStripe) * (stripe_steps(n2) / kGroup) * kStripe;
}
// LDS row buffer entries (H or F): slot 63 + j holds column j; lanes still in
// the skew write up to 64 slots before column 1 and up to 72 after column n2,
// and lane 0 reads one group ahead. (A multiple of 4 entries, so that 16-byte
// reads of the buffers stay aligned.)
__host__ __device__ inline int row_slots(int n2max) { return (n2max + 2 * kStripe + 4 * kGroup + 3) & ~3; }
// rowF doubles as the last-column buffer (n1 + 1 entries) after the DP.
__host__ __device__ inline int fslots(int n1max, int n2max)
{
    return row_slots(n2max) > n1max + 1 ? row_slots(n2max) : ((n1max + 4) & ~3);
}
// Haplotype bases (bytes): 64 leading pads (lanes still in the skew), then the
// columns, then pads up to the last step of a stripe.
__host__ __device__ inline int alt_slots(int n2max) { return (kStripe + n2max + kStripe + 2 * kGroup + 3) & ~3; }

struct SwPair {
    int64_t ref_off;   // seq1 bytes in refs[]
    int64_t alt_off;   // seq2 bytes in alts[]
    int64_t bt_off;    // first backtrack word in bt[]
    int64_t el_off;    // first CIGAR element in elems[] (capacity n1 + n2 + 3)
    int32_t n1, n2;
};

// DP result of one pair: best end point (PairWiseSW.h:201-233).
struct SwResult {
    int32_t score;
    int32_t max_i, max_j;
    int32_t shortcut;   // 1: all-match shortcut taken (intel_smithwaterman.hpp:36-37)
};

struct SwDpArgs {
    const SwPair* pairs;
    const int32_t* order;   // wave -> pair id (longest first)
    int n;
    const uint8_t* refs;
    const uint8_t* alts;
    uint32_t* bt;
    SwResult* res;
    uint32_t* elems;   // per-pair scratch (n1 + n2 + 3 words): last-column H during the DP
    int match, mismatch, open, extend;
    int overhang;
    int shortcut;
    int n1max, n2max;   // size the dynamic LDS
    int fast;    // host-proven: no cutoff, no int32 overflow (sw_engine.cpp fast_ok)
    int wpg;       // pairs (waves) per workgroup: 1, 2 or 4
    int lds_wave_bytes;   // set by launch_dp
};

struct SwTraceArgs {
    const SwPair* pairs;
    const SwResult* res;
    const uint32_t* bt;
    int n;
    int overhang;
    uint32_t* elems;     // per-pair scratch: (len << 4) | op, traceback order (CIGAR end first)
    uint16_t* slots;     // the first kSlotElems elements of pair p as uint16 at p * kSlotElems
    int32_t* n_elems;
    int32_t* offsets;
};

// Fixed per-pair result slots: CIGAR elements fit 16 bits (len <= n1 + n2 < 2^11,
// op < 16); pairs with more elements are read back from their scratch.
constexpr int kSlotElems = 32;

// CIGAR element op codes (smithwaterman_common.h:21-26).
constexpr int kOpM = 0, kOpI = 1, kOpD = 2, kOpS = 9;

size_t dp_lds_bytes(int n1max, int n2max);
hipError_t launch_dp(const SwDpArgs& a, int n1max, hipStream_t s);
hipError_t launch_trace(const SwTraceArgs& a, hipStream_t s);

}  // namespace hcsw
