// Driver around the REFERENCE Smith-Waterman aligner — TEST INFRASTRUCTURE ONLY.
//
// Compiled by oracle/Makefile against the reference headers where they lie
// (/root/reference/src/haplotypecaller/smithwaterman/native/avx2-smithwaterman.h);
// no reference source is copied into this repository. The output goes to
// oracle/_ref/ (git-ignored) and is used to generate tests/golden/sw_golden.npz
// and to time the reference aligner beside the GPU in bench.py.
//
// The flags are the reference's own (-O3 -mavx -mavx2, CMakeLists.txt:5).
// IntelSWAligner::align (intel_smithwaterman.hpp:29-44) needs cigar.hpp, which
// pulls Boost (absent here), so its 10-line all-match shortcut is restated in
// ref_sw_align_batch and runSWOnePairBT_avx2 is called directly.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "avx2-smithwaterman.h"

extern "C" {

// One pair through runSWOnePairBT_avx2 (PairWiseSW.h:418-447). Returns the
// alignment offset, or INT_MIN if the CIGAR does not fit in cap.
int ref_sw_align(int match, int mismatch, int open, int extend, const uint8_t* seq1, int len1,
                 const uint8_t* seq2, int len2, int overhang, char* cigar, int cap)
{
    // The reference sizes its buffer 2*max(len) (intel_smithwaterman.hpp:42);
    // give the sprintf loop room so no test input can overrun it.
    std::vector<char> buf(size_t(4) * size_t(len1 + len2) + 64, 0);
    int16_t count = 0;
    const int off = runSWOnePairBT_avx2(match, mismatch, open, extend, const_cast<uint8_t*>(seq1),
                                        const_cast<uint8_t*>(seq2), len1, len2, int8_t(overhang), buf.data(),
                                        &count);
    const size_t n = std::strlen(buf.data());
    if (n + 1 > size_t(cap)) return INT_MIN;
    std::memcpy(cigar, buf.data(), n + 1);
    return off;
}

// IntelSWAligner::align over many pairs: the all-match shortcut
// (intel_smithwaterman.hpp:36-37,47-58) when shortcut != 0, then
// runSWOnePairBT_avx2. Single-threaded, as the reference calls it.
int ref_sw_align_batch(long n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
                       const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts, int match,
                       int mismatch, int open, int extend, int overhang, int shortcut, int32_t* offsets,
                       char* cigars, int stride)
{
    int bad = 0;
    for (long k = 0; k < n; ++k) {
        const uint8_t* r = refs + ref_off[k];
        const uint8_t* a = alts + alt_off[k];
        char* out = cigars + size_t(k) * size_t(stride);
        if (shortcut && ref_len[k] == alt_len[k]) {
            int mm = 0;
            for (int i = 0; mm <= 2 && i < ref_len[k]; ++i) mm += r[i] != a[i];
            if (mm <= 2) {
                offsets[k] = 0;
                bad |= std::snprintf(out, size_t(stride), "%dM", ref_len[k]) >= stride;
                continue;
            }
        }
        offsets[k] = ref_sw_align(match, mismatch, open, extend, r, ref_len[k], a, alt_len[k], overhang, out,
                                  stride);
        bad |= offsets[k] == INT_MIN;
    }
    return bad ? -1 : 0;
}

}  // extern "C"
