// hc_sw.hpp — C++ drop-in for the reference's IntelSWAligner.
//
// The assembler aligns every candidate haplotype of a region against the
// region's reference window (src/haplotypecaller/assembler/graph_wrapper.hpp:232-240):
//
//     IntelSWAligner aligner;
//     for (auto& h : haplotypes) {
//         auto [alignment_begin, cigar] = aligner.align(ref, h.bases);
//         h.alignment_begin_wrt_ref = alignment_begin;
//         h.cigar = std::move(cigar);
//     }
//
// `hc::MI355XSWAligner` keeps that loop compiling unchanged (align() has the
// signature of intel_smithwaterman.hpp:29-44 and returns the CIGAR as the text
// the reference's Cigar is built from, `Cigar(const std::string&)`), and
// align_haplotypes() replaces the whole loop with one device pass. Results are
// the reference's: all-match shortcut, then the SOFTCLIP Smith-Waterman with
// its tie-breaks. Header-only over the C ABI of hc_sw.h; no reference headers.
#pragma once

#include <algorithm>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "hc_pairhmm.h"
#include "hc_sw.h"

namespace hc {

class MI355XSWAligner {
public:
    struct SWParameters {
        int w_match;
        int w_mismatch;
        int w_open;
        int w_extend;
    };
    // intel_smithwaterman.hpp:21-24
    static constexpr SWParameters ORIGINAL_DEFAULT{3, -1, -4, -3};
    static constexpr SWParameters STANDARD_NGS{25, -50, -110, -6};
    static constexpr SWParameters NEW_SW_PARAMETERS{200, -150, -260, -11};
    static constexpr SWParameters ALIGNMENT_TO_BEST_HAPLOTYPE_SW_PARAMETERS{10, -15, -30, -5};
    static constexpr std::size_t MINIMAL_MISMATCH_TO_TOLERANCE = 2;

    explicit MI355XSWAligner(int device = -1) : device_(device) {}

    // IntelSWAligner::align: (offset, CIGAR text).
    std::pair<std::size_t, std::string> align(std::string_view ref, std::string_view alt,
                                              const SWParameters& params = NEW_SW_PARAMETERS)
    {
        if (ref.empty() || alt.empty())
            throw std::invalid_argument("Non-null sequences are required for the SW aligner");
        auto r = align_many(ref, std::vector<std::string_view>{alt}, params);
        return std::move(r[0]);
    }

    // Every alt against one reference window, one device pass.
    std::vector<std::pair<std::size_t, std::string>> align_many(std::string_view ref,
                                                                const std::vector<std::string_view>& alts,
                                                                const SWParameters& params = NEW_SW_PARAMETERS)
    {
        if (ref.empty()) throw std::invalid_argument("Non-null sequences are required for the SW aligner");
        const int64_t n = static_cast<int64_t>(alts.size());
        std::vector<std::pair<std::size_t, std::string>> out;
        if (n == 0) return out;
        std::vector<int64_t> ref_off(alts.size(), 0), alt_off(alts.size());
        std::vector<int32_t> ref_len(alts.size(), static_cast<int32_t>(ref.size())), alt_len(alts.size());
        std::string pool;
        for (size_t k = 0; k < alts.size(); ++k) {
            if (alts[k].empty()) throw std::invalid_argument("Non-null sequences are required for the SW aligner");
            alt_off[k] = static_cast<int64_t>(pool.size());
            alt_len[k] = static_cast<int32_t>(alts[k].size());
            pool.append(alts[k]);
        }
        size_t longest = 0;
        for (auto a : alts) longest = std::max(longest, a.size());
        const int32_t stride = static_cast<int32_t>(4 * (ref.size() + longest) + 16);
        std::vector<int32_t> offsets(alts.size());
        std::vector<char> cigars(alts.size() * static_cast<size_t>(stride));
        check(hc_sw_init(device_));
        const hc_sw_params p{params.w_match, params.w_mismatch, params.w_open, params.w_extend};
        check(hc_sw_align_flat(n, ref_off.data(), ref_len.data(), reinterpret_cast<const uint8_t*>(ref.data()),
                               alt_off.data(), alt_len.data(), reinterpret_cast<const uint8_t*>(pool.data()), p,
                               HC_SW_SOFTCLIP, 1, offsets.data(), cigars.data(), stride));
        out.reserve(alts.size());
        for (size_t k = 0; k < alts.size(); ++k)
            out.emplace_back(static_cast<std::size_t>(offsets[k]), std::string(cigars.data() + k * stride));
        return out;
    }

    // The loop of graph_wrapper.hpp:232-240 in one pass: sets
    // h.alignment_begin_wrt_ref and h.cigar (assigned from the CIGAR text) of
    // every haplotype.
    template <class HaplotypeT>
    void align_haplotypes(std::string_view ref, std::vector<HaplotypeT>& haplotypes,
                          const SWParameters& params = NEW_SW_PARAMETERS)
    {
        std::vector<std::string_view> alts;
        alts.reserve(haplotypes.size());
        for (const auto& h : haplotypes) alts.emplace_back(h.bases);
        auto r = align_many(ref, alts, params);
        for (size_t k = 0; k < haplotypes.size(); ++k) {
            haplotypes[k].alignment_begin_wrt_ref = r[k].first;
            haplotypes[k].cigar = std::move(r[k].second);
        }
    }

private:
    static void check(int rc)
    {
        if (rc != HC_SW_OK) throw std::runtime_error(std::string("hc_sw: ") + hc_phmm_last_error());
    }
    int device_;
};

}  // namespace hc
