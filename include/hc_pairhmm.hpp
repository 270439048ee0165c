// hc_pairhmm.hpp — C++ drop-in for the reference's IntelPairHMM.
//
// The HaplotypeCaller driver calls (src/haplotypecaller/haplotypecaller.hpp:90,103)
//
//     IntelPairHMM pairhmm;
//     auto likelihoods = pairhmm.compute_likelihoods(haplotypes, reads);
//
// Replacing `IntelPairHMM` with `hc::MI355XPairHMM` keeps that call site as is:
// same signature (pairhmm/intel_pairhmm.hpp:48-56), same result (read-major
// vector<vector<double>> of log10 likelihoods, capped at best - 4.5), same
// side effect (poorly modelled reads are erased from `reads`, :24-46). The
// work runs in libhcpairhmm.so through the C ABI of hc_pairhmm.h.
//
// Header-only; templated on the caller's Haplotype (needs `.bases`) and
// SAMRecord (needs `.SEQ`, `.QUAL`, `.insertionGOP()`, `.deletionGOP()`,
// `.overallGCP()`) so it does not depend on the reference's headers.
// Reads longer than the reference's 200-byte GOP/GCP strings (sam.hpp:30-32,
// undefined behaviour there) get 'I' (73) / '+' (43) for every base.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "hc_pairhmm.h"

namespace hc {

class MI355XPairHMM {
public:
    // use_double: initNative(use_double) (intel_pairhmm.hpp:71,81): every pair
    // in fp64 only. Per instance, as the reference's g_use_double: each call
    // passes it (hc_phmm_compute_likelihoods_ex), so instances with different
    // modes in different threads do not interfere.
    explicit MI355XPairHMM(int device = -1, bool use_double = false) : device_(device), use_double_(use_double) {}

    template <class HaplotypeT, class SAMRecordT>
    std::vector<std::vector<double>> compute_likelihoods(const std::vector<HaplotypeT>& haplotypes,
                                                         std::vector<SAMRecordT>& reads)
    {
        check(hc_phmm_init(HC_PHMM_FLAG_KEEP_MODE, device_));   // device only: the mode goes with the call
        const int nr = static_cast<int>(reads.size()), nh = static_cast<int>(haplotypes.size());
        std::vector<std::string> gaps;   // owned i/d/c strings where the record's are short
        gaps.reserve(3 * reads.size());
        std::vector<hc_phmm_read> rv(reads.size());
        for (int r = 0; r < nr; ++r) {
            const auto& rec = reads[r];
            const size_t n = rec.SEQ.size();
            auto pick = [&](auto view, char fill) -> const char* {
                if (view.size() >= n) return view.data();
                gaps.emplace_back(n, fill);
                return gaps.back().data();
            };
            rv[r].length = static_cast<int32_t>(n);
            rv[r].bases = rec.SEQ.data();
            rv[r].q = rec.QUAL.data();
            rv[r].i = pick(rec.insertionGOP(), 'I');
            rv[r].d = pick(rec.deletionGOP(), 'I');
            rv[r].c = pick(rec.overallGCP(), '+');
        }
        std::vector<hc_phmm_hap> hv(haplotypes.size());
        for (int h = 0; h < nh; ++h) {
            hv[h].length = static_cast<int32_t>(haplotypes[h].bases.size());
            hv[h].bases = haplotypes[h].bases.data();
        }
        std::vector<double> flat(static_cast<size_t>(nr) * nh);
        std::vector<uint8_t> keep(reads.size());
        int32_t kept = 0;
        check(hc_phmm_compute_likelihoods_ex(rv.data(), nr, hv.data(), nh, flat.data(), keep.data(), &kept,
                                             use_double_ ? HC_PHMM_FLAG_F64 : 0u));
        std::vector<std::vector<double>> out;
        out.reserve(kept);
        std::vector<SAMRecordT> survivors;
        survivors.reserve(kept);
        for (int r = 0; r < nr; ++r) {
            if (!keep[r]) continue;
            out.emplace_back(flat.begin() + static_cast<size_t>(r) * nh,
                             flat.begin() + static_cast<size_t>(r + 1) * nh);
            survivors.push_back(std::move(reads[r]));
        }
        reads.swap(survivors);
        return out;
    }

private:
    static void check(int rc)
    {
        if (rc != HC_PHMM_OK)
            throw std::runtime_error(std::string("hc_pairhmm: ") + hc_phmm_last_error());
    }
    int device_;
    bool use_double_;
};

}  // namespace hc
