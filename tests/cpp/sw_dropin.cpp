// C++ drop-in check for include/hc_sw.hpp: the loop of
// assembler/graph_wrapper.hpp:232-240 compiled against hc::MI355XSWAligner with
// Haplotype / Cigar stand-ins (the reference's Cigar is assignable from the
// CIGAR text, sam/cigar.hpp:77-83). Input: <n_regions> then per region the ref
// and its haps (length-prefixed). Output per hap: offset and CIGAR from the
// per-hap loop, then from align_haplotypes(), one line each.
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "hc_sw.hpp"

struct Cigar {   // stand-in: only the assignment the call site uses
    std::string text;
    Cigar& operator=(const std::string& s) { text = s; return *this; }
};
struct Haplotype {
    std::string bases;
    std::size_t alignment_begin_wrt_ref = 0;
    Cigar cigar;
};

static std::string get(std::ifstream& in)
{
    int32_t n = 0;
    in.read(reinterpret_cast<char*>(&n), 4);
    std::string s(static_cast<size_t>(n), 0);
    in.read(s.data(), n);
    return s;
}

int main(int argc, char** argv)
{
    if (argc != 3) return 2;
    std::ifstream in(argv[1], std::ios::binary);
    std::FILE* out = std::fopen(argv[2], "w");
    int32_t nreg = 0, nh = 0;
    in.read(reinterpret_cast<char*>(&nreg), 4);
    hc::MI355XSWAligner aligner;
    for (int r = 0; r < nreg; ++r) {
        const std::string ref = get(in);
        in.read(reinterpret_cast<char*>(&nh), 4);
        std::vector<Haplotype> haplotypes(static_cast<size_t>(nh)), batch;
        for (auto& h : haplotypes) h.bases = get(in);
        batch = haplotypes;
        for (auto& h : haplotypes) {   // graph_wrapper.hpp:233-239, unchanged
            auto [alignment_begin, cigar] = aligner.align(ref, h.bases);
            h.alignment_begin_wrt_ref = alignment_begin;
            h.cigar = std::move(cigar);
        }
        aligner.align_haplotypes(ref, batch);
        for (size_t k = 0; k < haplotypes.size(); ++k)
            std::fprintf(out, "%zu %s %zu %s\n", haplotypes[k].alignment_begin_wrt_ref,
                         haplotypes[k].cigar.text.c_str(), batch[k].alignment_begin_wrt_ref,
                         batch[k].cigar.text.c_str());
    }
    std::fclose(out);
    return 0;
}
