// Drop-in check for include/hc_pairhmm.hpp: reads one region (reads x haps)
// from a binary file, runs hc::MI355XPairHMM::compute_likelihoods with
// SAMRecord/Haplotype stand-ins shaped like the reference's
// (src/haplotypecaller/sam/sam.hpp:17-82, haplotype/haplotype.hpp:15-52),
// and also the reference's own accelerator slot shacc_pairhmm::calculate
// (pairhmm/native/shacc_pairhmm.h:35). Writes the results for the test to
// compare with the oracle.
//
// in:  int32 nR, nH; per read: int32 len, bases, quals; per hap: int32 len, bases
// out: int32 n_kept; uint8 keep_mask[nR] (1 = kept); double L[n_kept][nH];
//      float shacc[nR][nH]
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <string>
#include <string_view>
#include <vector>

#include "hc_pairhmm.hpp"

struct SAMRecord {
    std::string QNAME, SEQ, QUAL;
    static inline const std::string GOP = std::string(200, 'I');   // sam.hpp:30-32
    static inline const std::string GCP = std::string(200, '+');
    auto insertionGOP() const { return std::string_view{GOP}.substr(0, SEQ.size()); }
    auto deletionGOP() const { return std::string_view{GOP}.substr(0, SEQ.size()); }
    auto overallGCP() const { return std::string_view{GCP}.substr(0, SEQ.size()); }
    auto size() const { return SEQ.size(); }
};
struct Haplotype {
    std::string bases;
};

namespace shacc_pairhmm {
struct Read { int length; const char *bases, *q, *i, *d, *c; };
struct Haplotype { int length; const char* bases; };
struct Batch { int num_reads; int num_haps; long num_cells; Read* reads; Haplotype* haps; float* results; };
bool calculate(Batch& batch);
}

static std::string rd(std::ifstream& f)
{
    int32_t n = 0;
    f.read(reinterpret_cast<char*>(&n), 4);
    std::string s(n, '\0');
    f.read(s.data(), n);
    return s;
}

int main(int argc, char** argv)
{
    if (argc != 3) return 2;
    std::ifstream in(argv[1], std::ios::binary);
    int32_t nR = 0, nH = 0;
    in.read(reinterpret_cast<char*>(&nR), 4);
    in.read(reinterpret_cast<char*>(&nH), 4);
    std::vector<SAMRecord> reads(nR);
    for (auto& r : reads) {
        r.SEQ = rd(in);
        r.QUAL = rd(in);
        r.QNAME = std::to_string(&r - reads.data());
    }
    std::vector<Haplotype> haps(nH);
    for (auto& h : haps) h.bases = rd(in);

    // The reference's own slot, before compute_likelihoods erases reads.
    std::vector<shacc_pairhmm::Read> sr(nR);
    std::vector<std::string> gop(nR), gcp(nR);
    for (int r = 0; r < nR; ++r) {
        gop[r] = std::string(reads[r].SEQ.size(), 'I');
        gcp[r] = std::string(reads[r].SEQ.size(), '+');
        sr[r] = {int(reads[r].SEQ.size()), reads[r].SEQ.data(), reads[r].QUAL.data(), gop[r].data(),
                 gop[r].data(), gcp[r].data()};
    }
    std::vector<shacc_pairhmm::Haplotype> sh(nH);
    for (int h = 0; h < nH; ++h) sh[h] = {int(haps[h].bases.size()), haps[h].bases.data()};
    std::vector<float> sres(size_t(nR) * nH);
    shacc_pairhmm::Batch batch{nR, nH, 0, sr.data(), sh.data(), sres.data()};
    if (!shacc_pairhmm::calculate(batch)) return 3;

    hc::MI355XPairHMM phmm(0);
    auto L = phmm.compute_likelihoods(haps, reads);   // haplotypecaller.hpp:103
    std::ofstream out(argv[2], std::ios::binary);
    const int32_t kept = int32_t(L.size());
    out.write(reinterpret_cast<const char*>(&kept), 4);
    std::vector<uint8_t> mask(nR, 0);
    for (const auto& r : reads) mask[std::stoi(r.QNAME)] = 1;
    out.write(reinterpret_cast<const char*>(mask.data()), nR);
    for (const auto& row : L) out.write(reinterpret_cast<const char*>(row.data()), sizeof(double) * nH);
    out.write(reinterpret_cast<const char*>(sres.data()), sizeof(float) * sres.size());
    return 0;
}
