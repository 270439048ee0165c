// Region-pipeline parity harness (the reachable part):
// seeded synthetic active regions go through the three drop-ins in the order of
// HaplotypeCaller::call_region (src/haplotypecaller/haplotypecaller.hpp:83-107)
//
//   haplotypes vs the padded reference window  hc::MI355XSWAligner      (assembler, graph_wrapper.hpp:232-240)
//   reads x haplotypes, normalise + erase reads hc::MI355XPairHMM        (haplotypecaller.hpp:103)
//   per variant site: marginalise, genotype     hc_gt_genotype_sites     (genotyper.hpp:369-398)
//
// and through the same chain built on the reference's own kernels compiled
// from /root/reference (oracle/_ref: the AVX2 aligner with the all-match
// shortcut, the AVX PairHMM kernels with the rescue loop of
// intel_pairhmm.hpp:128-147, MathUtils::approximate_log10_sum_log10) plus the
// oracle's restated normalise/filter and genotyper loops. Everything the two
// chains produce is compared bit for bit: offsets and CIGARs, kept reads,
// likelihood matrices, per-site genotype likelihoods, genotype and quality.
//
// The event bookkeeping between the kernels (CIGAR -> events -> alleles ->
// haplotype/read maps) is the harness's own, shared by both chains: the
// reference's genotyper.hpp needs Boost (sam.hpp) and cannot be built here.
// VCF parity with the reference binary stays unpinned (Boost and chrM absent).
//
// usage: region_pipeline <n_regions> <seed> <out.json>
#include <algorithm>
#include <cinttypes>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <string_view>
#include <tuple>
#include <vector>

#include "hc_gt.h"
#include "hc_pairhmm.hpp"
#include "hc_sw.hpp"

extern "C" {
// oracle/_ref (reference sources compiled in place) and oracle/liboracle.so
int ref_sw_align_batch(long n, const int64_t* ref_off, const int32_t* ref_len, const uint8_t* refs,
                       const int64_t* alt_off, const int32_t* alt_len, const uint8_t* alts, int match, int mismatch,
                       int open, int extend, int overhang, int shortcut, int32_t* offsets, char* cigars, int stride);
long ref_pairs(long n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off, const int32_t* H,
               const uint8_t* rs, const uint8_t* q, const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
               const uint8_t* hap, float* raw_f32, double* raw_f64, uint8_t* rescued, double* loglik, int nthreads);
double ref_approx_log10_sum_log10(double a, double b);
int hco_normalize(int nReads, int nHaps, const int32_t* read_len, double* L, uint8_t* keep);
void hco_gt_site_with(const double* L, int n_haps, const int32_t* keep, int n_keep, const int32_t* hap_allele,
                      int n_alleles, double* gl, int32_t* gt_index, int32_t* gq, double (*approx)(double, double));
}

namespace {

constexpr int kRegion = 245, kPad = 85;              // HaplotypeCaller::do_work defaults (:111-112)
constexpr int kWindow = kRegion + 2 * kPad;
constexpr int kAlleleExtension = 2;                  // Genetyper::ALLELE_EXTENSION

// Stand-ins shaped like the reference's SAMRecord / Haplotype (sam.hpp:17-82,
// haplotype.hpp:15-52): what the drop-ins read from them.
struct SAMRecord {
    std::string SEQ, QUAL;
    int begin = 0, end = 0;   // interval on the padded window
    int id = 0;
    static inline const std::string GOP = std::string(256, 'I');   // sam.hpp:30-32
    static inline const std::string GCP = std::string(256, '+');
    std::string_view insertionGOP() const { return std::string_view{GOP}.substr(0, SEQ.size()); }
    std::string_view deletionGOP() const { return std::string_view{GOP}.substr(0, SEQ.size()); }
    std::string_view overallGCP() const { return std::string_view{GCP}.substr(0, SEQ.size()); }
    std::size_t size() const { return SEQ.size(); }
};
struct Haplotype {
    std::string bases;
    std::size_t alignment_begin_wrt_ref = 0;
    std::string cigar;
};

struct Variant {
    int pos;    // window position of the first affected reference base
    int type;   // 0 SNP, 1 insertion after pos, 2 deletion of pos .. pos+len-1
    std::string alt;
    int len;
};

struct Region {
    std::string ref;
    std::vector<Haplotype> haps;
    std::vector<SAMRecord> reads;
};

const char kACGT[4] = {'A', 'C', 'G', 'T'};

std::string apply(const std::string& ref, const std::vector<Variant>& vs, unsigned mask)
{
    std::string h;
    int p = 0;
    for (size_t k = 0; k < vs.size(); ++k) {
        if (!(mask >> k & 1)) continue;
        const Variant& v = vs[k];
        h.append(ref, p, v.pos - p);
        if (v.type == 0) {
            h += v.alt;
            p = v.pos + 1;
        } else if (v.type == 1) {
            h += ref[v.pos];
            h += v.alt;
            p = v.pos + 1;
        } else {
            p = v.pos + v.len;
        }
    }
    h.append(ref, p, std::string::npos);
    return h;
}

// hap coordinate -> window coordinate for the variants in `mask`
int to_ref(const std::vector<Variant>& vs, unsigned mask, int hpos)
{
    int shift = 0;
    for (size_t k = 0; k < vs.size(); ++k) {
        if (!(mask >> k & 1)) continue;
        const Variant& v = vs[k];
        if (v.pos + shift >= hpos) break;
        shift += v.type == 1 ? int(v.alt.size()) : v.type == 2 ? -v.len : 0;
    }
    return std::max(0, hpos - shift);
}

Region make_region(std::mt19937_64& g)
{
    auto U = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(g); };
    Region rg;
    rg.ref.resize(kWindow);
    for (auto& c : rg.ref) c = kACGT[U(0, 3)];
    // 1-4 true variants in the origin region, well apart
    std::vector<Variant> vs;
    const int nv = U(1, 4);
    for (int t = 0; t < 200 && int(vs.size()) < nv; ++t) {
        Variant v{U(kPad + 8, kPad + kRegion - 12), 0, "", 1};
        const int r = U(0, 9);
        if (r < 6) {
            v.type = 0;
            char a;
            do a = kACGT[U(0, 3)]; while (a == rg.ref[v.pos]);
            v.alt = std::string(1, a);
        } else if (r < 8) {
            v.type = 1;
            v.len = U(1, 3);
            for (int k = 0; k < v.len; ++k) v.alt += kACGT[U(0, 3)];
        } else {
            v.type = 2;
            v.len = U(1, 3);
        }
        bool ok = true;
        for (const auto& w : vs) ok &= std::abs(w.pos - v.pos) > 8;
        if (ok) vs.push_back(v);
    }
    std::sort(vs.begin(), vs.end(), [](const Variant& a, const Variant& b) { return a.pos < b.pos; });
    // candidate haplotypes: every subset of the variants (ref first), plus an
    // assembly artefact (a private SNP) now and then
    std::vector<unsigned> masks;
    for (unsigned m = 0; m < (1u << vs.size()); ++m) masks.push_back(m);
    for (unsigned m : masks) rg.haps.push_back(Haplotype{apply(rg.ref, vs, m)});
    if (U(0, 2) == 0) {
        std::string h = rg.haps.back().bases;
        const int p = U(kPad, kPad + kRegion - 1);
        h[size_t(p)] = h[size_t(p)] == 'A' ? 'C' : 'A';
        rg.haps.push_back(Haplotype{h});
    }
    // diploid sample: two of the subsets
    const unsigned m1 = masks[size_t(U(0, int(masks.size()) - 1))], m2 = masks[size_t(U(0, int(masks.size()) - 1))];
    const std::string s1 = apply(rg.ref, vs, m1), s2 = apply(rg.ref, vs, m2);
    const int nreads = U(40, 240);
    for (int k = 0; k < nreads; ++k) {
        const bool first = U(0, 1) == 0;
        const std::string& src = first ? s1 : s2;
        const int len = std::min<int>(U(100, 151), int(src.size()));
        const int st = U(0, int(src.size()) - len);
        SAMRecord r;
        r.SEQ = src.substr(size_t(st), size_t(len));
        r.QUAL.resize(size_t(len));
        for (int i = 0; i < len; ++i) {
            r.QUAL[size_t(i)] = char(33 + U(20, 40));
            if (U(0, 299) == 0) r.SEQ[size_t(i)] = kACGT[U(0, 3)];
        }
        if (U(0, 49) == 0)   // a junk read the filter removes
            for (auto& c : r.SEQ) c = kACGT[U(0, 3)];
        r.begin = to_ref(vs, first ? m1 : m2, st);
        r.end = std::min(kWindow, r.begin + len);
        r.id = k;
        rg.reads.push_back(std::move(r));
    }
    return rg;
}

// --- shared event bookkeeping (stands in for genotyper.hpp's) --------------
struct Event {
    int pos;
    int type;   // 0 SNP, 1 insertion, 2 deletion
    std::string alt;
    int span;   // reference bases covered
    bool operator<(const Event& o) const { return std::tie(pos, type, alt, span) < std::tie(o.pos, o.type, o.alt, o.span); }
    bool operator==(const Event& o) const { return !(*this < o) && !(o < *this); }
};

std::vector<Event> events_of(const std::string& ref, const std::string& hap, size_t offset, const std::string& cigar)
{
    std::vector<Event> ev;
    int rp = int(offset), hp = 0;
    size_t i = 0;
    while (i < cigar.size()) {
        int n = 0;
        while (i < cigar.size() && cigar[i] >= '0' && cigar[i] <= '9') n = n * 10 + (cigar[i++] - '0');
        const char op = cigar[i++];
        if (op == 'M' || op == '=' || op == 'X') {
            for (int k = 0; k < n; ++k)
                if (ref[size_t(rp + k)] != hap[size_t(hp + k)]) ev.push_back({rp + k, 0, std::string(1, hap[size_t(hp + k)]), 1});
            rp += n;
            hp += n;
        } else if (op == 'I') {
            ev.push_back({rp - 1, 1, hap.substr(size_t(hp), size_t(n)), 1});
            hp += n;
        } else if (op == 'D') {
            ev.push_back({rp - 1, 2, "", n + 1});
            rp += n;
        } else if (op == 'S') {
            hp += n;
        }
    }
    return ev;
}

struct Site {
    int region;
    std::vector<int32_t> keep, hap_allele;
    int n_alleles;
};

// Sites of one region: event starts inside the origin region; alleles = the
// reference plus the distinct events starting there (<= 7); haplotype ->
// allele; reads kept when they overlap the allele span +- the extension.
std::vector<Site> sites_of(int region, const std::vector<std::vector<Event>>& hap_events,
                           const std::vector<SAMRecord>& reads)
{
    std::map<int, std::vector<Event>> at;
    for (const auto& he : hap_events)
        for (const auto& e : he)
            if (e.pos >= kPad && e.pos < kPad + kRegion) at[e.pos].push_back(e);
    std::vector<Site> out;
    for (auto& [pos, evs] : at) {
        std::sort(evs.begin(), evs.end());
        evs.erase(std::unique(evs.begin(), evs.end()), evs.end());
        if (evs.size() + 1 > HC_GT_MAX_ALLELES) continue;
        Site s{region, {}, {}, int(evs.size()) + 1};
        int span = 1;
        for (const auto& e : evs) span = std::max(span, e.span);
        for (const auto& he : hap_events) {
            int a = 0;
            for (const auto& e : he)
                if (e.pos == pos) a = 1 + int(std::lower_bound(evs.begin(), evs.end(), e) - evs.begin());
            s.hap_allele.push_back(a);
        }
        const int lo = pos - kAlleleExtension, hi = pos + span + kAlleleExtension;
        for (size_t r = 0; r < reads.size(); ++r)
            if (reads[r].begin < hi && lo < reads[r].end) s.keep.push_back(int32_t(r));
        out.push_back(std::move(s));
    }
    return out;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc != 4) return 2;
    const int nreg = std::atoi(argv[1]);
    std::mt19937_64 g(std::strtoull(argv[2], nullptr, 10));
    std::vector<Region> regions;
    for (int k = 0; k < nreg; ++k) regions.push_back(make_region(g));

    long n_haps = 0, n_reads = 0, n_kept = 0, n_sites = 0, n_called = 0, n_rescued = 0;
    long bad_sw = 0, bad_keep = 0, bad_L = 0, bad_gl = 0, bad_gt = 0;
    hc::MI355XSWAligner aligner(0);
    hc::MI355XPairHMM pairhmm(0);
    std::vector<hc_gt_site> gpu_sites;
    std::vector<Site> all_sites;
    std::vector<std::vector<double>> region_L;   // GPU matrices (kept reads), read-major
    std::vector<std::vector<double>> ref_gl;
    std::vector<int32_t> ref_gt, ref_gq;
    std::vector<int> region_nh;
    for (int k = 0; k < nreg; ++k) {
        Region& rg = regions[size_t(k)];
        const int nh = int(rg.haps.size()), nr = int(rg.reads.size());
        n_haps += nh;
        n_reads += nr;
        // --- GPU chain, call_region's order ---
        std::vector<Haplotype> haps = rg.haps;
        aligner.align_haplotypes(rg.ref, haps);              // assembler's SW loop
        std::vector<SAMRecord> reads = rg.reads;
        auto L = pairhmm.compute_likelihoods(haps, reads);    // erases poorly modelled reads
        // --- reference chain ---
        std::vector<int64_t> roff(static_cast<size_t>(nh), 0), aoff(static_cast<size_t>(nh));
        std::vector<int32_t> rlen(static_cast<size_t>(nh), kWindow), alen(static_cast<size_t>(nh));
        std::string pool;
        for (int h = 0; h < nh; ++h) {
            aoff[size_t(h)] = int64_t(pool.size());
            alen[size_t(h)] = int32_t(rg.haps[size_t(h)].bases.size());
            pool += rg.haps[size_t(h)].bases;
        }
        const int stride = 4 * (kWindow + 600) + 16;
        std::vector<int32_t> off(static_cast<size_t>(nh));
        std::vector<char> cig(size_t(nh) * size_t(stride));
        if (ref_sw_align_batch(nh, roff.data(), rlen.data(), reinterpret_cast<const uint8_t*>(rg.ref.data()),
                               aoff.data(), alen.data(), reinterpret_cast<const uint8_t*>(pool.data()), 200, -150, -260,
                               -11, HC_SW_SOFTCLIP, 1, off.data(), cig.data(), stride))
            return 3;
        std::vector<std::vector<Event>> ev_gpu, ev_ref;
        for (int h = 0; h < nh; ++h) {
            const std::string rc(cig.data() + size_t(h) * size_t(stride));
            bad_sw += size_t(off[size_t(h)]) != haps[size_t(h)].alignment_begin_wrt_ref || rc != haps[size_t(h)].cigar;
            ev_gpu.push_back(events_of(rg.ref, haps[size_t(h)].bases, haps[size_t(h)].alignment_begin_wrt_ref,
                                       haps[size_t(h)].cigar));
            ev_ref.push_back(events_of(rg.ref, rg.haps[size_t(h)].bases, size_t(off[size_t(h)]), rc));
        }
        // reads x haps through the reference kernels (rescue loop restated in the driver)
        std::vector<int64_t> pro, pho;
        std::vector<int32_t> pR, pH;
        std::string rs, q, gi, gc, hb;
        for (const auto& h : rg.haps) hb += h.bases;
        std::vector<int64_t> hoff(static_cast<size_t>(nh));
        for (int h = 1; h < nh; ++h) hoff[size_t(h)] = hoff[size_t(h - 1)] + int64_t(rg.haps[size_t(h - 1)].bases.size());
        for (const auto& r : rg.reads) {
            const int64_t o = int64_t(rs.size());
            rs += r.SEQ;
            q += r.QUAL;
            gi += std::string(r.SEQ.size(), 'I');
            gc += std::string(r.SEQ.size(), '+');
            for (int h = 0; h < nh; ++h) {
                pro.push_back(o);
                pR.push_back(int32_t(r.SEQ.size()));
                pho.push_back(hoff[size_t(h)]);
                pH.push_back(int32_t(rg.haps[size_t(h)].bases.size()));
            }
        }
        std::vector<double> RL(size_t(nr) * size_t(nh));
        auto U8 = [](const std::string& s) { return reinterpret_cast<const uint8_t*>(s.data()); };
        n_rescued += ref_pairs(long(pro.size()), pro.data(), pR.data(), pho.data(), pH.data(), U8(rs), U8(q), U8(gi),
                               U8(gi), U8(gc), U8(hb), nullptr, nullptr, nullptr, RL.data(), 0);
        std::vector<int32_t> rl;
        for (const auto& r : rg.reads) rl.push_back(int32_t(r.SEQ.size()));
        std::vector<uint8_t> keep(static_cast<size_t>(nr));
        hco_normalize(nr, nh, rl.data(), RL.data(), keep.data());
        std::vector<SAMRecord> ref_reads;
        std::vector<double> RLk;
        for (int r = 0; r < nr; ++r)
            if (keep[size_t(r)]) {
                ref_reads.push_back(rg.reads[size_t(r)]);
                RLk.insert(RLk.end(), RL.begin() + long(r) * nh, RL.begin() + long(r + 1) * nh);
            }
        // kept reads and matrices
        bool same_keep = reads.size() == ref_reads.size();
        for (size_t r = 0; same_keep && r < reads.size(); ++r) same_keep = reads[r].id == ref_reads[r].id;
        bad_keep += !same_keep;
        n_kept += long(reads.size());
        std::vector<double> GL;
        for (const auto& row : L) GL.insert(GL.end(), row.begin(), row.end());
        if (!same_keep || GL.size() != RLk.size() || std::memcmp(GL.data(), RLk.data(), sizeof(double) * GL.size()))
            ++bad_L;
        // sites (shared bookkeeping; identical inputs when SW and PairHMM agree)
        auto sg = sites_of(k, ev_gpu, reads);
        auto sr = sites_of(k, ev_ref, ref_reads);
        if (sg.size() != sr.size()) {
            ++bad_gt;
            continue;
        }
        region_L.push_back(std::move(GL));
        region_nh.push_back(nh);
        for (size_t s = 0; s < sr.size(); ++s) {
            std::vector<double> gl(size_t(sr[s].n_alleles * (sr[s].n_alleles + 1) / 2));
            int32_t gt = 0, gq = 0;
            hco_gt_site_with(RLk.data(), nh, sr[s].keep.data(), int(sr[s].keep.size()), sr[s].hap_allele.data(),
                             sr[s].n_alleles, gl.data(), &gt, &gq, ref_approx_log10_sum_log10);
            ref_gl.push_back(std::move(gl));
            ref_gt.push_back(gt);
            ref_gq.push_back(gq);
            sg[s].region = int(region_L.size()) - 1;
            all_sites.push_back(std::move(sg[s]));
        }
    }
    // the genotyper's arithmetic for every site of every region in one device call
    n_sites = long(all_sites.size());
    std::vector<std::vector<double>> gpu_gl(all_sites.size());
    std::vector<int32_t> gpu_gt(all_sites.size()), gpu_gq(all_sites.size());
    for (size_t s = 0; s < all_sites.size(); ++s) {
        const Site& st = all_sites[s];
        const int nh = region_nh[size_t(st.region)];
        gpu_gl[s].resize(size_t(st.n_alleles * (st.n_alleles + 1) / 2));
        gpu_sites.push_back(hc_gt_site{region_L[size_t(st.region)].data(),
                                       int32_t(region_L[size_t(st.region)].size() / size_t(nh)), nh, st.keep.data(),
                                       int32_t(st.keep.size()), st.hap_allele.data(), st.n_alleles, gpu_gl[s].data(),
                                       &gpu_gt[s], &gpu_gq[s]});
    }
    if (!gpu_sites.empty() && hc_gt_genotype_sites(gpu_sites.data(), int32_t(gpu_sites.size())) != 0) return 4;
    for (size_t s = 0; s < all_sites.size(); ++s) {
        bad_gl += gpu_gl[s].size() != ref_gl[s].size() ||
                  std::memcmp(gpu_gl[s].data(), ref_gl[s].data(), sizeof(double) * gpu_gl[s].size()) != 0;
        bad_gt += gpu_gt[s] != ref_gt[s] || gpu_gq[s] != ref_gq[s];
        n_called += ref_gt[s] != 0;
    }
    FILE* f = std::fopen(argv[3], "w");
    if (!f) return 5;
    std::fprintf(f,
                 "{\"regions\": %d, \"haplotypes\": %ld, \"reads\": %ld, \"reads_kept\": %ld, \"rescued\": %ld, "
                 "\"sites\": %ld, \"non_ref_genotypes\": %ld, \"sw_mismatch\": %ld, \"keep_mismatch\": %ld, "
                 "\"likelihood_mismatch\": %ld, \"gl_mismatch\": %ld, \"gt_gq_mismatch\": %ld}\n",
                 nreg, n_haps, n_reads, n_kept, n_rescued, n_sites, n_called, bad_sw, bad_keep, bad_L, bad_gl, bad_gt);
    std::fclose(f);
    return (bad_sw | bad_keep | bad_L | bad_gl | bad_gt) ? 1 : 0;
}
