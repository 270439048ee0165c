// Host planner of a part (the reference's getData, intel_pairhmm.hpp:154-203,
// and the per-pair set-up of compute_full_prob_avx{s,d}, done once per batch):
// length-bin the pairs, choose each pair's column-segmented shape, pack the
// pairs into 64-lane waves, fill the pinned staging image, and enqueue the
// H2D and the device packing. Cross products (regions) take the structured
// planner (plan_grid), whose descriptors and waves are built on the device.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <numeric>

#include "engine_core.hpp"
#include "luts.hpp"
#include "plan_model.hpp"
#include "pool.hpp"

namespace hcphmm {
namespace eng {
namespace {

constexpr int kW64Threshold = 768;     // anti-diagonal kernel: H above this -> one pair per wave
constexpr int kLaneMaxH = 4096;        // longer haps stay on the anti-diagonal kernel (policy "auto")
constexpr int kSegWavesPerSimd = 3;    // resident seg waves per SIMD (phmm_seg_kernel occupancy)

int lane_variant_id() { return int(env_i64("HC_PHMM_LANE_VARIANT", 0)); }

// HC_PHMM_LANE_SEG = auto (default) | all | off. Returns -1 auto, 0 off, 1 all.
int lane_seg_policy()
{
    const char* e = std::getenv("HC_PHMM_LANE_SEG");
    if (!e || !*e || !std::strcmp(e, "auto")) return -1;
    return std::strcmp(e, "all") ? 0 : 1;
}

// HC_PHMM_KERNEL = auto (lane kernels for H <= kLaneMaxH) | lane | diag.
int kernel_policy()
{
    const char* e = std::getenv("HC_PHMM_KERNEL");
    if (!e || !*e || !std::strcmp(e, "auto")) return 0;
    if (!std::strcmp(e, "lane")) return 1;
    return 2;
}

// LSD radix sort of `idx` by a 32-bit key, DESCENDING, stable (fallback of
// the counting sort when the key range is wide).
void sort_desc(std::vector<int>& idx, const std::vector<uint32_t>& key)
{
    if (idx.size() < 2) return;
    uint32_t kmax = 0;
    for (int p : idx) kmax = std::max(kmax, key[p]);
    const size_t n = idx.size();
    std::vector<uint64_t> v(n), tmp(n);
    for (size_t k = 0; k < n; ++k) v[k] = (uint64_t(kmax - key[idx[k]]) << 32) | uint32_t(idx[k]);
    constexpr int kBits = 11, kBuckets = 1 << kBits;
    for (int shift = 0; shift < 32 && (kmax >> shift) != 0; shift += kBits) {
        size_t cnt[kBuckets + 1] = {};
        for (uint64_t x : v) ++cnt[((x >> (32 + shift)) & (kBuckets - 1)) + 1];
        for (int k = 1; k <= kBuckets; ++k) cnt[k] += cnt[k - 1];
        for (uint64_t x : v) tmp[cnt[(x >> (32 + shift)) & (kBuckets - 1)]++] = x;
        v.swap(tmp);
    }
    for (size_t k = 0; k < n; ++k) idx[k] = int(uint32_t(v[k]));
}

// Stable parallel counting sort of `idx` by bucket(p) DESCENDING, buckets < nb.
template <typename B>
void counting_sort_desc(std::vector<int>& idx, std::vector<int>& out, std::vector<int64_t>& hist, int nb, B bucket)
{
    const int64_t n = int64_t(idx.size());
    if (n < 2) return;
    const int T = int(std::min<int64_t>(64, std::max<int64_t>(1, n / 8192)));
    const int64_t chunk = (n + T - 1) / T;
    hist.assign(size_t(T) * nb, 0);
    WorkerPool::get().run(T, [&](int t) {
        int64_t* h = hist.data() + size_t(t) * nb;
        for (int64_t k = t * chunk, e = std::min(n, k + chunk); k < e; ++k) ++h[bucket(idx[k])];
    });
    int64_t run = 0;
    for (int b = nb - 1; b >= 0; --b)
        for (int t = 0; t < T; ++t) {
            int64_t& h = hist[size_t(t) * nb + b];
            const int64_t c = h;
            h = run;
            run += c;
        }
    out.resize(size_t(n));
    WorkerPool::get().run(T, [&](int t) {
        int64_t* h = hist.data() + size_t(t) * nb;
        for (int64_t k = t * chunk, e = std::min(n, k + chunk); k < e; ++k) out[h[bucket(idx[k])]++] = idx[k];
    });
    idx.swap(out);
}

// Bump allocator over one region: 256-B aligned segments.
struct Layout {
    size_t off = 0;
    size_t take(size_t bytes)
    {
        const size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    }
};

// Whether a read's (i, d, c) gap qualities are the same on every row (then
// they travel once, in its descriptor). Blocks of 64 rows without early exit
// inside a block, so the compiler vectorises the compare.
bool constant_gaps(const ReadView& v)
{
    const uint8_t i0 = v.i[0], d0 = v.d[0], c0 = v.c[0];
    int k = 0;
    for (; k + 64 <= v.len; k += 64) {
        uint8_t a = 0;
        for (int j = 0; j < 64; ++j) a |= uint8_t((v.i[k + j] ^ i0) | (v.d[k + j] ^ d0) | (v.c[k + j] ^ c0));
        if (a) return false;
    }
    uint8_t a = 0;
    for (; k < v.len; ++k) a |= uint8_t((v.i[k] ^ i0) | (v.d[k] ^ d0) | (v.c[k] ^ c0));
    return a == 0;
}

// The part's reads / haps in part-local order, and the (read, hap) of each
// part-local pair.
struct Local {
    const Src* src;
    const PartSpec* spec;
    int64_t nr = 0, nh = 0, np = 0;
    std::vector<int64_t> blk_r, blk_h, blk_p;   // per block: first local read / hap / pair

    Local(const Src& s, const PartSpec& p) : src(&s), spec(&p)
    {
        if (p.flat) {
            nr = nh = np = p.hi - p.lo;
            return;
        }
        for (const Block& b : p.blocks) {
            blk_r.push_back(nr);
            blk_h.push_back(nh);
            blk_p.push_back(np);
            nr += b.nr;
            nh += b.nh;
            np += int64_t(b.nr) * b.nh;
        }
        blk_p.push_back(np);
    }
    int64_t read_id(int64_t lr) const   // Src read index of local read lr
    {
        if (spec->flat) return spec->lo + lr;
        const size_t b = size_t(std::upper_bound(blk_r.begin(), blk_r.end(), lr) - blk_r.begin()) - 1;
        return spec->blocks[b].r0 + (lr - blk_r[b]);
    }
    int64_t hap_mult(int64_t lh) const   // reads paired with local hap lh
    {
        if (spec->flat) return 1;
        const size_t b = size_t(std::upper_bound(blk_h.begin(), blk_h.end(), lh) - blk_h.begin()) - 1;
        return spec->blocks[b].nr;
    }
    int64_t hap_id(int64_t lh) const
    {
        if (spec->flat) return spec->lo + lh;
        const size_t b = size_t(std::upper_bound(blk_h.begin(), blk_h.end(), lh) - blk_h.begin()) - 1;
        return spec->blocks[b].h0 + (lh - blk_h[b]);
    }
    // f(k, local read, local hap) for pairs k in [lo, hi).
    template <typename F>
    void pairs(int64_t lo, int64_t hi, F&& f) const
    {
        if (lo >= hi) return;
        if (spec->flat) {
            for (int64_t k = lo; k < hi; ++k) f(k, k, k);
            return;
        }
        size_t b = size_t(std::upper_bound(blk_p.begin(), blk_p.end(), lo) - blk_p.begin()) - 1;
        int64_t k = lo;
        while (k < hi) {
            const Block& B = spec->blocks[b];
            const int64_t base = blk_p[b], end = std::min(hi, blk_p[b + 1]);
            int64_t r = (k - base) / B.nh, h = (k - base) % B.nh;
            for (; k < end; ++k) {
                f(k, blk_r[b] + r, blk_h[b] + h);
                if (++h == B.nh) {
                    h = 0;
                    ++r;
                }
            }
            ++b;
        }
    }
};

// A structured plan's segment tables for the device (launch_grid_waves).
struct GridDev {
    std::vector<GridSeg> segs;
    std::vector<int> rord, hord;
    int64_t slots = 0, waves = 0;
};

// Grow-only per-thread scratch of the planner: fresh large vectors would be
// fresh mmap'd pages, zero-filled by the kernel on first touch, every call.
struct PlanScratch {
    std::vector<int32_t> rlen, gapw, hlen;
    std::vector<int64_t> row_off, gap_off, hap_w, hap_b;
    std::vector<uint8_t> hcls, cls, seg_bc, seg_nb, used, in_tail;
    std::vector<uint32_t> srec;   // (BC, nb, R) of the segmented pairs in sorted order
    std::vector<uint32_t> hcand, key;
    std::vector<Cand> ctab;
    GridDev gdev;
    std::vector<int> seg_in, one_ord, ord2[2], seg_ord, sort_tmp;
    std::vector<LaneWave> lw, ordered;
    std::vector<int64_t> wcost;
    std::vector<uint64_t> wkey;
    std::vector<std::vector<LaneWave>> part_w;
    std::vector<int64_t> hist;
};
thread_local PlanScratch t_scr;

template <typename T>
void grow(std::vector<T>& v, size_t n)
{
    if (v.size() < n) v.resize(n);
}


// The candidate policy of a structured plan: each hap's cheaper candidate
// (-1), or candidate 0 / 1 for every hap, whichever the pass model prices
// lowest over the plan's actual waves. The per-hap choice can push a pass over
// a waves-per-SIMD boundary the width cap's model (choose_cap: ~60 lanes per
// wave) did not count on: a 415 x 32 region took 10 lanes of 42 columns per
// hap, 6 pairs per wave, 2 214 waves — 190 SIMDs with a third wave, which ran
// alone after the other two: fp32 pass 0.40 ms, where 9 lanes of 48 columns
// (7 pairs, 1 898 waves, two per SIMD) take 0.21 ms. The model: a SIMD with n
// waves takes 3 floor(n/3) rounds plus 2 for a partial round (its last one or
// two waves issue alone or in a pair), up to 9 waves per SIMD (a region's
// waves are alike, so the SIMDs holding one more wave set the pass); past
// that, rounds follow the total work (priced up to 12, it moved a 415 x 200
// region to 11 858 narrower waves: 1.32 -> 1.43 ms; up to 6, it left a
// 415 x 128 region at 6 491 waves where 5 903 take 4 % less).
template <typename CandOf>
int grid_policy(const Local& loc, const int32_t* rlen, CandOf&& hcand, const float* waste, int n_simd,
                double* est_out = nullptr)
{
    const PartSpec& spec = *loc.spec;
    int best_pol = -1;
    double best = 0;
    std::vector<std::pair<uint16_t, int>> cnt;
    for (int pol = -1; pol <= 1; ++pol) {
        double waves = 0, work = 0;
        for (size_t b = 0; b < spec.blocks.size(); ++b) {
            const Block& B = spec.blocks[b];
            if (B.nr <= 0 || B.nh <= 0) continue;
            const int64_t r0 = loc.blk_r[b], h0 = loc.blk_h[b];
            int64_t rs = 0;
            for (int r = 0; r < B.nr; ++r) rs += rlen[r0 + r];
            const int Rm = int((rs + B.nr / 2) / B.nr);
            cnt.clear();
            for (int h = 0; h < B.nh; ++h) {
                const Cand cd = hcand(h0 + h);
                const int q = pol >= 0 ? pol
                              : seg_cost(cd.nb[1], cd.bc[1], Rm, waste) < seg_cost(cd.nb[0], cd.bc[0], Rm, waste) ? 1
                                                                                                                 : 0;
                const uint16_t k = uint16_t(cd.bc[q] << 8 | cd.nb[q]);
                auto it = std::find_if(cnt.begin(), cnt.end(), [&](const auto& e) { return e.first == k; });
                if (it == cnt.end()) cnt.push_back({k, 1});
                else ++it->second;
            }
            for (const auto& e : cnt) {
                const int bc = e.first >> 8, nb = e.first & 0xff, per = 64 / nb;
                const double w = double((int64_t(B.nr) * e.second + per - 1) / per);
                waves += w;
                work += w * (13.0 * bc + 26.0) * double(Rm + nb - 1);
            }
        }
        if (waves <= 0) {
            if (est_out) *est_out = 0;
            return -1;
        }
        const double per_simd = waves / double(n_simd);
        double rounds = per_simd;
        if (per_simd <= 9.0) {
            const int n = std::max(1, int(std::ceil(per_simd - 1e-9)));
            rounds = 3.0 * (n / 3) + (n % 3 ? 2.0 : 0.0);
        }
        const double est = rounds * work / waves;
        if (pol == -1 || est < best * 0.98) {
            best = est;
            best_pol = pol;
        }
    }
    if (est_out) *est_out = best;
    return best_pol;
}

// Cross-product fast path of the planner (regions: hc_phmm_cross,
// cross_regions, submit_regions) when every hap takes segmented waves. The
// pairs of a block are reads x haps, so their sorted order need not be found
// by sorting pairs: each hap takes one (BC, nb) candidate (chosen at its
// block's mean read length), the block's haps are grouped by (BC, nb) and its
// reads sorted by R, and a group's pairs in (read by R descending) x (hap)
// order fill waves of floor(64 / nb) pairs — the order the general planner's
// sort + greedy packing reaches on such a batch, built in one parallel pass
// over segments (one per block and group; a segment's last wave may be
// partial). Segments run widest block first, so co-resident waves share a
// width's code. Writes every pair's descriptor, the slot order and the waves;
// returns the batch's cells.
int64_t plan_grid(const Local& loc, const int32_t* rlen, const int32_t* hlen, const int64_t* row_off,
                  const int64_t* hap_w, const Cand* hcand, const float* waste, int qforce, PairDesc* pd,
                  bool write_pairs, std::vector<int>& seg_ord, std::vector<LaneWave>& lw, PhaseTimer& tm,
                  GridDev* gd)
{
    const PartSpec& spec = *loc.spec;
    const size_t nblk = spec.blocks.size();
    // Per block: reads by R descending, haps grouped by their (BC, nb) key.
    std::vector<int> rord(size_t(loc.nr)), hord(size_t(loc.nh));
    std::vector<uint16_t> hkey(size_t(loc.nh));
    struct Seg {
        uint32_t key;   // bc << 8 | nb
        int blk;
        int g0, G;      // haps hord[g0 .. g0 + G) (local ids)
        int64_t n, slot0, w0;
    };
    std::vector<std::vector<Seg>> bsegs(nblk);
    parallel_for(int64_t(nblk), [&](int64_t lo, int64_t hi) {
        for (int64_t b = lo; b < hi; ++b) {
            const Block& B = spec.blocks[size_t(b)];
            const int64_t r0 = loc.blk_r[size_t(b)], h0 = loc.blk_h[size_t(b)];
            int64_t rs = 0;
            for (int r = 0; r < B.nr; ++r) {
                rord[size_t(r0 + r)] = int(r0 + r);
                rs += rlen[r0 + r];
            }
            std::stable_sort(rord.begin() + r0, rord.begin() + r0 + B.nr,
                             [&](int x, int y) { return rlen[x] > rlen[y]; });
            const int Rm = int((rs + B.nr / 2) / std::max(1, B.nr));
            for (int h = 0; h < B.nh; ++h) {
                const int lh = int(h0 + h);
                const Cand cd = hcand[lh];
                const int q = qforce >= 0 ? qforce
                              : seg_cost(cd.nb[1], cd.bc[1], Rm, waste) < seg_cost(cd.nb[0], cd.bc[0], Rm, waste) ? 1
                                                                                                                 : 0;
                hkey[size_t(lh)] = uint16_t(cd.bc[q] << 8 | cd.nb[q]);
                hord[size_t(lh)] = lh;
            }
            std::stable_sort(hord.begin() + h0, hord.begin() + h0 + B.nh,
                             [&](int x, int y) { return hkey[size_t(x)] > hkey[size_t(y)]; });
            auto& out = bsegs[size_t(b)];
            out.clear();
            for (int g = 0; g < B.nh;) {
                const uint16_t k = hkey[size_t(hord[size_t(h0 + g)])];
                int e = g;
                while (e < B.nh && hkey[size_t(hord[size_t(h0 + e)])] == k) ++e;
                out.push_back(Seg{k, int(b), int(h0 + g), e - g, int64_t(B.nr) * (e - g), 0, 0});
                g = e;
            }
        }
    }, 1);
    tm.mark("grid: blocks");
    std::vector<Seg> segs;
    for (auto& v : bsegs) segs.insert(segs.end(), v.begin(), v.end());
    std::stable_sort(segs.begin(), segs.end(), [](const Seg& x, const Seg& y) { return x.key > y.key; });
    int64_t slots = 0, waves = 0;
    for (Seg& g : segs) {
        g.slot0 = slots;
        g.w0 = waves;
        slots += g.n;
        waves += (g.n + 64 / int(g.key & 0xff) - 1) / (64 / int(g.key & 0xff));
    }
    if (gd) {   // order and waves built on the device from the segments (launch_grid_waves)
        gd->slots = slots;
        gd->waves = waves;
        gd->segs.resize(segs.size());
        for (size_t k = 0; k < segs.size(); ++k) {
            const Seg& g = segs[k];
            const Block& B = spec.blocks[size_t(g.blk)];
            gd->segs[k] = GridSeg{g.slot0, loc.blk_p[size_t(g.blk)], int(g.w0), int(loc.blk_r[size_t(g.blk)]), B.nr,
                                  B.nh, int(loc.blk_h[size_t(g.blk)]), g.g0, g.G, int(g.key >> 8),
                                  int(g.key & 0xff), 0};
        }
        gd->rord.swap(rord);
        gd->hord.swap(hord);
        seg_ord.clear();
        lw.clear();
    } else {
    seg_ord.resize(size_t(slots));
    lw.resize(size_t(waves));
    parallel_for(int64_t(segs.size()), [&](int64_t lo, int64_t hi) {
        for (int64_t t = lo; t < hi; ++t) {
            const Seg& g = segs[size_t(t)];
            const Block& B = spec.blocks[size_t(g.blk)];
            const int64_t r0 = loc.blk_r[size_t(g.blk)], h0 = loc.blk_h[size_t(g.blk)], p0 = loc.blk_p[size_t(g.blk)];
            const int bc = int(g.key >> 8), nb = int(g.key & 0xff), per = 64 / nb;
            int* o = seg_ord.data() + g.slot0;
            int64_t i = 0;
            for (int rr = 0; rr < B.nr; ++rr) {
                const int64_t rowbase = p0 + (rord[size_t(r0 + rr)] - r0) * int64_t(B.nh) - h0;
                for (int hh = 0; hh < g.G; ++hh) o[i++] = int(rowbase + hord[size_t(g.g0 + hh)]);
            }
            for (int64_t w = 0; w * per < g.n; ++w) {
                const int64_t a = w * per, e = std::min(g.n, a + per);
                const int Rmax = rlen[rord[size_t(r0 + a / g.G)]];
                const int Rmin = rlen[rord[size_t(r0 + (e - 1) / g.G)]];
                LaneWave v{};
                v.slot0 = int(g.slot0 + a);
                v.ncols = bc;
                v.npairs = int(e - a);
                v.rmax = Rmax;
                v.rmin = Rmin;
                v.nsteps = Rmax + nb - 1;
                lw[size_t(g.w0 + w)] = v;
            }
        }
    }, 1);
    }   // host order and waves
    tm.mark("grid: slots + waves");
    if (!write_pairs) {   // descriptors built on the device (launch_grid_pairs): cells from block sums
        int64_t cells = 0;
        for (size_t b = 0; b < nblk; ++b) {
            const Block& B = spec.blocks[b];
            int64_t sr = 0, sh = 0;
            for (int r = 0; r < B.nr; ++r) sr += rlen[loc.blk_r[b] + r];
            for (int h = 0; h < B.nh; ++h) sh += hlen[loc.blk_h[b] + h];
            cells += sr * sh;
        }
        return cells;
    }
    // Pair descriptors (read-major within each block, as Local::pairs).
    std::atomic<int64_t> cells{0};
    parallel_for(loc.np, [&](int64_t lo, int64_t hi) {
        int64_t c = 0;
        loc.pairs(lo, hi, [&](int64_t k, int64_t r, int64_t h) {
            const int R = rlen[r], H = hlen[h];
            pd[k] = PairDesc{int(row_off[r]), R, int(hap_w[h]), H};
            c += int64_t(R) * H;
        });
        cells += c;
    }, 16384);
    return cells.load();
}

// Plan one part on device d: host binning + staging, then the H2D, device
// packing and (with_run) the device pass and the D2H of the results, all
// enqueued on d's stream. slot == nullptr: the part owns its memory (batches).
}  // namespace

int plan_part(Device& dv, const Src& src, const PartSpec& spec, Slot* slot, bool with_run, PlanMode mode,
              Part** out)
{
    const bool dry = mode == PlanMode::Dry;
    PhaseTimer tm;
    Local loc(src, spec);
    const int64_t nr = loc.nr, nh = loc.nh, npairs = loc.np;
    if (npairs > (int64_t(1) << 31) - 1) return fail(HC_PHMM_EINVAL, "too many pairs for one batch");

    // Reads: validate, lengths, gap-quality constancy; haps: validate, lengths.
    PlanScratch& S = t_scr;
    grow(S.rlen, size_t(nr));
    grow(S.gapw, size_t(nr));
    grow(S.hlen, size_t(nh));
    int32_t* rlen = S.rlen.data();
    int32_t* gapw = S.gapw.data();
    int32_t* hlen = S.hlen.data();
    std::atomic<int> bad_read{0}, bad_hap{0}, rlen_max{0};
    std::atomic<int64_t> rows_sum{0};
    parallel_for(nr, [&](int64_t lo, int64_t hi) {
        int rm = 0;
        int64_t rs = 0;
        for (int64_t r = lo; r < hi; ++r) {
            const ReadView v = src.read(loc.read_id(r));
            if (v.len <= 0 || v.len > HC_PHMM_MAX_READ_LEN || !v.bases || !v.q || !v.i || !v.d || !v.c) {
                bad_read.store(1);
                rlen[size_t(r)] = 0;
                gapw[size_t(r)] = 0;
                continue;
            }
            rlen[size_t(r)] = v.len;
            rm = std::max(rm, v.len);
            rs += v.len;
            gapw[size_t(r)] = constant_gaps(v) ? int32_t((v.i[0] & 127) | ((v.d[0] & 127) << 7) | ((v.c[0] & 127) << 14))
                                               : -1;
        }
        rows_sum.fetch_add(rs);
        int cur = rlen_max.load();
        while (rm > cur && !rlen_max.compare_exchange_weak(cur, rm)) {
        }
    }, 2048);
    if (bad_read.load()) return fail(HC_PHMM_EINVAL, "read with invalid length or null array");
    parallel_for(nh, [&](int64_t lo, int64_t hi) {
        for (int64_t h = lo; h < hi; ++h) {
            const HapView v = src.hapv(loc.hap_id(h));
            const bool ok = v.len > 0 && v.len <= HC_PHMM_MAX_HAP_LEN && v.bases;
            if (!ok) bad_hap.store(1);
            hlen[size_t(h)] = ok ? v.len : 0;
        }
    }, 8192);
    if (bad_hap.load())
        return fail(HC_PHMM_EINVAL, "haplotype with invalid length (1.." + std::to_string(HC_PHMM_MAX_HAP_LEN) +
                                        ") or null bases");
    // rows / irregular gap rows / table words / hap code bytes. Bases and hap
    // bases are staged as ConvertChar codes, two per byte; a read's rows start
    // at a multiple of 4, a hap's codes at a multiple of 8 columns: the packer
    // loads 4 rows / 8 hap columns per lane (launch_pack_batch).
    std::vector<int64_t>&row_off = S.row_off, &gap_off = S.gap_off, &hap_w = S.hap_w, &hap_b = S.hap_b;
    prefix_sum(nr, row_off, [&](int64_t r) -> int64_t { return (rlen[size_t(r)] + 3) & ~3; });
    prefix_sum(nr, gap_off, [&](int64_t r) -> int64_t { return gapw[size_t(r)] < 0 ? (rlen[size_t(r)] + 3) & ~3 : 0; });
    prefix_sum(nh, hap_w, [&](int64_t h) -> int64_t { return hap_table_words(hlen[size_t(h)]); });
    prefix_sum(nh, hap_b, [&](int64_t h) -> int64_t { return ((hlen[size_t(h)] + 7) & ~7) / 2; });
    const int64_t nrows = row_off[size_t(nr)], ngap = gap_off[size_t(nr)];
    if (nrows > INT32_MAX || hap_w[size_t(nh)] > INT32_MAX || hap_b[size_t(nh)] > INT32_MAX || ngap > INT32_MAX)
        return fail(HC_PHMM_EINVAL, "batch too large (row or hap pool exceeds 2^31)");
    tm.mark("reads/haps scan");

    // Staging layout (upload part first; waves last, their count is known later).
    Layout U;
    const size_t o_pairs = U.take(sizeof(PairDesc) * size_t(npairs));
    const size_t o_rd = U.take(sizeof(int4) * size_t(nr));
    const size_t o_hd = U.take(sizeof(int4) * size_t(nh));
    const size_t o_ord = U.take(sizeof(int) * size_t(npairs));
    const size_t o_slotof = U.take(sizeof(int) * size_t(npairs));   // pair -> seg slot (-1: other kernels)
    const size_t o_bases = U.take(size_t(nrows) / 2 + 16);
    const size_t o_quals = U.take(size_t(nrows) + 16);
    const size_t gap_stride = (size_t(ngap) + 16 + 15) & ~size_t(15);
    const size_t o_gaps = U.take(ngap ? 3 * gap_stride : 0);
    const size_t o_hb = U.take(size_t(hap_b[size_t(nh)]) + 16);
    const size_t o_lw = U.off;   // LaneWave array, sized after packing

    // Pinned staging: upper bound for the waves (one per seg pair at most, plus
    // one-lane waves) and the results image after the upload.
    const size_t waves_max = sizeof(LaneWave) * (size_t(npairs) + 1) + sizeof(GridBlock) * spec.blocks.size() +
                             sizeof(GridSeg) * size_t(nh) + sizeof(int) * size_t(nr + nh) + 1024;
    const size_t n1 = size_t(std::max<int64_t>(npairs, 1));
    const ResLayout RL = res_layout(n1);
    const size_t res_bytes = RL.bytes;
    const size_t host_upload_cap = o_lw + waves_max;
    const size_t host_res_off = (host_upload_cap + 255) & ~size_t(255);
    char* host = nullptr;
    bool own_host = false;
    thread_local std::vector<char> dry_host;   // dry runs: plain memory
    if (dry) {
        if (dry_host.size() < host_res_off + res_bytes) dry_host.resize(host_res_off + res_bytes);
        host = dry_host.data();
    } else if (slot) {
        const int rc = slot_reserve(*slot, 0, host_res_off + res_bytes);
        if (rc) return rc;
        host = slot->host;
    } else {
        if (hipHostMalloc(&host, std::max<size_t>(host_upload_cap, 1), hipHostMallocPortable) != hipSuccess)
            return fail(HC_PHMM_ENOMEM, "pinned staging buffer");
        own_host = true;
    }
    struct HostGuard {
        char* p;
        bool own;
        ~HostGuard()
        {
            if (own && p) (void)hipHostFree(p);
        }
    } hguard{host, own_host};
    tm.mark("staging alloc");

    // Per hap: kernel class, lanes at each width cap (times the reads it pairs
    // with), then the pass's cap and the hap's two (BC, nb) candidates.
    PairDesc* pd = reinterpret_cast<PairDesc*>(host + o_pairs);
    const int pol = kernel_policy();
    const bool use_lane = pol != 2;
    const int seg_max_h = lane_seg_policy() == 0 ? 0 : 64 * kSegMaxBC;
    // class: 0 seg, 1 one-lane, 2 diag W16, 3 diag W64
    grow(S.hcls, size_t(nh));
    uint8_t* hcls = S.hcls.data();
    std::atomic<int64_t> wide_a{0};
    std::atomic<int> hmax_a{0};
    // Modelled wave instructions at each cap (plan_model.hpp), for the cap choice.
    const double ravg = double(rows_sum.load()) / double(std::max<int64_t>(nr, 1));
    std::mutex work_mu;
    std::array<int64_t, kNCaps> lanes_at{};
    std::array<double, kNCaps> work_at{};
    // The cap model needs only totals: past 8k haps it prices every stride-th
    // hap (weighted by the stride), which is all the cap choice can resolve.
    const int64_t cap_stride = std::max<int64_t>(1, nh / 8192);
    parallel_for(nh, [&](int64_t lo, int64_t hi) {
        int64_t w = 0;
        int hm = 0;
        const int32_t* __restrict hl = hlen;
        uint8_t* __restrict hc = hcls;
        for (int64_t h = lo; h < hi; ++h) {
            const int H = hl[h];
            int cl;
            if (use_lane && (pol == 1 || H <= kLaneMaxH))
                cl = H > seg_max_h ? 1 : 0;
            else
                cl = H > kW64Threshold ? 3 : 2;
            hc[h] = uint8_t(cl);
            hm = std::max(hm, H);
            w += H > kSeg64MaxH ? loc.hap_mult(h) : 0;
        }
        wide_a += w;
        int cur = hmax_a.load();
        while (hm > cur && !hmax_a.compare_exchange_weak(cur, hm)) {
        }
    }, 1 << 14);
    parallel_for((nh + cap_stride - 1) / cap_stride, [&](int64_t lo, int64_t hi) {
        int64_t lanes[kNCaps] = {};
        double work[kNCaps] = {};
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t h = i * cap_stride;
            if (hcls[size_t(h)] != 0) continue;
            cap_sample(hlen[size_t(h)], ravg, cap_stride * loc.hap_mult(h), lanes, work);
        }
        std::lock_guard<std::mutex> lk(work_mu);
        for (int q = 0; q < kNCaps; ++q) {
            lanes_at[size_t(q)] += lanes[q];
            work_at[size_t(q)] += work[q];
        }
    }, 4096);
    tm.mark("hap classes: cost");
    CapChoice cc = choose_cap(lanes_at.data(), work_at.data(), dv.n_cu);
    {
        const int64_t forced = env_i64("HC_PHMM_SEG_CAP", 0);
        if (forced > 0) cc = CapChoice{int(std::max<int64_t>(kSegMinBC, std::min<int64_t>(kSegMaxBC, forced))), false};
    }
    const int cap = cc.cap;
    // A pass with few waves per SIMD is latency-bound: its time is one wave's,
    // so the candidate with the shorter wave wins there (S1: 11 lanes of 14
    // columns beat 10 of 16; S1w: 12 of 22 beat 11 of 24).
    const float* waste = cc.few_waves ? waste_per_lane() : waste_half();
    grow(S.hcand, size_t(nh));
    Cand* hcand = reinterpret_cast<Cand*>(S.hcand.data());
    // Many haps (flat batches: one per pair): the candidates by H from a table
    // (divisions once per length, not per hap).
    const int hmax_seg = std::min(hmax_a.load(), seg_max_h);
    std::vector<Cand>& ctab = S.ctab;
    const bool by_table = nh > 4 * int64_t(hmax_seg + 1);
    if (by_table) {
        ctab.resize(size_t(hmax_seg) + 1);
        for (int H = 1; H <= hmax_seg; ++H) ctab[size_t(H)] = cand_of(H, cap);
    }
    parallel_for(nh, [&](int64_t lo, int64_t hi) {
        for (int64_t h = lo; h < hi; ++h) {
            if (hcls[size_t(h)] != 0) continue;
            const int H = hlen[size_t(h)];
            hcand[size_t(h)] = by_table ? ctab[size_t(H)] : cand_of(H, cap);
        }
    }, 1 << 14);
    tm.mark("hap classes");

    std::atomic<int64_t> cells_a{0};
    std::vector<int>&one_ord = S.one_ord, (&ord2)[2] = S.ord2;
    std::vector<int>& seg_ord = S.seg_ord;
    std::vector<LaneWave>& lw = S.lw;
    lw.clear();
    const int qforce = int(env_i64("HC_PHMM_SEG_Q", -1));   // sweeps: force the nb0 (0) or nb0 + 1 (1) candidate
    // Cross products whose haps all take segmented waves (every region call):
    // the structured planner (plan_grid); HC_PHMM_GRID_PLAN=0 forces the
    // general one (A/B, tests).
    bool grid = !spec.flat && env_i64("HC_PHMM_GRID_PLAN", 1) != 0;
    for (int64_t h = 0; grid && h < nh; ++h) grid = hcls[size_t(h)] == 0;
    // Structured plans outside dry runs: pair descriptors, slot order and waves
    // are built on the device from the block and segment tables.
    const bool dev_plan = grid && !dry;
    GridDev& gd = S.gdev;
    if (grid) {
        one_ord.clear();
        ord2[0].clear();
        ord2[1].clear();
        // The width cap and candidate policy of a structured plan, priced over
        // its actual waves (grid_policy) at every cap: the cap model's ~60
        // filled lanes per wave misjudges haps that need more than 32 lanes
        // (one pair per wave): a 415 x 8 region took 12-column blocks, 35
        // lanes, one pair per wave, 3 320 waves (a fourth wave on a quarter
        // of the SIMDs), where 16-column blocks give two pairs per wave and
        // 1 660 waves.
        int qgrid = qforce;
        if (qforce < 0 && env_i64("HC_PHMM_GRID_POLICY", 1) != 0) {
            const int n_simd = 4 * dv.n_cu;
            double best = 0;
            qgrid = grid_policy(loc, rlen, [&](int64_t h) { return hcand[h]; }, waste, n_simd, &best);
            const double best_default = best;
            int best_cap = cap;
            if (env_i64("HC_PHMM_SEG_CAP", 0) <= 0 && env_i64("HC_PHMM_GRID_CAPS", 1) != 0)
                for (int c : kCaps) {
                    if (c == cap) continue;
                    double e = 0;
                    const int q = grid_policy(loc, rlen, [&](int64_t h) { return cand_of(hlen[size_t(h)], c); }, waste,
                                              n_simd, &e);
                    if (e > 0 && e < best * 0.98 && e < best_default * 0.95) {   // (another cap only for a clear gain)
                        best = e;
                        best_cap = c;
                        qgrid = q;
                    }
                }
            if (best_cap != cap)
                parallel_for(nh, [&](int64_t lo, int64_t hi) {
                    for (int64_t h = lo; h < hi; ++h)
                        if (hcls[size_t(h)] == 0) hcand[size_t(h)] = cand_of(hlen[size_t(h)], best_cap);
                }, 1 << 14);
        }
        cells_a = plan_grid(loc, rlen, hlen, row_off.data(), hap_w.data(), hcand, waste, qgrid, pd, !dev_plan, seg_ord, lw,
                            tm, dev_plan ? &gd : nullptr);
        tm.mark("grid: pairs");
    } else {
        // Per pair: descriptor straight into the staging image, class, and for
        // segmented pairs the cheaper candidate for its R.
        grow(S.cls, size_t(npairs));
        grow(S.seg_bc, size_t(npairs));
        grow(S.seg_nb, size_t(npairs));
        uint8_t *cls = S.cls.data(), *seg_bc = S.seg_bc.data(), *seg_nb = S.seg_nb.data();
        std::atomic<int> rmin_a{INT32_MAX}, rmax_a{0};
        // Pairs per planning task (a 415 x 128 region call on the GPU box: 2.0 ms
        // at 8192, 2.96 ms on one task; tools/region_ab.py).
        const int64_t task_pairs = std::max<int64_t>(1024, env_i64("HC_PHMM_TASK_PAIRS", 8192));
        const int T = int(std::min<int64_t>(64, std::max<int64_t>(1, npairs / task_pairs)));
        const int64_t pchunk = (npairs + T - 1) / T;
        std::vector<std::array<int64_t, 4>> tcnt(size_t(T) + 1);
        WorkerPool::get().run(T, [&](int t) {
            const int64_t lo = t * pchunk, hi = std::min(npairs, lo + pchunk);
            // Plain restrict locals: the uint8_t stores below may alias anything,
            // so anything reached through a capture would be reloaded per pair.
            const int32_t* __restrict rl = rlen;
            const int32_t* __restrict hl = hlen;
            const int64_t* __restrict ro = row_off.data();
            const int64_t* __restrict hw = hap_w.data();
            const uint8_t* __restrict hc = hcls;
            const Cand* __restrict cand = hcand;
            PairDesc* __restrict pdo = pd;
            uint8_t* __restrict clo = cls;
            uint8_t* __restrict bco = seg_bc;
            uint8_t* __restrict nbo = seg_nb;
            int64_t c = 0, cn0 = 0, cn1 = 0, cn2 = 0, cn3 = 0;
            int rlo = INT32_MAX, rhi = 0;
            auto one = [=, &c, &cn0, &cn1, &cn2, &cn3, &rlo, &rhi](int64_t k, int64_t r, int64_t h) {
                const int R = rl[r], H = hl[h];
                pdo[k] = PairDesc{int(ro[r]), R, int(hw[h]), H};
                c += int64_t(R) * H;
                const int cl = hc[h];
                clo[k] = uint8_t(cl);
                if (cl == 0) {
                    ++cn0;
                    const Cand cd = cand[h];
                    // modelled wave instructions: nb lanes x (13 per column + 26 per
                    // step) x (R + nb - 1) steps, times half the lane waste of a
                    // wave of such pairs alone (floor(64 / nb) groups): uniform
                    // batches pack like that, mixed ones fill the gaps with others;
                    // with few waves, the wave's own time (per lane)
                    auto cost = [&](int q) { return seg_cost(cd.nb[q], cd.bc[q], R, waste); };
                    const int q = qforce >= 0 ? qforce : cost(1) < cost(0) ? 1 : 0;
                    bco[k] = cd.bc[q];
                    nbo[k] = cd.nb[q];
                    rlo = R < rlo ? R : rlo;
                    rhi = R > rhi ? R : rhi;
                } else {
                    cn1 += cl == 1;
                    cn2 += cl == 2;
                    cn3 += cl == 3;
                }
            };
            if (spec.flat) {
                for (int64_t k = lo; k < hi; ++k) one(k, k, k);
            } else {
                loc.pairs(lo, hi, one);
            }
            cells_a += c;
            tcnt[size_t(t) + 1] = {cn0, cn1, cn2, cn3};
            int cur = rmin_a.load();
            while (rlo < cur && !rmin_a.compare_exchange_weak(cur, rlo)) {
            }
            cur = rmax_a.load();
            while (rhi > cur && !rmax_a.compare_exchange_weak(cur, rhi)) {
            }
        });
        // Stable split of the pairs by class (per-task offsets, parallel scatter).
        std::array<int64_t, 4> cls_tot{};
        for (int t = 1; t <= T; ++t)
            for (int q = 0; q < 4; ++q) {
                const int64_t v = tcnt[size_t(t)][size_t(q)];
                tcnt[size_t(t)][size_t(q)] = cls_tot[size_t(q)];
                cls_tot[size_t(q)] += v;
            }
        std::vector<int>& seg_in = S.seg_in;
        seg_in.resize(size_t(cls_tot[0]));
        one_ord.resize(size_t(cls_tot[1]));
        ord2[0].resize(size_t(cls_tot[2]));
        ord2[1].resize(size_t(cls_tot[3]));
        WorkerPool::get().run(T, [&](int t) {
            int* dst[4] = {seg_in.data(), one_ord.data(), ord2[0].data(), ord2[1].data()};
            int64_t pos[4];
            for (int q = 0; q < 4; ++q) pos[q] = tcnt[size_t(t) + 1][size_t(q)];
            for (int64_t k = t * pchunk, e = std::min(npairs, k + pchunk); k < e; ++k) {
                const int q = cls[size_t(k)];
                dst[q][pos[q]++] = int(k);
            }
        });
        tm.mark("pairs");
        if (!seg_in.empty()) {
            const int rlo = rmin_a.load(), rspan = rmax_a.load() - rlo + 1;
            const int nbk = (kSegMaxBC / 2 + 1) * rspan;
            if (nbk <= (1 << 18)) {
                counting_sort_desc(seg_in, S.sort_tmp, S.hist, nbk,
                                   [&](int p) { return (seg_bc[size_t(p)] / 2) * rspan + (pd[p].y - rlo); });
            } else {
                std::vector<uint32_t>& key = S.key;
                grow(key, size_t(npairs));
                for (int p : seg_in) key[size_t(p)] = (uint32_t(seg_bc[size_t(p)]) << 16) | uint32_t(std::min(pd[p].y, 65535));
                sort_desc(seg_in, key);
            }
        }
        tm.mark("seg sort");
        // Greedy packing in independent segments of the sorted list (one per task;
        // a segment boundary costs at most one partly filled wave).
        const int64_t ns = int64_t(seg_in.size());
        seg_ord.resize(size_t(ns));
        {
            const int T = int(std::min<int64_t>(64, std::max<int64_t>(1, ns / task_pairs)));
            const int64_t chunk = (ns + T - 1) / T;
            std::vector<std::vector<LaneWave>>& part_w = S.part_w;
            if (part_w.size() < size_t(T)) part_w.resize(size_t(T));
            for (auto& W : part_w) W.clear();
            S.used.assign(size_t(ns), 0);
            // The packing reads (BC, nb, R) of the pairs in sorted order: gather
            // them once into a sequential array (one parallel pass of random
            // reads, instead of three per look-ahead probe on one task per 16k
            // pairs: 0.3 ms of a 415 x 128 region's planning on the GPU box).
            std::vector<uint32_t>& srec = S.srec;
            grow(srec, size_t(ns));
            parallel_for(ns, [&](int64_t lo, int64_t hi) {
                for (int64_t k = lo; k < hi; ++k) {
                    const int p = seg_in[size_t(k)];
                    srec[size_t(k)] = uint32_t(seg_bc[size_t(p)]) | uint32_t(seg_nb[size_t(p)]) << 8 |
                                      uint32_t(std::min(pd[p].y, 65535)) << 16;
                }
            });
            // Smallest nb of each width in the part: a wave whose free lanes drop
            // below it cannot take another pair of its width, so its look-ahead
            // stops there (a uniform region once scanned all 64 entries per wave).
            std::array<uint8_t, kSegMaxBC + 1> minnb;
            minnb.fill(64);
            for (int64_t k = 0; k < ns; ++k) {
                uint8_t& m = minnb[srec[size_t(k)] & 0xff];
                m = std::min<uint8_t>(m, uint8_t(srec[size_t(k)] >> 8));
            }
            WorkerPool::get().run(T, [&](int t) {
                const int64_t b = t * chunk, e = std::min(ns, b + chunk);
                if (b >= e) return;
                const int64_t m = e - b;
                const int* __restrict in = seg_in.data() + b;
                const uint32_t* __restrict rec = srec.data() + b;
                int* __restrict ordo = seg_ord.data();
                uint8_t* __restrict used = S.used.data() + b;
                auto& W = part_w[size_t(t)];
                int64_t slot_n = b;
                constexpr int64_t kLook = 64;
                for (int64_t i = 0; i < m; ++i) {
                    if (used[i]) continue;
                    const int bc = int(rec[i] & 0xff);
                    LaneWave w{};
                    w.slot0 = int(slot_n);
                    w.ncols = bc;
                    int rmin = INT32_MAX, rmax = 0, nst = 0, np = 0;
                    int free = 64;
                    const int need = minnb[size_t(bc)];
                    const int64_t jend = std::min(m, i + kLook);
                    for (int64_t j = i; j < jend && free >= need; ++j) {
                        if (used[j]) continue;
                        const uint32_t r = rec[j];
                        if (int(r & 0xff) != bc) break;
                        const int nb = int((r >> 8) & 0xff);
                        if (nb > free) continue;
                        used[j] = 1;
                        free -= nb;
                        ordo[slot_n++] = in[j];
                        ++np;
                        const int R = int(r >> 16);
                        rmax = R > rmax ? R : rmax;
                        rmin = R < rmin ? R : rmin;
                        nst = R + nb - 1 > nst ? R + nb - 1 : nst;
                    }
                    w.npairs = np;
                    w.rmax = rmax;
                    w.rmin = rmin;
                    w.nsteps = nst;
                    W.push_back(w);
                }
            });
            size_t nw = 0;
            for (auto& W : part_w) nw += W.size();
            lw.reserve(nw);
            for (auto& W : part_w) lw.insert(lw.end(), W.begin(), W.end());
        }
    }
    tm.mark("seg pack: greedy");
    // Dispatch order: the bulk in packing order (co-resident waves share one
    // width's code), the shortest waves filling the last tail_rounds rounds of
    // wave slots last, longest first (LPT, duration ~ BC * nsteps), so the chip
    // drains evenly. Waves address their pairs through slot0: no pair moves.
    {
        // Structured (region) plans keep their order: their waves are in width
        // then read-length order already, and the reorder measured slower there
        // (415 x 128 region: fp32 0.937 -> 0.908 ms without it, call 1.43 -> 1.30 ms,
        // profiles/r02_region_dev_sweep.jsonl).
        const int64_t tail_rounds = std::max<int64_t>(0, env_i64("HC_PHMM_TAIL_ROUNDS", grid ? 0 : 2));
        const size_t nw = lw.size();
        const size_t K = std::min(nw, size_t(tail_rounds) * 4 * size_t(dv.n_cu) * kSegWavesPerSimd);
        std::vector<int64_t>& wc = S.wcost;
        wc.resize(nw);
        int64_t cmin = INT64_MAX, cmax = 0;
        for (size_t k = 0; k < nw; ++k) {
            wc[k] = int64_t(lw[k].ncols) * lw[k].nsteps;
            cmin = std::min(cmin, wc[k]);
            cmax = std::max(cmax, wc[k]);
        }
        // Waves of (nearly) equal length (one region's cross product) drain
        // evenly in any order: no reorder.
        if (K > 0 && K < nw && cmax * 20 > cmin * 21) {
            // Keys (cost, index) in one word each: the K shortest by one
            // nth_element, then those longest first, ties in packing order.
            std::vector<uint64_t>& key = S.wkey;
            key.resize(nw);
            for (size_t k = 0; k < nw; ++k) key[k] = uint64_t(wc[k]) << 32 | k;
            std::nth_element(key.begin(), key.begin() + long(K), key.end());
            for (size_t k = 0; k < K; ++k) key[k] = uint64_t(cmax - int64_t(key[k] >> 32)) << 32 | (key[k] & 0xffffffffu);
            std::sort(key.begin(), key.begin() + long(K));
            std::vector<uint8_t>& in_tail = S.in_tail;
            in_tail.assign(nw, 0);
            for (size_t k = 0; k < K; ++k) in_tail[key[k] & 0xffffffffu] = 1;
            std::vector<LaneWave>& ordered = S.ordered;
            ordered.clear();
            ordered.reserve(nw);
            for (size_t k = 0; k < nw; ++k)
                if (!in_tail[k]) ordered.push_back(lw[k]);
            for (size_t k = 0; k < K; ++k) ordered.push_back(lw[key[k] & 0xffffffffu]);
            lw.swap(ordered);
        }
        // (A snake order over the SIMDs for one-round plans, heaviest wave
        // beside the lightest, cut S4's busiest-SIMD modelled sum from 1.30x
        // the mean to 1.10x but not the pass, 0.278 vs 0.274 ms: two waves of
        // this pass on one SIMD are latency-bound. Removed)
    }
    tm.mark("seg pack");
    const int n_seg_waves = dev_plan ? int(gd.waves) : int(lw.size());
    const int n_seg_slots = dev_plan ? int(gd.slots) : int(seg_ord.size());
    // One lane per pair with the carry buffer (haps longer than the segmented
    // kernel's reach, or policy "off"): binned by (H rounded up to 16, R).
    const int lane_var = lane_variant_id();
    const LaneVariant& LV = lane_variant(lane_var);
    int64_t carry_rows = 0;
    {
        std::vector<uint32_t>& key = S.key;
        grow(key, size_t(npairs));
        auto cols16 = [&](int p) { return (pd[p].w + 15) / 16 * 16; };
        for (int p : one_ord) key[size_t(p)] = (uint32_t(cols16(p)) << 16) | uint32_t(std::min(pd[p].y, 65535));
        sort_desc(one_ord, key);
        const size_t per_wave = size_t(64) * LV.P;
        for (size_t s0 = 0; s0 < one_ord.size(); s0 += per_wave) {
            LaneWave w{};
            w.slot0 = n_seg_slots + int(s0);
            w.rmin = INT32_MAX;
            for (size_t k = s0; k < std::min(one_ord.size(), s0 + per_wave); ++k) {
                const int p = one_ord[k];
                w.rmax = std::max(w.rmax, pd[p].y);
                w.rmin = std::min(w.rmin, pd[p].y);
                w.ncols = std::max(w.ncols, cols16(p));
            }
            w.carry_row = carry_rows;
            if (w.ncols > LV.BC) carry_rows += w.rmax + 1;
            lw.push_back(w);
        }
        // Anti-diagonal classes: W by H; (stripes, H) descending so the G pairs
        // sharing a wave have equal stripe counts and similar H, heaviest first.
        const int Wc[2] = {16, 64};
        for (int c = 0; c < 2; ++c) {
            for (int p : ord2[c]) key[size_t(p)] = (uint32_t((pd[p].y + Wc[c] - 1) / Wc[c]) << 16) | uint32_t(pd[p].w);
            sort_desc(ord2[c], key);
        }
    }
    tm.mark("one-lane/diag bins");

    // Staging fill: order, wave list, read descriptors + bytes, hap bytes.
    int* ordp = reinterpret_cast<int*>(host + o_ord);
    std::memcpy(ordp, seg_ord.data(), sizeof(int) * seg_ord.size());
    std::memcpy(ordp + n_seg_slots, one_ord.data(), sizeof(int) * one_ord.size());
    const size_t o_ord0 = size_t(n_seg_slots) + one_ord.size();
    std::memcpy(ordp + o_ord0, ord2[0].data(), sizeof(int) * ord2[0].size());
    std::memcpy(ordp + o_ord0 + ord2[0].size(), ord2[1].data(), sizeof(int) * ord2[1].size());
    if (!dev_plan) {   // structured plans build it on the device (grid_waves)
        int* so = reinterpret_cast<int*>(host + o_slotof);
        parallel_for(npairs, [&](int64_t lo, int64_t hi) { std::fill(so + lo, so + hi, -1); }, 1 << 16);
        parallel_for(int64_t(seg_ord.size()), [&](int64_t lo, int64_t hi) {
            for (int64_t k = lo; k < hi; ++k) so[seg_ord[size_t(k)]] = int(k);
        }, 1 << 16);
    }
    std::memcpy(host + o_lw, lw.data(), sizeof(LaneWave) * lw.size());
    size_t upload = o_lw + sizeof(LaneWave) * (dev_plan ? size_t(n_seg_waves) : lw.size());
    // Structured plans: the pair descriptors, the slot order and the waves are
    // built on the device (launch_grid_pairs, launch_grid_waves), so the upload
    // skips them and carries the block and segment tables instead.
    const bool dev_pairs = dev_plan;
    const size_t up0 = dev_pairs ? o_rd : 0;
    const size_t up_mid = dev_plan ? o_ord : upload;   // [up0, up_mid) and [o_gb, upload) travel
    size_t o_gb = 0, o_gs = 0, o_gr = 0, o_gh = 0;
    if (dev_pairs) {
        o_gb = (upload + 15) & ~size_t(15);
        GridBlock* gb = reinterpret_cast<GridBlock*>(host + o_gb);
        for (size_t b = 0; b < spec.blocks.size(); ++b)
            gb[b] = GridBlock{loc.blk_p[b], spec.blocks[b].nr, spec.blocks[b].nh, int(loc.blk_r[b]), int(loc.blk_h[b])};
        o_gs = (o_gb + sizeof(GridBlock) * spec.blocks.size() + 15) & ~size_t(15);
        std::memcpy(host + o_gs, gd.segs.data(), sizeof(GridSeg) * gd.segs.size());
        o_gr = (o_gs + sizeof(GridSeg) * gd.segs.size() + 15) & ~size_t(15);
        std::memcpy(host + o_gr, gd.rord.data(), sizeof(int) * gd.rord.size());
        o_gh = (o_gr + sizeof(int) * gd.rord.size() + 15) & ~size_t(15);
        std::memcpy(host + o_gh, gd.hord.data(), sizeof(int) * gd.hord.size());
        upload = o_gh + sizeof(int) * gd.hord.size();
    }
    // Reads (haps) per staging task: a region's few hundred reads go on this
    // thread alone below HC_PHMM_FILL_GRAIN (a pool wake-up cost about what
    // the packing of 415 reads does).
    const int64_t fill_grain = std::max<int64_t>(1, env_i64("HC_PHMM_FILL_GRAIN", 256));
    int4* rdesc = reinterpret_cast<int4*>(host + o_rd);
    uint8_t* hb = reinterpret_cast<uint8_t*>(host + o_bases);
    uint8_t* hq = reinterpret_cast<uint8_t*>(host + o_quals);
    uint8_t* hg = reinterpret_cast<uint8_t*>(host + o_gaps);
    parallel_for(nr, [&](int64_t b, int64_t e) {
        for (int64_t r = b; r < e; ++r) {
            const ReadView v = src.read(loc.read_id(r));
            const size_t o = size_t(row_off[size_t(r)]);
            pack_nibbles(v.bases, v.len, hb + o / 2);
            std::memcpy(hq + o, v.q, size_t(v.len));
            const int32_t g = gapw[size_t(r)];
            int go = 0;
            if (g < 0) {
                go = int(gap_off[size_t(r)]);
                std::memcpy(hg + go, v.i, size_t(v.len));
                std::memcpy(hg + gap_stride + size_t(go), v.d, size_t(v.len));
                std::memcpy(hg + 2 * gap_stride + size_t(go), v.c, size_t(v.len));
            }
            rdesc[r] = make_int4(int(o), v.len, g, go);
        }
    }, fill_grain);
    int4* hdesc = reinterpret_cast<int4*>(host + o_hd);
    uint8_t* hbytes = reinterpret_cast<uint8_t*>(host + o_hb);
    parallel_for(nh, [&](int64_t b, int64_t e) {
        for (int64_t h = b; h < e; ++h) {
            const HapView v = src.hapv(loc.hap_id(h));
            pack_nibbles(v.bases, v.len, hbytes + hap_b[size_t(h)]);
            hdesc[h] = make_int4(int(hap_b[size_t(h)]), v.len, int(hap_w[size_t(h)]), 0);
        }
    }, fill_grain);
    tm.mark("staging fill");
    if (dry) {
        // Dry runs keep the last part's plan for the host-logic tests
        // (hcx_dump_*): pair descriptors, slot order, segmented waves.
        std::lock_guard<std::mutex> lk(g_dump.mu);
        g_dump.pairs.assign(pd, pd + npairs);
        g_dump.order.assign(seg_ord.begin(), seg_ord.end());
        g_dump.order.insert(g_dump.order.end(), one_ord.begin(), one_ord.end());
        g_dump.waves.assign(lw.begin(), lw.begin() + n_seg_waves);
        g_dump.n_seg_slots = n_seg_slots;
        g_dump.grid = grid;
        *out = nullptr;
        return HC_PHMM_OK;
    }

    // Device region: the upload image, then packed rows / tables, outputs, scratch.
    Layout L;
    L.off = (upload + 255) & ~size_t(255);
    // Packed rows with slack on both sides: the segmented kernels prefetch
    // read words PD steps ahead without clamping to the read (run_seg), so a
    // lane in pipeline fill reads up to 64 words before its read and a pair
    // shorter than its wave's longest read up to that length + 64 past it;
    // those words only feed rows that are never used.
    const size_t row_pad = kRowPadBefore + size_t(rlen_max.load()) + 256;
    if (int64_t(nrows) + int64_t(row_pad) > kMaxRowWords)
        return fail(HC_PHMM_EINVAL, "batch too large (read bases of one part exceed 2^30)");
    if (int64_t(hap_w[size_t(nh)]) + 16 > kMaxHapWords)
        return fail(HC_PHMM_EINVAL, "batch too large (hap match tables of one part exceed 2^30 words)");
    const size_t o_rows = L.take(sizeof(uint32_t) * (size_t(nrows) + row_pad));
    const size_t o_hapw = L.take(sizeof(uint32_t) * (size_t(hap_w[size_t(nh)]) + 16));
    const size_t o_res = L.take(res_bytes);
    const size_t o_rec = L.take(sizeof(uint4) * std::max<size_t>(size_t(n_seg_slots), 1));   // seg slot records
    const size_t o_sdesc = L.take(sizeof(PairDesc) * std::max<size_t>(size_t(n_seg_slots), 1));   // slot -> descriptor
    const size_t o_list = L.take(2 * sizeof(int) * n1);   // pair ids, then pack_rh (Seg64Args::list_rh)
    const size_t o_sorted = L.take(sizeof(int) * n1);
    const size_t o_worder = L.take(sizeof(int) * n1);
    const size_t o_big = L.take(sizeof(int) * n1);
    const size_t o_bigc = L.take(sizeof(int));
    const size_t o_plan = L.take(sizeof(Seg64Plan));
    const size_t o_carry = L.take(sizeof(float2) * size_t(carry_rows) * 64 * LV.P);
    // Anti-diagonal stripe rings too long for the LDS (kernels.hpp
    // diag_ring_in_lds) live in global memory, one slice per workgroup; the
    // fp32 classes and the fp64 wide-hap pass run one after another and share it.
    const int Wc[2] = {16, 64};
    int cls_ring[2] = {0, 0};
    size_t ring_bytes = 0;
    for (int c = 0; c < 2; ++c) {
        int hm = 0;
        for (int p : ord2[c]) hm = std::max(hm, pd[p].w);
        cls_ring[c] = hm + 2 * Wc[c] + 16;
        if (!ord2[c].empty() && !diag_ring_in_lds(Wc[c], cls_ring[c], false)) {
            const size_t G = size_t(64 / Wc[c]);
            const size_t blocks = std::min<size_t>((ord2[c].size() + G - 1) / G, kDiagRingBlocks);
            ring_bytes = std::max(ring_bytes, blocks * G * size_t(cls_ring[c]) * sizeof(float2));
        }
    }
    const int Hmax = hmax_a.load();
    // The fp64 wide pass runs only for rescued wide pairs (usually none or a
    // few), so its global ring is sized for kWideRing64Blocks workgroups (each
    // loops over its share of the list), not for every wide pair: a call with
    // a thousand 262k-base haps would otherwise reserve ~4 GB, kept by its slot
    // (advisor round 3).
    int wide_ring_blocks = 0;
    if (wide_a.load() > 0 && !diag_ring_in_lds(64, Hmax + 2 * 64 + 16, true)) {
        wide_ring_blocks = int(std::min<int64_t>(wide_a.load(), kWideRing64Blocks));
        ring_bytes = std::max(ring_bytes, size_t(wide_ring_blocks) * size_t(Hmax + 2 * 64 + 16) * 2 * sizeof(double));
    }
    const size_t o_ring = L.take(ring_bytes);
    const size_t total = L.off;

    auto* b = new_part(&dv);
    PartGuard guard(b);   // error returns and exceptions discard it (the caller returns the slot)
    b->slot = slot;
    b->spec = spec;
    char* dev = nullptr;
    int rc = HC_PHMM_OK;
    if (slot) {
        rc = slot_reserve(*slot, total, 0);
        dev = slot->dev;
    } else if (hipMalloc(&dev, total) != hipSuccess) {
        rc = fail(HC_PHMM_ENOMEM, "device allocation failed (" + std::to_string(total >> 20) + " MiB)");
    }
    if (rc) return rc;
    b->dev_base = dev;
    b->n = npairs;
    b->cells = cells_a.load();
    b->Hmax = Hmax;
    b->n_lane = int(size_t(n_seg_slots) + one_ord.size());
    b->n_seg_waves = n_seg_waves;
    b->lane_variant = lane_var;
    b->lane_waves = dev_plan ? n_seg_waves : int(lw.size());
    b->upload_bytes = dev_pairs ? (up_mid - up0) + (o_lw - o_bases) + (upload - o_gb) : upload - up0;
    b->d_pairs = reinterpret_cast<PairDesc*>(dev + o_pairs);
    b->d_rows = reinterpret_cast<uint32_t*>(dev + o_rows) + kRowPadBefore;
    b->d_hapw = reinterpret_cast<uint32_t*>(dev + o_hapw);
    int* d_ord = reinterpret_cast<int*>(dev + o_ord);
    b->d_lane_order = d_ord;
    b->cls[0].d_order = d_ord + o_ord0;
    b->cls[1].d_order = d_ord + o_ord0 + ord2[0].size();
    for (int c = 0; c < 2; ++c) {
        b->cls[c].W = Wc[c];
        b->cls[c].n = int(ord2[c].size());
        b->cls[c].ring_len = cls_ring[c];
    }
    b->d_ring = ring_bytes ? dev + o_ring : nullptr;
    b->d_lane_waves = reinterpret_cast<LaneWave*>(dev + o_lw);
    b->res_bytes = res_bytes;
    b->res_o64 = RL.o64;
    b->res_ofl = RL.ofl;
    b->res_ocnt = RL.ocnt;
    b->own_raw32 = b->d_raw32 = reinterpret_cast<float*>(dev + o_res);
    b->own_raw64 = b->d_raw64 = reinterpret_cast<double*>(dev + o_res + RL.o64);
    b->own_flag = b->d_flag = reinterpret_cast<uint8_t*>(dev + o_res + RL.ofl);
    b->d_list = reinterpret_cast<int*>(dev + o_list);
    b->d_count = reinterpret_cast<int*>(dev + o_res + RL.ocnt);   // run counters (kNumCounters): the results block's tail
    b->d_sorted = reinterpret_cast<int*>(dev + o_sorted);
    b->d_worder = reinterpret_cast<int*>(dev + o_worder);
    b->d_big = reinterpret_cast<int*>(dev + o_big);
    b->d_big_count = reinterpret_cast<int*>(dev + o_bigc);
    b->d_plan = reinterpret_cast<Seg64Plan*>(dev + o_plan);
    b->d_rec = n_seg_slots > 0 ? reinterpret_cast<uint4*>(dev + o_rec) : nullptr;
    b->d_slot_of = reinterpret_cast<int*>(dev + o_slotof);
    b->d_sdesc = reinterpret_cast<PairDesc*>(dev + o_sdesc);
    b->n_wide = wide_a.load();
    b->wide_ring_blocks = wide_ring_blocks;
    b->d_carry = carry_rows ? reinterpret_cast<float2*>(dev + o_carry) : nullptr;
    if (slot) b->host_res = host + host_res_off;

    if (slot) {
        b->stream = slot->stream;
        b->side = slot->side;
        b->fork = slot->fork;
        b->join = slot->join;
        b->slot_ev = true;
        b->pack_ev[0] = slot->ev[0];
        b->pack_ev[1] = slot->ev[1];
        b->ev_pool.push_back({slot->ev[2], slot->ev[3], slot->ev[4]});
        b->done = slot->ev[5];
        b->early = slot->ev[6];
    } else {
        b->stream = dv.stream;
        b->side = dv.side;
        b->fork = dv.fork;
        b->join = dv.join;
    }
    hipStream_t s = b->stream;
    PackArgs pack{};
    pack.bases = reinterpret_cast<const uint8_t*>(dev + o_bases);
    pack.quals = reinterpret_cast<const uint8_t*>(dev + o_quals);
    pack.gaps = reinterpret_cast<const uint8_t*>(dev + o_gaps);
    pack.gap_stride = (long long)gap_stride;
    pack.rdesc = reinterpret_cast<const int4*>(dev + o_rd);
    pack.nreads = int(nr);
    pack.rows = b->d_rows;
    pack.hap_bytes = reinterpret_cast<const uint8_t*>(dev + o_hb);
    pack.hdesc = reinterpret_cast<const int4*>(dev + o_hd);
    pack.nhaps = int(nh);
    pack.hapw = b->d_hapw;
    pack.pairs = b->d_pairs;
    pack.order = d_ord;
    pack.nslots = dev_pairs ? 0 : n_seg_slots;   // structured plans: grid_waves writes them
    pack.sdesc = b->d_sdesc;
    auto enqueue = [&]() -> int {
        if (!b->slot_ev)
            for (auto& e : b->pack_ev) HIP_TRY(hipEventCreate(&e));
        if (dev_pairs) {
            // [o_rd, o_ord): read / hap descriptors; the order and waves between
            // are built on the device; then the read / hap bytes and the block
            // and segment tables. One fused launch prepares everything.
            // Zero copy (a part whose upload is at most HC_PHMM_ZERO_COPY_MAX
            // bytes, default 4 MiB: one region): the prep launch reads the
            // pinned staging image itself over PCIe — it is the only reader of
            // those bytes — instead of three DMA copies ahead of it.
            char* src = dev;
            const int64_t up_bytes = int64_t(up_mid - up0) + int64_t(o_lw - o_bases) + int64_t(upload - o_gb);
            if (slot && up_bytes <= env_i64("HC_PHMM_ZERO_COPY_MAX", int64_t(4) << 20)) {
                void* hp = nullptr;
                if (hipHostGetDevicePointer(&hp, host, 0) == hipSuccess && hp) src = static_cast<char*>(hp);
            }
            if (src == dev) {
                HIP_TRY(hipMemcpyAsync(dev + up0, host + up0, up_mid - up0, hipMemcpyHostToDevice, s));
                HIP_TRY(hipMemcpyAsync(dev + o_bases, host + o_bases, o_lw - o_bases, hipMemcpyHostToDevice, s));
                HIP_TRY(hipMemcpyAsync(dev + o_gb, host + o_gb, upload - o_gb, hipMemcpyHostToDevice, s));
            } else {
                pack.bases = reinterpret_cast<const uint8_t*>(src + o_bases);
                pack.quals = reinterpret_cast<const uint8_t*>(src + o_quals);
                pack.gaps = reinterpret_cast<const uint8_t*>(src + o_gaps);
                pack.rdesc = reinterpret_cast<const int4*>(src + o_rd);
                pack.hap_bytes = reinterpret_cast<const uint8_t*>(src + o_hb);
                pack.hdesc = reinterpret_cast<const int4*>(src + o_hd);
            }
            HIP_TRY(hipEventRecord(b->pack_ev[0], s));
            GridPrepArgs g{};
            g.pack = pack;
            g.blocks = reinterpret_cast<const GridBlock*>(src + o_gb);
            g.nblocks = int(spec.blocks.size());
            g.npairs = (long long)npairs;
            g.pairs = b->d_pairs;
            g.segs = reinterpret_cast<const GridSeg*>(src + o_gs);
            g.nsegs = int(gd.segs.size());
            g.nslots = (long long)n_seg_slots;
            g.nwaves = n_seg_waves;
            g.rord = reinterpret_cast<const int*>(src + o_gr);
            g.hord = reinterpret_cast<const int*>(src + o_gh);
            g.order = reinterpret_cast<int*>(dev + o_ord);
            g.slot_of = b->d_slot_of;
            g.sdesc = b->d_sdesc;
            g.waves = reinterpret_cast<LaneWave*>(dev + o_lw);
            g.counters = b->d_count;
            HIP_TRY(launch_prepare_grid(g, s));
            HIP_TRY(hipEventRecord(b->pack_ev[1], s));
        } else {
            HIP_TRY(hipMemcpyAsync(dev + up0, host + up0, upload - up0, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemsetAsync(b->d_count, 0, kNumCounters * sizeof(int), s));
            HIP_TRY(hipEventRecord(b->pack_ev[0], s));
            HIP_TRY(launch_pack_batch(pack, s));
            HIP_TRY(hipEventRecord(b->pack_ev[1], s));
        }
        if (with_run) {
            const int r = run_part(b, s);
            if (r) return r;
            const int e = enqueue_results(b, s);
            if (e) return e;
        }
        // A part-owned staging buffer is freed on return: the copy must be done.
        if (own_host) HIP_TRY(hipStreamSynchronize(s));
        return HC_PHMM_OK;
    };
    rc = enqueue();
    tm.mark("enqueue");
    if (rc) return rc;   // the guard drains the stream and discards the part
    *out = guard.release();
    return HC_PHMM_OK;
}

}  // namespace eng
}  // namespace hcphmm
