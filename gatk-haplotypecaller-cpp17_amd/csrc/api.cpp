// Splitting calls into parts over the device slots, the asynchronous submit /
// collect machinery, and the C ABI of libhcpairhmm.so (include/hc_pairhmm.h):
// the drop-in for IntelPairHMM::compute_likelihoods (intel_pairhmm.hpp:48-56)
// and the reference's own accelerator slot shacc_pairhmm::calculate
// (pairhmm/native/shacc_pairhmm.h:10-36).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <new>

#include "engine_core.hpp"
#include "luts.hpp"
#include "pool.hpp"

namespace hcphmm {
namespace eng {
const char* last_error();
int timeline_records(unsigned long long* out, int max_waves);
int shutdown_engine();
}  // namespace eng
}  // namespace hcphmm

using namespace hcphmm;
using namespace hcphmm::eng;

namespace {

// ---------------------------------------------------------------------------
// Splitting a call into parts.

// Cut a sequence of units with weights into `nparts` contiguous ranges of
// (nearly) equal weight: returns nparts + 1 boundaries.
std::vector<int64_t> equal_cuts(const std::vector<int64_t>& prefix, int nparts)
{
    const int64_t n = int64_t(prefix.size()) - 1;
    const int64_t tot = prefix.back();
    std::vector<int64_t> cut(static_cast<size_t>(nparts) + 1, 0);
    cut[size_t(nparts)] = n;
    for (int j = 1; j < nparts; ++j) {
        const int64_t target = (tot * j + nparts / 2) / nparts;
        int64_t c = int64_t(std::lower_bound(prefix.begin(), prefix.end(), target) - prefix.begin());
        // the nearer of the boundaries either side of the target (two halves of
        // a region just under half each must not both land in the first part)
        if (c > 0 && c <= n && target - prefix[size_t(c) - 1] < prefix[size_t(c)] - target) --c;
        cut[size_t(j)] = std::max(cut[size_t(j) - 1], std::min(n, c));
    }
    return cut;
}

// How many parts for `cells` over the configured devices: one part below
// HC_PHMM_SHARD_MIN_CELLS; above, per device at least HC_PHMM_MIN_CHUNKS (1)
// and about one per HC_PHMM_CHUNK_CELLS, so the planning of part k + 1
// overlaps the device pass of part k (the parts of one device run on their
// slots' streams, concurrently). One 415 x 128 region (3.3e9 cells) stays
// whole: cut in 2 / 3 / 4 parts it took 2.23 / 1.99 / 1.84 ms vs 1.89 ms
// (tools/region_ab.py; each part pays its own planning fixed costs and fp64
// pass).
int part_count(int64_t cells, int ndev)
{
    const int64_t shard_min = env_i64("HC_PHMM_SHARD_MIN_CELLS", int64_t(2000000000));
    const int64_t chunk = std::max<int64_t>(1, env_i64("HC_PHMM_CHUNK_CELLS", int64_t(12000000000)));
    const int64_t min_chunks = std::max<int64_t>(1, env_i64("HC_PHMM_MIN_CHUNKS", 1));
    if (cells < shard_min) return 1;
    const int64_t per_dev = (cells + ndev - 1) / ndev;
    const int64_t chunks = std::max<int64_t>(min_chunks, (per_dev + chunk / 2) / chunk);
    return int(std::min<int64_t>(int64_t(ndev) * chunks, 4096));
}

Device* least_loaded(const std::vector<Device*>& devs)
{
    std::lock_guard<std::mutex> lk(g_mu);
    Device* best = devs[0];
    for (Device* d : devs)
        if (d->outstanding < best->outstanding) best = d;
    return best;
}

// Plan one part of a call on device d: flat parts are planned on the device
// when their pairs allow it (flat_plan.cpp), everything else on the host.
int plan_call_part(Device& d, const Src& src, const PartSpec& spec, Slot* sl, bool with_run, Part** p)
{
    *p = nullptr;
    if (spec.flat) {
        const int rc = plan_flat_device(d, src, spec, sl, with_run, p);
        if (rc || *p) return rc;
    }
    return plan_part(d, src, spec, sl, with_run, PlanMode::Real, p);
}

// Prepared batches keep the host planner unless HC_PHMM_BATCH_PLAN=device:
// the plan is made once and run many times, and its mixed-width greedy
// packing fills the waves best.
int plan_batch_part(Device& d, const Src& src, const PartSpec& spec, Part** p)
{
    *p = nullptr;
    const char* e = std::getenv("HC_PHMM_BATCH_PLAN");
    if (e && !std::strcmp(e, "device")) {
        const int rc = plan_flat_device(d, src, spec, nullptr, false, p);
        if (rc || *p) return rc;
    }
    return plan_part(d, src, spec, nullptr, false, PlanMode::Real, p);
}

// Plan + enqueue every part of a call (device of part j = j mod #devices, or
// the least loaded device for a one-part call); returns the job.
int submit(const std::vector<Device*>& devs, const Src& src, const std::vector<PartSpec>& specs,
           const std::vector<double>& part_cells, const Outputs& out, hc_phmm_job** job)
{
    auto* J = new hc_phmm_job();
    J->out = out;
    const size_t G = devs.size();
    if (std::getenv("HC_PHMM_TRACE")) std::fprintf(stderr, "[hc_phmm] submit: %zu part(s)\n", specs.size());
    Device* solo = specs.size() == 1 ? least_loaded(devs) : nullptr;
    for (size_t j = 0; j < specs.size(); ++j) {
        Device& d = solo ? *solo : *devs[j % G];
        int rc = hipSetDevice(d.ordinal) == hipSuccess ? HC_PHMM_OK : fail(HC_PHMM_EHIP, "hipSetDevice");
        Slot* sl = rc ? nullptr : take_slot(d);
        if (!rc && !sl) rc = HC_PHMM_EHIP;
        Part* p = nullptr;
        if (!rc) rc = plan_call_part(d, src, specs[j], sl, true, &p);
        if (rc) {
            if (sl && !p) give_slot(sl);
            for (size_t k = 0; k < J->parts.size(); ++k) {
                Part* q = J->parts[k];
                (void)hipSetDevice(q->dev->ordinal);
                (void)hipStreamSynchronize(q->stream);
                {
                    std::lock_guard<std::mutex> lk(g_mu);
                    q->dev->outstanding -= J->cells_per_part[k];
                }
                free_part(q);
            }
            delete J;
            return rc;
        }
        {
            std::lock_guard<std::mutex> lk(g_mu);
            d.outstanding += part_cells[j];
        }
        J->parts.push_back(p);
        J->cells_per_part.push_back(part_cells[j]);
    }
    *job = J;
    return HC_PHMM_OK;
}

int collect(hc_phmm_job* J)
{
    int rc = HC_PHMM_OK;
    PhaseTimer tm;
    for (size_t j = 0; j < J->parts.size(); ++j) {
        Part* p = J->parts[j];
        if (rc == HC_PHMM_OK) {
            (void)hipSetDevice(p->dev->ordinal);
            const hipError_t e = hipEventSynchronize(p->done);
            if (e != hipSuccess) {
                rc = fail(HC_PHMM_EHIP, std::string("device pass: ") + hipGetErrorString(e));
            } else {
                tm.mark("collect: wait");
                if (tm.on) {
                    float a = 0, f32 = 0, f64 = 0;
                    (void)hipEventElapsedTime(&a, p->pack_ev[0], p->pack_ev[1]);
                    (void)hipEventElapsedTime(&f32, p->ev[0], p->ev[1]);
                    (void)hipEventElapsedTime(&f64, p->ev[1], p->ev[2]);
                    std::fprintf(stderr, "[hc_phmm]   device: pack %.3f ms, fp32 %.3f ms, fp64 %.3f ms (%lld pairs)\n", a,
                                 f32, f64, (long long)p->n);
                }
                const char* h = p->host_res;
                finish_part(*p, reinterpret_cast<const float*>(h), reinterpret_cast<const double*>(h + p->res_o64),
                            reinterpret_cast<const uint8_t*>(h + p->res_ofl), J->out);
                tm.mark("collect: finish");
            }
        } else {
            (void)hipSetDevice(p->dev->ordinal);
            (void)hipEventSynchronize(p->done);
        }
        {
            std::lock_guard<std::mutex> lk(g_mu);
            p->dev->outstanding -= J->cells_per_part[j];
        }
        free_part(p);
    }
    delete J;
    return rc;
}

// Flat pairs [0, n): cut into parts of equal cells.
int submit_flat(const std::vector<Device*>& devs, const Src& src, int64_t n, const Outputs& out, hc_phmm_job** job)
{
    std::vector<int64_t> pre;
    prefix_sum(n, pre, [&](int64_t p) { return int64_t(src.R[p] > 0 ? src.R[p] : 0) * (src.H[p] > 0 ? src.H[p] : 0); });
    const int np = part_count(pre.back(), int(devs.size()));
    const std::vector<int64_t> cut = equal_cuts(pre, np);
    std::vector<PartSpec> specs;
    std::vector<double> pc;
    for (int j = 0; j < np; ++j) {
        if (cut[size_t(j)] == cut[size_t(j) + 1] && np > 1) continue;
        PartSpec s;
        s.flat = true;
        s.lo = cut[size_t(j)];
        s.hi = cut[size_t(j) + 1];
        specs.push_back(s);
        pc.push_back(double(pre[size_t(s.hi)] - pre[size_t(s.lo)]));
    }
    return submit(devs, src, specs, pc, out, job);
}

// Cross-product blocks (regions): a block larger than one part's share is cut
// into read ranges; then contiguous runs of blocks form parts of equal cells.
int submit_blocks(const std::vector<Device*>& devs, const Src& src, std::vector<Block> blocks, hc_phmm_job** job)
{
    int64_t cells = 0;
    std::vector<int64_t> bc(blocks.size());
    for (size_t k = 0; k < blocks.size(); ++k) {
        int64_t rl = 0, hl = 0;
        for (int32_t r = 0; r < blocks[k].nr; ++r) rl += std::max(0, src.read_len(blocks[k].r0 + r));
        for (int32_t h = 0; h < blocks[k].nh; ++h) hl += std::max(0, src.hap_len(blocks[k].h0 + h));
        bc[k] = rl * hl;
        cells += bc[k];
    }
    const int np = part_count(cells, int(devs.size()));
    if (np > 1) {
        const int64_t share = (cells + np - 1) / np;
        std::vector<Block> split;
        for (size_t k = 0; k < blocks.size(); ++k) {
            const Block& B = blocks[k];
            const int pieces = int(std::min<int64_t>(B.nr, (bc[k] + share - 1) / std::max<int64_t>(share, 1)));
            if (pieces <= 1) {
                split.push_back(B);
                continue;
            }
            for (int q = 0; q < pieces; ++q) {
                const int32_t a = int32_t(int64_t(B.nr) * q / pieces), e = int32_t(int64_t(B.nr) * (q + 1) / pieces);
                if (a == e) continue;
                split.push_back(Block{B.r0 + a, e - a, B.h0, B.nh, B.out + int64_t(a) * B.ostride, B.ostride});
            }
        }
        blocks.swap(split);
    }
    std::vector<int64_t> pre(blocks.size() + 1, 0);
    for (size_t k = 0; k < blocks.size(); ++k) {
        int64_t rl = 0, hl = 0;
        for (int32_t r = 0; r < blocks[k].nr; ++r) rl += std::max(0, src.read_len(blocks[k].r0 + r));
        for (int32_t h = 0; h < blocks[k].nh; ++h) hl += std::max(0, src.hap_len(blocks[k].h0 + h));
        pre[k + 1] = pre[k] + rl * hl;
    }
    const int nparts = std::max(1, std::min<int>(np, int(blocks.size())));
    const std::vector<int64_t> cut = equal_cuts(pre, nparts);
    std::vector<PartSpec> specs;
    std::vector<double> pc;
    for (int j = 0; j < nparts; ++j) {
        if (cut[size_t(j)] == cut[size_t(j) + 1]) continue;
        PartSpec s;
        s.flat = false;
        s.blocks.assign(blocks.begin() + long(cut[size_t(j)]), blocks.begin() + long(cut[size_t(j) + 1]));
        specs.push_back(std::move(s));
        pc.push_back(double(pre[size_t(cut[size_t(j) + 1])] - pre[size_t(cut[size_t(j)])]));
    }
    if (specs.empty()) {
        *job = new hc_phmm_job();
        return HC_PHMM_OK;
    }
    return submit(devs, src, specs, pc, Outputs{}, job);
}

Src flat_src(const int64_t* read_off, const int32_t* R, const int64_t* hap_off, const int32_t* H, const uint8_t* rs,
             const uint8_t* q, const uint8_t* ins, const uint8_t* del, const uint8_t* gcp, const uint8_t* hap)
{
    Src s;
    s.read_off = read_off;
    s.R = R;
    s.hap_off = hap_off;
    s.H = H;
    s.rs = rs;
    s.q = q;
    s.ins = ins;
    s.del = del;
    s.gcp = gcp;
    s.hap = hap;
    return s;
}

bool flat_args_ok(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off, const int32_t* H,
                  const uint8_t* rs, const uint8_t* q, const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
                  const uint8_t* hap)
{
    return n == 0 || (read_off && R && hap_off && H && rs && q && ins && del && gcp && hap);
}

// Regions -> one Src over concatenated read / hap structs + one block per region.
struct RegionSet {
    std::vector<hc_phmm_read> reads;
    std::vector<hc_phmm_hap> haps;
    std::vector<Block> blocks;
};

int gather_regions(const hc_phmm_region* regions, int32_t n_regions, RegionSet& rs)
{
    if (n_regions < 0 || (n_regions > 0 && !regions)) return fail(HC_PHMM_EINVAL, "bad region list");
    size_t tr = 0, th = 0;
    for (int k = 0; k < n_regions; ++k) {
        const hc_phmm_region& g = regions[k];
        if (g.n_reads < 0 || g.n_haps < 0) return fail(HC_PHMM_EINVAL, "negative count in region");
        if (g.n_reads == 0 || g.n_haps == 0) continue;
        if (!g.reads || !g.haps || !g.out) return fail(HC_PHMM_EINVAL, "null pointer in region");
        tr += size_t(g.n_reads);
        th += size_t(g.n_haps);
    }
    rs.reads.resize(tr);
    rs.haps.resize(th);
    size_t r0 = 0, h0 = 0;
    for (int k = 0; k < n_regions; ++k) {
        const hc_phmm_region& g = regions[k];
        if (g.n_reads == 0 || g.n_haps == 0) continue;
        std::memcpy(rs.reads.data() + r0, g.reads, sizeof(hc_phmm_read) * size_t(g.n_reads));
        std::memcpy(rs.haps.data() + h0, g.haps, sizeof(hc_phmm_hap) * size_t(g.n_haps));
        rs.blocks.push_back(Block{int64_t(r0), g.n_reads, int64_t(h0), g.n_haps, g.out, g.n_haps});
        r0 += size_t(g.n_reads);
        h0 += size_t(g.n_haps);
    }
    return HC_PHMM_OK;
}

}  // namespace

// C ABI entry points never let a C++ exception cross the boundary (a planner
// allocation failing with std::bad_alloc becomes HC_PHMM_ENOMEM).
#define HC_API_TRY try {
#define HC_API_CATCH                                                              \
    }                                                                             \
    catch (const std::bad_alloc&) { return fail(HC_PHMM_ENOMEM, "host allocation failed"); } \
    catch (const std::exception& e_) { return fail(HC_PHMM_EHIP, e_.what()); }    \
    catch (...) { return fail(HC_PHMM_EHIP, "unexpected exception"); }

// --------------------------------------------------------------------------
// C ABI
extern "C" {

int hc_phmm_version(void) { return 30000; }

const char* hc_phmm_last_error(void) { return hcphmm::eng::last_error(); }

int hc_phmm_init(uint32_t /*flags*/, int device)
{
    std::lock_guard<std::mutex> lk(g_mu);
    const int32_t d = device;
    return init_devices_locked(&d, 1, device < 0);
}

int hc_phmm_init_devices(uint32_t /*flags*/, const int32_t* devices, int32_t n)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return init_devices_locked(devices, n, false);
}

int hc_phmm_device_count(void)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return int(g_devs.size());
}

int hc_phmm_shutdown(void)
{
    bool busy;
    {
        // Refuse while calls run or jobs / batches hold parts (they keep raw
        // Device and Slot pointers): shutdown_engine reports it, re-checking
        // under its own lock (g_mu is not recursive: not held here).
        std::lock_guard<std::mutex> lk(g_mu);
        busy = g_active_calls > 0 || g_live_parts > 0;
    }
    if (busy) return shutdown_engine();
    hcphmm::sw_release();
    hcphmm::gt_release();
    return shutdown_engine();
}

int hc_phmm_get_luts(float* pf, double* pd, float* mf, double* md)
{
    const Luts& L = luts();
    if (pf) std::memcpy(pf, L.ph2pr_f, sizeof(L.ph2pr_f));
    if (pd) std::memcpy(pd, L.ph2pr_d, sizeof(L.ph2pr_d));
    if (mf) std::memcpy(mf, L.mm_f.data(), sizeof(float) * kMMEntries);
    if (md) std::memcpy(md, L.mm_d.data(), sizeof(double) * kMMEntries);
    return HC_PHMM_OK;
}

int hc_phmm_submit_pairs(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                         const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                         const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, double* loglik,
                         float* raw_f32, double* raw_f64, uint8_t* rescued, hc_phmm_job** job)
{
    HC_API_TRY
    if (!job) return fail(HC_PHMM_EINVAL, "null job");
    *job = nullptr;
    if (n < 0) return fail(HC_PHMM_EINVAL, "negative pair count");
    if (!flat_args_ok(n, read_off, R, hap_off, H, rs, q, ins, del, gcp, hap))
        return fail(HC_PHMM_EINVAL, "null input array");
    CallGuard g;
    if (g.rc) return g.rc;
    if (n == 0) {
        *job = new hc_phmm_job();
        return HC_PHMM_OK;
    }
    Outputs o{loglik, raw_f32, raw_f64, rescued};
    return submit_flat(g.devs, flat_src(read_off, R, hap_off, H, rs, q, ins, del, gcp, hap), n, o, job);
    HC_API_CATCH
}

int hc_phmm_submit_regions(const hc_phmm_region* regions, int32_t n_regions, hc_phmm_job** job)
{
    HC_API_TRY
    if (!job) return fail(HC_PHMM_EINVAL, "null job");
    *job = nullptr;
    RegionSet rs;
    int rc = gather_regions(regions, n_regions, rs);
    if (rc) return rc;
    CallGuard g;
    if (g.rc) return g.rc;
    Src src;
    src.reads = rs.reads.data();
    src.haps = rs.haps.data();
    return submit_blocks(g.devs, src, rs.blocks, job);
    HC_API_CATCH
}

int hc_phmm_job_ready(hc_phmm_job* job)
{
    if (!job) return fail(HC_PHMM_EINVAL, "null job");
    for (Part* p : job->parts) {
        (void)hipSetDevice(p->dev->ordinal);
        const hipError_t e = hipEventQuery(p->done);
        if (e == hipErrorNotReady) return 0;
        if (e != hipSuccess) return fail(HC_PHMM_EHIP, std::string("device pass: ") + hipGetErrorString(e));
    }
    return 1;
}

int hc_phmm_collect(hc_phmm_job* job)
{
    HC_API_TRY
    if (!job) return fail(HC_PHMM_EINVAL, "null job");
    return collect(job);
    HC_API_CATCH
}

int hc_phmm_pairs_flat(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                       const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                       const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, double* loglik,
                       float* raw_f32, double* raw_f64, uint8_t* rescued)
{
    hc_phmm_job* job = nullptr;
    const int rc = hc_phmm_submit_pairs(n, read_off, R, hap_off, H, rs, q, ins, del, gcp, hap, loglik, raw_f32,
                                        raw_f64, rescued, &job);
    if (rc) return rc;
    return hc_phmm_collect(job);
}

int hc_phmm_cross(const hc_phmm_read* reads, int32_t n_reads, const hc_phmm_hap* haps, int32_t n_haps, double* out)
{
    if (n_reads < 0 || n_haps < 0) return fail(HC_PHMM_EINVAL, "negative count");
    if (n_reads == 0 || n_haps == 0) return HC_PHMM_OK;
    if (!reads || !haps || !out) return fail(HC_PHMM_EINVAL, "null argument");
    hc_phmm_region g{reads, n_reads, haps, n_haps, out};
    hc_phmm_job* job = nullptr;
    const int rc = hc_phmm_submit_regions(&g, 1, &job);
    if (rc) return rc;
    return hc_phmm_collect(job);
}

int hc_phmm_cross_regions(const hc_phmm_region* regions, int32_t n_regions)
{
    hc_phmm_job* job = nullptr;
    const int rc = hc_phmm_submit_regions(regions, n_regions, &job);
    if (rc) return rc;
    return hc_phmm_collect(job);
}

int hc_phmm_compute_likelihoods(const hc_phmm_read* reads, int32_t n_reads, const hc_phmm_hap* haps,
                                int32_t n_haps, double* out, uint8_t* keep, int32_t* n_kept)
{
    if (n_reads > 0 && !reads) return fail(HC_PHMM_EINVAL, "null reads");
    if (n_reads > 0 && (!keep || !n_kept)) return fail(HC_PHMM_EINVAL, "null keep/n_kept");
    int rc = hc_phmm_cross(reads, n_reads, haps, n_haps, out);
    if (rc) return rc;
    int kept = 0;
    // normalize_likelihoods_and_filter_poorly_modeled_reads, intel_pairhmm.hpp:24-46
    for (int r = 0; r < n_reads; ++r) {
        double* row = out + size_t(r) * size_t(n_haps);
        double best = n_haps ? row[0] : -INFINITY;
        for (int h = 1; h < n_haps; ++h)
            if (best < row[h]) best = row[h];
        const double cap = best + -4.5;
        for (int h = 0; h < n_haps; ++h)
            if (row[h] < cap) row[h] = cap;
        const double thr = std::min(2.0, std::ceil(double(reads[r].length) * 0.02)) * -4.0;
        keep[r] = !(best < thr);
        kept += keep[r];
    }
    if (n_kept) *n_kept = kept;
    return HC_PHMM_OK;
}

// ---- prepared batches (device-resident, one part per device slot)

int hc_phmm_batch_create(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off,
                         const int32_t* H, const uint8_t* rs, const uint8_t* q, const uint8_t* ins,
                         const uint8_t* del, const uint8_t* gcp, const uint8_t* hap, hc_phmm_batch** out)
{
    HC_API_TRY
    if (!out) return fail(HC_PHMM_EINVAL, "null out");
    *out = nullptr;
    if (n < 0) return fail(HC_PHMM_EINVAL, "negative pair count");
    if (!flat_args_ok(n, read_off, R, hap_off, H, rs, q, ins, del, gcp, hap))
        return fail(HC_PHMM_EINVAL, "null input array");
    CallGuard g;
    if (g.rc) return g.rc;
    int rc = HC_PHMM_OK;
    const Src src = flat_src(read_off, R, hap_off, H, rs, q, ins, del, gcp, hap);
    std::vector<int64_t> pre;
    prefix_sum(n, pre, [&](int64_t p) { return int64_t(std::max(0, R[p])) * std::max(0, H[p]); });
    const int G = int(g.devs.size());
    const std::vector<int64_t> cut = equal_cuts(pre, G);
    auto* B = new hc_phmm_batch();
    B->n = n;
    for (int j = 0; j < G; ++j) {
        if (j > 0 && cut[size_t(j)] == cut[size_t(j) + 1]) continue;
        PartSpec s;
        s.flat = true;
        s.lo = cut[size_t(j)];
        s.hi = cut[size_t(j) + 1];
        Device& d = *g.devs[size_t(j)];
        Part* p = nullptr;
        rc = hipSetDevice(d.ordinal) == hipSuccess ? plan_batch_part(d, src, s, &p)
                                                   : fail(HC_PHMM_EHIP, "hipSetDevice");
        if (rc) {
            for (Part* x : B->parts) free_part(x);
            delete B;
            return rc;
        }
        B->parts.push_back(p);
    }
    *out = B;
    return HC_PHMM_OK;
    HC_API_CATCH
}

int hc_phmm_batch_run(hc_phmm_batch* b, void* stream)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    if (stream && b->parts.size() > 1)
        return fail(HC_PHMM_EINVAL, "a caller stream selects one device; this batch spans several");
    for (Part* p : b->parts) {
        HIP_TRY(hipSetDevice(p->dev->ordinal));
        const int rc = run_part(p, stream ? static_cast<hipStream_t>(stream) : p->stream);
        if (rc) return rc;
    }
    return HC_PHMM_OK;
}

int hc_phmm_batch_results(hc_phmm_batch* b, double* loglik, float* raw_f32, double* raw_f64, uint8_t* rescued)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    const Outputs o{loglik, raw_f32, raw_f64, rescued};
    for (Part* p : b->parts) {
        if (!p->ran) return fail(HC_PHMM_EINVAL, "batch has not been run");
        if (p->n == 0) continue;
        HIP_TRY(hipSetDevice(p->dev->ordinal));
        HIP_TRY(hipStreamSynchronize(p->last_stream));
        std::vector<char> host(p->res_bytes);
        const size_t n = size_t(p->n);
        HIP_TRY(hipMemcpy(host.data(), p->d_raw32, sizeof(float) * n, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(host.data() + p->res_o64, p->d_raw64, sizeof(double) * n, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(host.data() + p->res_ofl, p->d_flag, n, hipMemcpyDeviceToHost));
        finish_part(*p, reinterpret_cast<const float*>(host.data()),
                    reinterpret_cast<const double*>(host.data() + p->res_o64),
                    reinterpret_cast<const uint8_t*>(host.data() + p->res_ofl), o);
    }
    return HC_PHMM_OK;
}

int hc_phmm_batch_device_results(hc_phmm_batch* b, void** raw_f32, void** raw_f64, void** rescued)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    if (b->parts.size() != 1) return fail(HC_PHMM_EINVAL, "device results of a batch split over several devices");
    Part* p = b->parts[0];
    if (raw_f32) *raw_f32 = p->d_raw32;
    if (raw_f64) *raw_f64 = p->d_raw64;
    if (rescued) *rescued = p->d_flag;
    return HC_PHMM_OK;
}

int hc_phmm_batch_bind_outputs(hc_phmm_batch* b, void* raw_f32, void* raw_f64, void* rescued)
{
    if (!b) return fail(HC_PHMM_EINVAL, "null batch");
    if (b->parts.size() != 1) return fail(HC_PHMM_EINVAL, "bind_outputs on a batch split over several devices");
    Part* p = b->parts[0];
    p->d_raw32 = raw_f32 ? static_cast<float*>(raw_f32) : p->own_raw32;
    p->d_raw64 = raw_f64 ? static_cast<double*>(raw_f64) : p->own_raw64;
    p->d_flag = rescued ? static_cast<uint8_t*>(rescued) : p->own_flag;
    return HC_PHMM_OK;
}

int hc_phmm_batch_stats(hc_phmm_batch* b, hc_phmm_stats* st)
{
    if (!b || !st) return fail(HC_PHMM_EINVAL, "null argument");
    std::memset(st, 0, sizeof(*st));
    st->n_pairs = b->n;
    st->n_devices = int64_t(b->parts.size());
    for (Part* p : b->parts) {
        HIP_TRY(hipSetDevice(p->dev->ordinal));
        st->cells += p->cells;
        st->n_launch_waves += p->launch_waves;
        st->n_lane_pairs += p->n_lane;
        if (p->d_nwaves && p->pack_ev[1]) {   // device-planned: the plan's own wave count
            int nw = 0;
            HIP_TRY(hipEventSynchronize(p->pack_ev[1]));
            HIP_TRY(hipMemcpy(&nw, p->d_nwaves, sizeof(int), hipMemcpyDeviceToHost));
            st->n_seg_waves += nw;
        } else {
            st->n_seg_waves += p->n_seg_waves;
        }
        st->upload_bytes += int64_t(p->upload_bytes);
        if (p->pack_ev[0]) {
            float pk = 0;
            HIP_TRY(hipEventSynchronize(p->pack_ev[1]));
            HIP_TRY(hipEventElapsedTime(&pk, p->pack_ev[0], p->pack_ev[1]));
            st->pack_ms = std::max(st->pack_ms, double(pk));
        }
        if (p->ran && p->ev_used > 0) {
            HIP_TRY(hipStreamSynchronize(p->last_stream));
            double sa = 0, sc = 0;
            for (size_t k = 0; k < p->ev_used; ++k) {
                float a = 0, c = 0;
                HIP_TRY(hipEventSynchronize(p->ev_pool[k][2]));
                HIP_TRY(hipEventElapsedTime(&a, p->ev_pool[k][0], p->ev_pool[k][1]));
                HIP_TRY(hipEventElapsedTime(&c, p->ev_pool[k][1], p->ev_pool[k][2]));
                sa += a;
                sc += c;
            }
            st->n_runs = std::max(st->n_runs, int64_t(p->ev_used));
            st->kernel_ms_f32 = std::max(st->kernel_ms_f32, sa / double(p->ev_used));
            st->kernel_ms_f64 = std::max(st->kernel_ms_f64, sc / double(p->ev_used));
            st->run_ms = std::max(st->run_ms, (sa + sc) / double(p->ev_used));
            p->ev_used = 0;
            int cnt[4] = {};
            HIP_TRY(hipMemcpy(cnt, p->d_count, sizeof(cnt), hipMemcpyDeviceToHost));
            // in-wave attempts past the limit were appended to the list instead
            st->n_rescued += cnt[p->parity ^ 1] + std::min(cnt[2 + (p->parity ^ 1)], p->inker_limit);
        }
    }
    return HC_PHMM_OK;
}

int hc_phmm_batch_destroy(hc_phmm_batch* b)
{
    if (!b) return HC_PHMM_OK;
    for (Part* p : b->parts) {
        (void)hipSetDevice(p->dev->ordinal);
        if (p->last_stream) (void)hipStreamSynchronize(p->last_stream);
        free_part(p);
    }
    delete b;
    return HC_PHMM_OK;
}

// ---- host-planning timing hooks (not part of the ABI: tools/plan_bench.py)
// Plan a call's parts on the host only, as submit would on `n_dev` slots of
// `n_cu` compute units, `reps` times; HC_PHMM_TRACE=1 prints the phases.
// Returns the mean milliseconds per call.
double hcx_plan_pairs(int64_t n, const int64_t* read_off, const int32_t* R, const int64_t* hap_off, const int32_t* H,
                      const uint8_t* rs, const uint8_t* q, const uint8_t* ins, const uint8_t* del, const uint8_t* gcp,
                      const uint8_t* hap, int n_cu, int n_dev, int reps)
{
    const Src src = flat_src(read_off, R, hap_off, H, rs, q, ins, del, gcp, hap);
    Device fake;
    fake.n_cu = n_cu;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < reps; ++k) {
        std::vector<int64_t> pre;
        prefix_sum(n, pre, [&](int64_t p) { return int64_t(std::max(0, R[p])) * std::max(0, H[p]); });
        const int np = part_count(pre.back(), n_dev);
        const std::vector<int64_t> cut = equal_cuts(pre, np);
        for (int j = 0; j < np; ++j) {
            PartSpec s;
            s.lo = cut[size_t(j)];
            s.hi = cut[size_t(j) + 1];
            Part* p = nullptr;
            (void)plan_part(fake, src, s, nullptr, false, PlanMode::Dry, &p);
        }
    }
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / reps;
}

// The last traced segmented pass (HC_PHMM_TIMELINE=1): up to max_waves
// records of {start, end, HW_ID} into out; returns the record count.
int hcx_timeline(unsigned long long* out, int max_waves) { return timeline_records(out, max_waves); }

// Sizes of the last dry-run plan: {pairs, order entries, segmented slots,
// segmented waves, structured (1) or general (0) planner}.
void hcx_dump_sizes(int64_t* out5)
{
    std::lock_guard<std::mutex> lk(g_dump.mu);
    out5[0] = int64_t(g_dump.pairs.size());
    out5[1] = int64_t(g_dump.order.size());
    out5[2] = g_dump.n_seg_slots;
    out5[3] = int64_t(g_dump.waves.size());
    out5[4] = g_dump.grid ? 1 : 0;
}

// The last dry-run plan: pairs as {row offset, R, table offset, H}, the slot
// order, and per segmented wave {slot0, rmax, rmin, ncols, npairs, nsteps}.
void hcx_dump_plan(int32_t* pairs4, int32_t* order, int32_t* waves6)
{
    std::lock_guard<std::mutex> lk(g_dump.mu);
    for (size_t k = 0; k < g_dump.pairs.size(); ++k) {
        const int4 p = g_dump.pairs[k];
        pairs4[4 * k] = p.x;
        pairs4[4 * k + 1] = p.y;
        pairs4[4 * k + 2] = p.z;
        pairs4[4 * k + 3] = p.w;
    }
    std::copy(g_dump.order.begin(), g_dump.order.end(), order);
    for (size_t w = 0; w < g_dump.waves.size(); ++w) {
        const LaneWave& v = g_dump.waves[w];
        const int32_t f[6] = {v.slot0, v.rmax, v.rmin, v.ncols, v.npairs, v.nsteps};
        std::copy(f, f + 6, waves6 + 6 * w);
    }
}

double hcx_plan_regions(const hc_phmm_region* regions, int32_t n_regions, int n_cu, int reps)
{
    RegionSet rs;
    if (gather_regions(regions, n_regions, rs)) return -1;
    Src src;
    src.reads = rs.reads.data();
    src.haps = rs.haps.data();
    Device fake;
    fake.n_cu = n_cu;
    PartSpec s;
    s.flat = false;
    s.blocks = rs.blocks;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < reps; ++k) {
        Part* p = nullptr;
        (void)plan_part(fake, src, s, nullptr, false, PlanMode::Dry, &p);
    }
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / reps;
}

}  // extern "C"


// --------------------------------------------------------------------------
// The reference's own accelerator slot: a strong definition of the weak
// `bool shacc_pairhmm::calculate(Batch&)` declared in
// pairhmm/native/shacc_pairhmm.h:10-36. The structs below are layout- and
// name-compatible declarations (same namespace, same member order) so the
// mangled symbol matches; results[r * num_haps + h] receives the fp32 cast of
// the log10 likelihood (the slot's `float* results`; hc_phmm_cross gives the
// full double).
namespace shacc_pairhmm {
struct Read {
    int length;
    const char* bases;
    const char* q;
    const char* i;
    const char* d;
    const char* c;
};
struct Haplotype {
    int length;
    const char* bases;
};
struct Batch {
    int num_reads;
    int num_haps;
    long num_cells;
    Read* reads;
    Haplotype* haps;
    float* results;
};
__attribute__((visibility("default"))) bool calculate(Batch& batch);
bool calculate(Batch& batch)
{
    static_assert(sizeof(Read) == sizeof(hc_phmm_read), "Read layout");
    static_assert(sizeof(Haplotype) == sizeof(hc_phmm_hap), "Haplotype layout");
    if (batch.num_reads < 0 || batch.num_haps < 0 || !batch.results) return false;
    std::vector<double> out(static_cast<size_t>(batch.num_reads) * size_t(batch.num_haps));
    const int rc = hc_phmm_cross(reinterpret_cast<const hc_phmm_read*>(batch.reads), batch.num_reads,
                                 reinterpret_cast<const hc_phmm_hap*>(batch.haps), batch.num_haps, out.data());
    if (rc != HC_PHMM_OK) return false;
    for (size_t k = 0; k < out.size(); ++k) batch.results[k] = float(out[k]);
    return true;
}
}  // namespace shacc_pairhmm