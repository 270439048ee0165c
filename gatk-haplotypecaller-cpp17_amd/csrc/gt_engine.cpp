// Host engine + C ABI of the genotyper numeric core (include/hc_gt.h).
//
// One call = every variant site of any number of regions: the regions'
// likelihood matrices are uploaded once each (sites of a region share it),
// with the kept-read lists and haplotype -> allele maps, in one H2D from a
// pinned staging block; one launch of gt_sites_kernel; one D2H of the genotype
// likelihoods, indices and qualities.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/hc_gt.h"
#include "../../include/hc_pairhmm.h"
#include "gt_kernels.hpp"
#include "pool.hpp"

// MathUtils Jacobian table as g++ folds it at compile time (tools/gen_jacobian.py).
#include "math_jacobian.inc"

namespace hcphmm {
void set_last_error(const std::string& msg);
int primary_device();
void gt_release();
}

using namespace hcgt;

namespace {

std::mutex g_mu;
hipStream_t g_stream = nullptr;
double* g_jac = nullptr;
char* g_dev = nullptr;
size_t g_dev_bytes = 0;
char* g_host = nullptr;
size_t g_host_bytes = 0;

int fail(int code, const std::string& msg)
{
    hcphmm::set_last_error(msg);
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(HC_PHMM_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Runs on the engine's first device slot, made current on the calling thread.
int ensure_init()
{
    const int rc = hc_phmm_init(0, -1);
    if (rc != HC_PHMM_OK) return rc;
    HIP_TRY(hipSetDevice(hcphmm::primary_device()));
    if (g_stream) return HC_PHMM_OK;
    HIP_TRY(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking));
    HIP_TRY(hipMalloc(&g_jac, sizeof(double) * kJacobianLen));
    static_assert(sizeof(kMathJacobianBits) == sizeof(double) * kJacobianLen, "table length");
    HIP_TRY(hipMemcpy(g_jac, kMathJacobianBits, sizeof(double) * kJacobianLen, hipMemcpyHostToDevice));
    return HC_PHMM_OK;
}

int reserve(size_t dev, size_t host)
{
    if (dev > g_dev_bytes) {
        if (g_dev) (void)hipFree(g_dev);
        g_dev = nullptr;
        g_dev_bytes = 0;
        if (hipMalloc(&g_dev, dev + dev / 4) != hipSuccess) return fail(HC_PHMM_ENOMEM, "genotyper device workspace");
        g_dev_bytes = dev + dev / 4;
    }
    if (host > g_host_bytes) {
        if (g_host) (void)hipHostFree(g_host);
        g_host = nullptr;
        g_host_bytes = 0;
        if (hipHostMalloc(&g_host, host + host / 4, hipHostMallocDefault) != hipSuccess)
            return fail(HC_PHMM_ENOMEM, "genotyper pinned workspace");
        g_host_bytes = host + host / 4;
    }
    return HC_PHMM_OK;
}

size_t up(size_t x) { return (x + 255) & ~size_t(255); }

int run(const hc_gt_site* sites, int32_t n)
{
    // Validate; one upload per distinct matrix.
    std::unordered_map<const double*, int32_t> mat_at;   // matrix -> index in mats
    std::vector<const hc_gt_site*> mats;                  // first site naming each matrix
    std::vector<int64_t> mat_off;                         // its offset in the L image
    std::vector<GtSite> ds(static_cast<size_t>(n));
    int64_t L_total = 0, keep_total = 0, map_total = 0, al_total = 0, out_total = 0;
    for (int32_t s = 0; s < n; ++s) {
        const hc_gt_site& x = sites[s];
        if (!x.L || x.n_reads < 0 || x.n_haps < 1 || x.n_keep < 0 || (x.n_keep && !x.keep) || !x.hap_allele ||
            x.n_alleles < 2 || x.n_alleles > HC_GT_MAX_ALLELES || !x.genotype_likelihoods || !x.genotype_index ||
            !x.genotype_quality)
            return fail(HC_PHMM_EINVAL, "site " + std::to_string(s) + ": bad argument");
        for (int32_t k = 0; k < x.n_keep; ++k)
            if (x.keep[k] < 0 || x.keep[k] >= x.n_reads)
                return fail(HC_PHMM_EINVAL, "site " + std::to_string(s) + ": kept read index out of range");
        for (int32_t h = 0; h < x.n_haps; ++h)
            if (x.hap_allele[h] < 0 || x.hap_allele[h] >= x.n_alleles)
                return fail(HC_PHMM_EINVAL, "site " + std::to_string(s) + ": haplotype allele out of range");
        auto it = mat_at.find(x.L);
        if (it == mat_at.end()) {
            it = mat_at.emplace(x.L, int32_t(mats.size())).first;
            mats.push_back(&x);
            mat_off.push_back(L_total);
            L_total += int64_t(x.n_reads) * x.n_haps;
        } else if (mats[size_t(it->second)]->n_reads != x.n_reads || mats[size_t(it->second)]->n_haps != x.n_haps) {
            // A matrix pointer shared by sites must describe the same shape.
            return fail(HC_PHMM_EINVAL, "sites sharing a matrix disagree on its shape");
        }
        GtSite& d = ds[size_t(s)];
        d.L_off = mat_off[size_t(it->second)];
        d.al_off = al_total;
        d.n_haps = x.n_haps;
        d.keep_off = int32_t(keep_total);
        d.n_keep = x.n_keep;
        d.map_off = int32_t(map_total);
        d.n_alleles = x.n_alleles;
        d.out_off = int32_t(out_total);
        keep_total += x.n_keep;
        map_total += x.n_haps;
        al_total += int64_t(x.n_keep) * x.n_alleles;
        out_total += x.n_alleles * (x.n_alleles + 1) / 2;
        if (keep_total > INT32_MAX || map_total > INT32_MAX || out_total > INT32_MAX)
            return fail(HC_PHMM_EINVAL, "too many sites for one call");
    }
    // Layout: [sites | L | keep | amap] uploaded, then [gl | gi | gq] read back, then scratch.
    const size_t o_sites = 0;
    const size_t o_L = up(o_sites + sizeof(GtSite) * size_t(n));
    const size_t o_keep = up(o_L + sizeof(double) * size_t(L_total));
    const size_t o_map = up(o_keep + sizeof(int32_t) * size_t(keep_total));
    const size_t in_bytes = up(o_map + sizeof(int32_t) * size_t(map_total));
    const size_t o_gl = in_bytes;
    const size_t o_gi = up(o_gl + sizeof(double) * size_t(out_total));
    const size_t o_gq = up(o_gi + sizeof(int32_t) * size_t(n));
    const size_t o_al = up(o_gq + sizeof(int32_t) * size_t(n));
    const size_t tail = o_al - o_gl;
    const size_t dev_bytes = up(o_al + sizeof(double) * size_t(std::max<int64_t>(al_total, 1)));
    int rc = reserve(dev_bytes, std::max(in_bytes, tail));
    if (rc) return rc;
    char* h = g_host;
    std::memcpy(h + o_sites, ds.data(), sizeof(GtSite) * size_t(n));
    // The likelihood matrices dominate the upload (512 regions of 415 x 32:
    // 54 MB): staged by the engine's worker pool, in slices so each slice's
    // H2D starts while the next is being copied.
    const int64_t nm = int64_t(mats.size());
    const int64_t slices = std::min<int64_t>(nm, 8);
    size_t sent = 0;
    for (int64_t sl = 0; sl < slices; ++sl) {
        const int64_t m0 = nm * sl / slices, m1 = nm * (sl + 1) / slices;
        hcphmm::parallel_for(m1 - m0, [&](int64_t lo, int64_t hi) {
            for (int64_t k = m0 + lo; k < m0 + hi; ++k) {
                const hc_gt_site* m = mats[size_t(k)];
                std::memcpy(h + o_L + sizeof(double) * size_t(mat_off[size_t(k)]), m->L,
                            sizeof(double) * size_t(m->n_reads) * size_t(m->n_haps));
            }
        }, 1);
        const size_t end = m1 < nm ? o_L + sizeof(double) * size_t(mat_off[size_t(m1)]) : o_keep;
        HIP_TRY(hipMemcpyAsync(g_dev + sent, h + sent, end - sent, hipMemcpyHostToDevice, g_stream));
        sent = end;
    }
    for (int32_t s = 0; s < n; ++s) {
        const hc_gt_site& x = sites[s];
        if (x.n_keep) std::memcpy(h + o_keep + sizeof(int32_t) * size_t(ds[size_t(s)].keep_off), x.keep, sizeof(int32_t) * size_t(x.n_keep));
        std::memcpy(h + o_map + sizeof(int32_t) * size_t(ds[size_t(s)].map_off), x.hap_allele, sizeof(int32_t) * size_t(x.n_haps));
    }
    HIP_TRY(hipMemcpyAsync(g_dev + sent, h + sent, in_bytes - sent, hipMemcpyHostToDevice, g_stream));
    GtArgs a{};
    a.sites = reinterpret_cast<const GtSite*>(g_dev + o_sites);
    a.n = n;
    a.L = reinterpret_cast<const double*>(g_dev + o_L);
    a.keep = reinterpret_cast<const int32_t*>(g_dev + o_keep);
    a.amap = reinterpret_cast<const int32_t*>(g_dev + o_map);
    a.jac = g_jac;
    const double table_step = 0.0001;   // JacobianLogTable::TABLE_STEP (math_utils.hpp:24)
    a.inv_step = 1.0 / table_step;      // INV_STEP (:25)
    a.log10_2 = std::log10(2.0);        // std::log10(2) (genotyper.hpp:280,321)
    a.al = reinterpret_cast<double*>(g_dev + o_al);
    a.gl = reinterpret_cast<double*>(g_dev + o_gl);
    a.gi = reinterpret_cast<int32_t*>(g_dev + o_gi);
    a.gq = reinterpret_cast<int32_t*>(g_dev + o_gq);
    HIP_TRY(launch_sites(a, g_stream));
    HIP_TRY(hipMemcpyAsync(h, g_dev + o_gl, tail, hipMemcpyDeviceToHost, g_stream));
    HIP_TRY(hipStreamSynchronize(g_stream));
    const double* gl = reinterpret_cast<const double*>(h);
    const int32_t* gi = reinterpret_cast<const int32_t*>(h + (o_gi - o_gl));
    const int32_t* gq = reinterpret_cast<const int32_t*>(h + (o_gq - o_gl));
    for (int32_t s = 0; s < n; ++s) {
        const hc_gt_site& x = sites[s];
        std::memcpy(x.genotype_likelihoods, gl + ds[size_t(s)].out_off,
                    sizeof(double) * size_t(x.n_alleles * (x.n_alleles + 1) / 2));
        *x.genotype_index = gi[s];
        *x.genotype_quality = gq[s];
    }
    return HC_PHMM_OK;
}

}  // namespace

extern "C" int hc_gt_genotype_sites(const hc_gt_site* sites, int32_t n_sites)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (n_sites < 0 || (n_sites && !sites)) return fail(HC_PHMM_EINVAL, "null sites / negative count");
    int rc = ensure_init();
    if (rc) return rc;
    if (n_sites == 0) return HC_PHMM_OK;
    return run(sites, n_sites);
}

// Called by hc_phmm_shutdown.
void hcphmm::gt_release()
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_stream) return;
    (void)hipStreamSynchronize(g_stream);
    if (g_jac) (void)hipFree(g_jac);
    if (g_dev) (void)hipFree(g_dev);
    if (g_host) (void)hipHostFree(g_host);
    (void)hipStreamDestroy(g_stream);
    g_stream = nullptr;
    g_jac = nullptr;
    g_dev = nullptr;
    g_host = nullptr;
    g_dev_bytes = g_host_bytes = 0;
}
