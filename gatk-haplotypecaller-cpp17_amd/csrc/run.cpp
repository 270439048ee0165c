// The device pass of a prepared part (computeLikelihoodsNative's per-pair
// loop, intel_pairhmm.hpp:128-146, as kernels over the whole part): the fp32
// kernels emit raw sums, rescue flags and the rescue list; the fp64 rescue
// pass recomputes the flagged pairs; then the host log10 finish.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#include "engine_core.hpp"
#include "luts.hpp"
#include "pool.hpp"

namespace hcphmm {
namespace eng {

int run_part(Part* b, hipStream_t s)
{
    Device& dv = *b->dev;
    b->last_stream = s;
    b->launch_waves = 0;
    if (b->ev_used == b->ev_pool.size()) {
        std::array<hipEvent_t, 3> t{};
        for (auto& e : t) HIP_TRY(hipEventCreate(&e));
        b->ev_pool.push_back(t);
    }
    const auto& ev = b->ev_pool[b->ev_used++];
    for (int k = 0; k < 3; ++k) b->ev[k] = ev[k];
    HIP_TRY(hipEventRecord(b->ev[0], s));
    // No memsets: the fp32 kernels zero each pair's raw f64 slot as they emit,
    // and the rescue planner zeroes the other parity's counter for the next run.
    const int par = b->parity;
    b->parity ^= 1;
    int* count = b->d_count + par;
    Seg64Args r{};
    r.pairs = b->d_pairs;
    r.rows = b->d_rows;
    r.hapw = b->d_hapw;
    r.lut = dv.lut_d;
    r.list = b->d_list;
    r.list_rh = b->d_list + b->n;
    r.count = count;
    r.count_reset = b->d_count + (par ^ 1);
    r.inker_reset = b->d_count + 2 + (par ^ 1);
    r.ticket = b->d_count + kPlanTicket + par;
    r.ticket_reset = b->d_count + kPlanTicket + (par ^ 1);
    r.ready = b->d_count + kPlanReady + par;
    r.ready_reset = b->d_count + kPlanReady + (par ^ 1);
    r.sorted = b->d_sorted;
    r.big = b->d_big;
    r.big_count = b->d_big_count;
    r.plan = b->d_plan;
    r.raw_out = b->d_raw64;
    r.min_lanes = int64_t(2) * 4 * dv.n_cu * 64;
    r.wave_order = env_i64("HC_PHMM_RESCUE_ORDER", 1) != 0 ? b->d_worder : nullptr;   // 0: class order (A/B)
    r.next_wave = b->d_count + kNextWave;
    // 64-lane pairs chained in passes of many waves; 1: none (A/B)
    r.chain = int(std::min<int64_t>(kMaxChain, std::max<int64_t>(1, env_i64("HC_PHMM_CHAIN", kMaxChain))));
    r.chain_tail = int(std::max<int64_t>(0, env_i64("HC_PHMM_CHAIN_TAIL", 2)));
    r.n_simd = 4 * dv.n_cu;
    r.n_pairs = int(b->n);
    // Issue priority by remaining steps (seg_common.hpp set_prio_by_remaining):
    // on for the fp64 pass (S4: fp64 0.476 -> 0.462 ms); for the fp32 pass on
    // region parts (cross products) of at most 8 waves per SIMD — their waves
    // are alike and the pass ends when each SIMD's last ones do, which the
    // priority makes finish together (415 x 64 0.63 -> 0.59 ms, x 128 0.98 ->
    // 0.94, x 144 1.09 -> 1.07; x 200, ten waves per SIMD: 1.37 -> 1.44,
    // profiles/r05_prio_ab.txt) — and off for flat batches (S2 8.66 -> 8.81 ms,
    // 125k pairs 1.22 -> 1.25 ms). HC_PHMM_PRIO / HC_PHMM_PRIO64 override (A/B,
    // 0 or 1).
    const int prio = env_i64("HC_PHMM_PRIO", !b->spec.flat && b->n_seg_waves > 0 &&
                                                 int64_t(b->n_seg_waves) <= int64_t(8) * 4 * dv.n_cu
                                             ? 1 : 0) != 0 ? 1 : 0;
    r.prio = int(env_i64("HC_PHMM_PRIO64", 1));
    r.raw32 = b->d_raw32;
    r.flag = b->d_flag;
    r.err = b->d_count + kErrWord;
    r.force_plan_timeout = test_plan_timeout() ? 1 : 0;   // test hook (hcx_test_plan_timeout), off in use
    // initNative(use_double = true): no fp32 pass, every pair to the fp64 one
    // (intel_pairhmm.hpp:71,81,135-140).
    const bool all_f64 = (b->spec.flags & HC_PHMM_FLAG_F64) != 0;   // the call's mode (PartSpec::flags)
    bool solo = false;   // no fp64 launch after the fp32 pass (below)
    if (all_f64) HIP_TRY(launch_all_f64_list(int(b->n), b->d_raw32, b->d_flag, b->d_list, count, b->d_pairs, b->d_list + b->n, s));
    if (b->n_lane > 0 && !all_f64) {
        LaneArgs a{};
        a.pairs = b->d_pairs;
        a.order = b->d_lane_order;
        a.n_slots = b->n_lane;
        a.carry = b->d_carry;
        a.rows = b->d_rows;
        a.hapw = b->d_hapw;
        a.lut = dv.lut_f;
        a.raw_out = b->d_raw32;
        a.rescue_flag = b->d_flag;
        a.rescue_list = b->d_list;
        a.rescue_rh = b->d_list + b->n;   // (the list block holds 2n ints)
        a.rescue_count = count;
        a.raw64_zero = b->d_raw64;
        a.lut64 = dv.lut_d;
        a.prio = prio;
        if (env_i64("HC_PHMM_RESCUE_IN_WAVE", 1) != 0) {
            a.inker_count = b->d_count + 2 + par;
            // A wave that rescues in place runs up to ~2.5x longer; a few such
            // waves hide inside the pass, hundreds of them (a region whose reads
            // miss some haps: ~440 rescues) drain late and cost more than the
            // separate fp64 pass they would save (415 x 128 region: fp32
            // 0.925 -> 0.80 ms at a cap of 32, S2's 19 rescues unchanged;
            // profiles/r02_in_wave_rescue_cap.jsonl). Past the cap, the list.
            a.inker_limit = int(std::max<int64_t>(0, env_i64("HC_PHMM_RESCUE_IN_WAVE_MAX", 32)));
        }
        b->inker_limit = a.inker_limit;
        if (env_i64("HC_PHMM_TIMELINE", 0) != 0 && b->n_seg_waves > 0) {
            // Diagnostics: this part's own record buffer (parts run concurrently
            // on slot streams); hcx_timeline reads the last traced part's fp32
            // seg waves, hcx_timeline64 its fp64 waves (records after them).
            const int need = b->n_seg_waves + int(b->n) + 3;   // + the fp64 plan's records
            if (b->timeline_n < need) {
                if (b->timeline) {
                    HIP_TRY(hipStreamSynchronize(s));
                    HIP_TRY(hipFree(b->timeline));
                    b->timeline = nullptr;
                }
                HIP_TRY(hipMalloc(&b->timeline, size_t(need) * 3 * sizeof(unsigned long long)));
                b->timeline_n = need;
            }
            b->timeline_n32 = b->n_seg_waves;
            HIP_TRY(hipMemsetAsync(b->timeline + 3 * size_t(b->n_seg_waves), 0,
                                   size_t(b->n + 3) * 3 * sizeof(unsigned long long), s));
            std::lock_guard<std::mutex> lk(g_tl.mu);
            g_tl.part = b;
            a.timeline = b->timeline;
            r.timeline = b->timeline + 3 * size_t(b->n_seg_waves);
        }
        b->launch_waves += b->lane_waves;
        const int n_one = b->lane_waves - b->n_seg_waves;
        const bool fork = b->n_seg_waves > 0 && n_one > 0;
        if (b->n_seg_waves > 0) {
            // Segmented waves; beside one-lane waves (long haps) they go on the
            // side stream, launched first so they are dispatched first.
            LaneArgs g = a;
            g.waves = b->d_lane_waves;
            g.n_waves = b->n_seg_waves;
            g.n_waves_dev = b->d_nwaves;
            g.sdesc = b->d_sdesc;
            // One wave per launched slot, the hardware dispatching them in the
            // plan's order (persistent waves fetching from per-XCD queues
            // measured no faster and were removed).
            if (fork) {
                HIP_TRY(hipEventRecord(b->fork, s));
                HIP_TRY(hipStreamWaitEvent(b->side, b->fork, 0));
            }
            // Per-slot records (gathered by the fp64 launch) pay off in HBM
            // writes on large parts; on small ones the gather's two dependent
            // loads sit on the pass's critical path, and the scattered stores
            // they replace are a few MB: parts below HC_PHMM_REC_MIN_PAIRS
            // write their results in place.
            const int64_t rec_min = b->spec.rec_min >= 0 ? b->spec.rec_min : env_i64("HC_PHMM_REC_MIN_PAIRS", 200000);
            const bool rec = b->d_rec && b->n >= rec_min;
            g.rec = rec ? b->d_rec : nullptr;
            r.rec = g.rec;   // the fp64 launch gathers the seg slots' records
            r.slot_of = b->d_slot_of;
            // Small parts of seg waves only, every hap within one wave's fp64
            // reach: each wave rescues all its flagged pairs itself and no fp64
            // launch follows (S1: that launch was ~6 us of a 73 us pass, for an
            // empty list). Larger parts keep the list: a region whose reads miss
            // many haps would serialise hundreds of rescues in its waves.
            solo = !rec && n_one == 0 && b->n_wide == 0 && b->cls[0].n == 0 && b->cls[1].n == 0 &&
                   a.inker_count != nullptr && b->Hmax <= kInWaveRescueMaxH &&
                   b->n <= env_i64("HC_PHMM_SOLO_MAX_PAIRS", 32768);
            // (The fused pass — rescues drained by the fp32 launch's own waves —
            // and stealable rescues measured slower than the fp64 launch after
            // the pass and were removed)
            if (solo) {
                g.solo_counters = b->d_count;
                g.solo_other = par ^ 1;
                g.inker_limit = std::numeric_limits<int>::max();
                b->inker_limit = g.inker_limit;
            }
            HIP_TRY(launch_lane_seg_f32(g, fork ? b->side : s));
            if (fork) HIP_TRY(hipEventRecord(b->join, b->side));
        }
        if (n_one > 0) {
            a.waves = b->d_lane_waves + b->n_seg_waves;
            a.n_waves = n_one;
            HIP_TRY(launch_lane_f32(b->lane_variant, a, s));
        }
        if (fork) HIP_TRY(hipStreamWaitEvent(s, b->join, 0));
    }
    for (auto& c : b->cls) {
        if (c.n == 0 || all_f64) continue;
        DiagArgs a{};
        a.pairs = b->d_pairs;
        a.order = c.d_order;
        a.n_slots = c.n;
        a.rows = b->d_rows;
        a.hapw = b->d_hapw;
        a.lut = dv.lut_f;
        a.ring_len = c.ring_len;
        a.ring_global = diag_ring_in_lds(c.W, c.ring_len, false) ? nullptr : b->d_ring;
        a.raw_out = b->d_raw32;
        a.rescue_flag = b->d_flag;
        a.rescue_list = b->d_list;
        a.rescue_rh = b->d_list + b->n;   // (the list block holds 2n ints)
        a.rescue_count = count;
        a.raw64_zero = b->d_raw64;
        const int G = 64 / c.W;
        const int grid = (c.n + G - 1) / G;
        b->launch_waves += grid;
        HIP_TRY(launch_diag_f32(c.W, a, grid, s));
    }
    HIP_TRY(hipEventRecord(b->ev[1], s));
    // Early results (a job part whose fp64 launch follows, results in place):
    // the fp32 pass's raw sums and rescue flags, final now, go to the pinned
    // image on the side stream while the fp64 launch runs, and collect()
    // finishes the unflagged pairs' log10 in that time; the fp64 sums and the
    // counters follow (enqueue_results). The 415 x 128 region's host finish
    // (~0.06 ms of log10f) overlapped its fp64 launch (~0.1 ms).
    b->early_used = b->early && b->host_res && !solo && !all_f64 && r.rec == nullptr && b->n > 0 &&
                    b->d_raw32 == b->own_raw32 && env_i64("HC_PHMM_EARLY_FINISH", 1) != 0;
    if (b->early_used) {
        HIP_TRY(hipStreamWaitEvent(b->side, b->ev[1], 0));
        HIP_TRY(launch_store_to_host(b->host_res, b->own_raw32, b->res_o64, b->side));
        HIP_TRY(launch_store_to_host(b->host_res + b->res_ofl, b->own_flag, b->res_ocnt - b->res_ofl, b->side));
        HIP_TRY(hipEventRecord(b->early, b->side));
    }
    if (b->n > 0 && !solo) {
        // fp64 rescue (intel_pairhmm.hpp:137-139) over the device-built list, no
        // host round trip for its length: device planning + column-segmented
        // fp64 waves (grid-stride), then the anti-diagonal fp64 kernel for haps
        // wider than 64 blocks of 32 (only launched if the batch has any). (The
        // plan folded into the fp32 pass's last workgroup measured slower on S1:
        // fp32 0.068 -> 0.075 ms for 2 us saved, the per-workgroup fences.)
        const int grid = int(std::min<int64_t>((b->n + 3) / 4, int64_t(2) * dv.n_cu));
        HIP_TRY(launch_rescue_seg64(r, grid, s));
        if (b->n_wide > 0) {
            DiagArgs a{};
            a.pairs = b->d_pairs;
            a.order = b->d_big;
            a.n_slots_dev = b->d_big_count;
            a.rows = b->d_rows;
            a.hapw = b->d_hapw;
            a.lut = dv.lut_d;
            a.ring_len = b->Hmax + 2 * 64 + 16;
            a.ring_global = diag_ring_in_lds(64, a.ring_len, true) ? nullptr : b->d_ring;
            a.raw_out = b->d_raw64;
            const int64_t cap = a.ring_global ? b->wide_ring_blocks : 2048;
            HIP_TRY(launch_diag_f64(64, a, int(std::max<int64_t>(1, std::min<int64_t>(b->n_wide, cap))), s));
        }
    }
    // A solo run's end is ev[1]: recording ev[2] right behind it would only add
    // the marker's own stream time (~5 us measured on S1, as much as the fp64
    // launch it replaces).
    if (!solo) HIP_TRY(hipEventRecord(b->ev[2], s));
    if (b->ev_solo.size() < b->ev_pool.size()) b->ev_solo.resize(b->ev_pool.size());
    b->ev_solo[b->ev_used - 1] = solo;
    b->ran = true;
    return HC_PHMM_OK;
}

// The device error word of a part's last runs (kErrWord) from a host copy of
// its counters: HC_PHMM_EHIP with a message if any kernel gave up.
int check_device_error(const int* counters)
{
    const int e = counters[kErrWord];
    if (e == 0) return HC_PHMM_OK;
    std::string m = "device pass incomplete (error word " + std::to_string(e) + ")";
    if (e & kErrPlanWait) m += ": fp64 rescue workgroups timed out waiting for the rescue plan";
    return fail(HC_PHMM_EHIP, m);
}

int enqueue_results(Part* b, hipStream_t s)
{
    if (b->early_used) {   // the rest: raw f64, flags again (same bytes), counters; done covers both
        HIP_TRY(launch_store_to_host(b->host_res + b->res_o64, reinterpret_cast<const char*>(b->own_raw32) + b->res_o64,
                                     b->res_bytes - b->res_o64, s));
        HIP_TRY(hipStreamWaitEvent(s, b->early, 0));
    } else {
        HIP_TRY(launch_store_to_host(b->host_res, b->own_raw32, b->res_bytes, s));
    }
    if (!b->done) HIP_TRY(hipEventCreateWithFlags(&b->done, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(b->done, s));
    return HC_PHMM_OK;
}

// log10 finish (intel_pairhmm.hpp:137-143, glibc log10 / log10f as in the
// reference) of a part's results, scattered into the caller's outputs. Chunks
// of 2 048 pairs: a 415 x 128 region's 53 120 log10 calls spread over the
// whole pool (in chunks of 8 192 they took 7 threads, ~0.07 ms).
void finish_part(const Part& P, const float* f, const double* d, const uint8_t* fl, const Outputs& o, Finish which)
{
    const Luts& L = luts();
    const float l10f = L.log10_init_f;
    const double l10d = L.log10_init_d;
    auto ll = [&](int64_t k) { return fl[k] ? std::log10(d[k]) - l10d : double(std::log10(f[k]) - l10f); };
    auto want = [&](int64_t k) { return which == Finish::All || (fl[k] != 0) == (which == Finish::Rescued); };
    if (which == Finish::Rescued) {
        // The flagged pairs after an early finish: usually a few hundred, done
        // on this thread, found eight flags at a time (the pool's wake-up
        // alone cost ~0.05 ms of a 415 x 128 region call here).
        std::vector<int64_t> base(P.spec.blocks.size() + 1, 0);
        for (size_t b = 0; b < P.spec.blocks.size(); ++b)
            base[b + 1] = base[b] + int64_t(P.spec.blocks[b].nr) * P.spec.blocks[b].nh;
        auto one = [&](int64_t k) {
            if (P.spec.flat) {
                const int64_t i = P.spec.lo + k;
                if (o.loglik) o.loglik[i] = ll(k);
                if (o.raw32) o.raw32[i] = f[k];
                if (o.raw64) o.raw64[i] = d[k];
                if (o.resc) o.resc[i] = fl[k];
                return;
            }
            const size_t b = size_t(std::upper_bound(base.begin(), base.end(), k) - base.begin()) - 1;
            const Block& B = P.spec.blocks[b];
            const int64_t r = (k - base[b]) / B.nh, h = (k - base[b]) % B.nh;
            B.out[r * B.ostride + h] = ll(k);
        };
        int64_t k = 0;
        for (; k + 8 <= P.n; k += 8) {
            uint64_t w;
            std::memcpy(&w, fl + k, 8);
            if (w == 0) continue;
            for (int j = 0; j < 8; ++j)
                if (fl[k + j]) one(k + j);
        }
        for (; k < P.n; ++k)
            if (fl[k]) one(k);
        return;
    }
    if (P.spec.flat) {
        const int64_t id0 = P.spec.lo;
        parallel_for(P.n, [&](int64_t lo, int64_t hi) {
            for (int64_t k = lo; k < hi; ++k) {
                if (!want(k)) continue;
                if (o.loglik) o.loglik[id0 + k] = ll(k);
                if (o.raw32) o.raw32[id0 + k] = f[k];
                if (o.raw64) o.raw64[id0 + k] = which == Finish::Plain ? 0.0 : d[k];
                if (o.resc) o.resc[id0 + k] = fl[k];
            }
        }, 2048);
        return;
    }
    // Blocks: pair k of block b is (r, h) = divmod(k - base, nh).
    std::vector<int64_t> base(P.spec.blocks.size() + 1, 0);
    for (size_t b = 0; b < P.spec.blocks.size(); ++b)
        base[b + 1] = base[b] + int64_t(P.spec.blocks[b].nr) * P.spec.blocks[b].nh;
    parallel_for(P.n, [&](int64_t lo, int64_t hi) {
        size_t b = size_t(std::upper_bound(base.begin(), base.end(), lo) - base.begin()) - 1;
        int64_t k = lo;
        while (k < hi) {
            const Block& B = P.spec.blocks[b];
            const int64_t end = std::min(hi, base[b + 1]);
            int64_t r = (k - base[b]) / B.nh, h = (k - base[b]) % B.nh;
            for (; k < end; ++k) {
                if (want(k)) B.out[r * B.ostride + h] = ll(k);
                if (++h == B.nh) {
                    h = 0;
                    ++r;
                }
            }
            ++b;
        }
    }, 2048);
}

}  // namespace eng
}  // namespace hcphmm
