// obs_pass.hpp -- rsvio_ba_set_problem's observation pass (host code, no device code).
//
// SlidingWindow::optimize (src/estimator/sliding_window.rs:274-300) hands over one observation per
// (landmark, keyframe, camera): obs_lm, obs_kf, obs_cam and the normalised (u, v).  Before the
// window goes up, set_problem turns them into packed keys l << 6 | k << 1 | c, one (keyframe,
// camera) bit mask per landmark, and the (u, v) narrowed to f32 when that is exact -- a pass over
// ~25 B in and ~12 B out per observation (24,000 observations at config 3: ~0.9 MB), bound by one
// core's cache bandwidth.  On the headline step it sits on the critical path before the solve can
// start, so it is cut into landmark-run-aligned chunks that the calling thread and a few helper
// threads take by a CAS on one word (HostPool): a helper that is parked or descheduled only leaves
// its chunks to the others, so the pass is never slower than the caller alone by more than one
// futex wake.  Every chunk writes disjoint keys, (u, v) and -- its runs being whole -- disjoint
// masks; a landmark split over two runs (not a landmark-major list) or a duplicate is caught by the
// total bit count after the join, exactly as the single-threaded pass catches it.
#pragma once

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace rsvio_obs {

// ---- the (u, v) as f32 when every value is exactly an f32 (the estimator's are: normalised
// coordinates unprojected from f32 pixels and stored as f32 features, frame.rs:107-134 ->
// sliding_window.rs:274-300), halving the largest part of the window's PCIe upload; false (nothing
// usable written) if one is not, and the caller copies the f64 values.
__attribute__((target("avx2"))) static bool uv_narrow_avx2(size_t n2, const double* uv, float* out) {
    size_t i = 0;
    __m256d bad = _mm256_setzero_pd();
    for (; i + 4 <= n2; i += 4) {
        const __m256d d = _mm256_loadu_pd(uv + i);
        const __m128 f = _mm256_cvtpd_ps(d);
        bad = _mm256_or_pd(bad, _mm256_cmp_pd(_mm256_cvtps_pd(f), d, _CMP_NEQ_UQ));
        _mm_storeu_ps(out + i, f);
    }
    bool ok = _mm256_movemask_pd(bad) == 0;
    for (; i < n2; ++i) {
        out[i] = (float)uv[i];
        ok &= (double)out[i] == uv[i];
    }
    return ok;
}
static bool uv_narrow(size_t n2, const double* uv, float* out) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) return uv_narrow_avx2(n2, uv, out);
    bool ok = true;
    for (size_t i = 0; i < n2; ++i) {
        out[i] = (float)uv[i];
        ok &= (double)out[i] == uv[i];
    }
    return ok;
}

// ---- keys l << 6 | k << 1 | c with the index validation, 8 observations per AVX2 step (when the
// host has it); false if an index is out of range (the exact pass then reports which).
__attribute__((target("avx2"))) static bool obs_keys_avx2(int n_obs, const int32_t* lm, const int32_t* kf,
                                                        const uint8_t* cam, int n_lm, int n_kf, unsigned* key) {
    const __m256i nl1 = _mm256_set1_epi32(n_lm - 1), nk1 = _mm256_set1_epi32(n_kf - 1), one = _mm256_set1_epi32(1);
    __m256i bad = _mm256_setzero_si256();
    int i = 0;
    for (; i + 8 <= n_obs; i += 8) {
        const __m256i l = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(lm + i));
        const __m256i k = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(kf + i));
        const __m256i c = _mm256_cvtepu8_epi32(_mm_loadl_epi64(reinterpret_cast<const __m128i*>(cam + i)));
        // x > n - 1 (unsigned; negative indices are huge)  <=>  max(x, n - 1) != n - 1
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu32(l, nl1), nl1));
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu32(k, nk1), nk1));
        bad = _mm256_or_si256(bad, _mm256_xor_si256(_mm256_max_epu32(c, one), one));
        const __m256i kk = _mm256_or_si256(_mm256_or_si256(_mm256_slli_epi32(l, 6), _mm256_slli_epi32(k, 1)), c);
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(key + i), kk);
    }
    unsigned bad_t = 0;
    for (; i < n_obs; ++i) {
        const unsigned l = (unsigned)lm[i], k = (unsigned)kf[i], c = cam[i];
        bad_t |= (unsigned)(l >= (unsigned)n_lm) | (unsigned)(k >= (unsigned)n_kf) | (unsigned)(c > 1);
        key[i] = l << 6 | k << 1 | c;
    }
    return _mm256_testz_si256(bad, bad) && !bad_t;
}

static bool obs_keys(int n_obs, const int32_t* lm, const int32_t* kf, const uint8_t* cam, int n_lm, int n_kf,
                     unsigned* key) {
    if (n_lm <= 0 || n_kf <= 0) return false;
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) return obs_keys_avx2(n_obs, lm, kf, cam, n_lm, n_kf, key);
    unsigned bad = 0;
    for (int i = 0; i < n_obs; ++i) {
        const unsigned l = (unsigned)lm[i], k = (unsigned)kf[i], c = cam[i];
        bad |= (unsigned)(l >= (unsigned)n_lm) | (unsigned)(k >= (unsigned)n_kf) | (unsigned)(c > 1);
        key[i] = l << 6 | k << 1 | c;
    }
    return !bad;
}

// ---- the masks of the runs in key[a, b), four independent chains over run-aligned quarters, each
// keeping its current run's mask in a register and storing it (no load on the chain).  The caller
// zeroes m2 first and checks the total bit count afterwards (n_obs bits iff no duplicate and no
// landmark in two runs).
static void masks_of_runs(int a, int b, const unsigned* key, unsigned long long* m2) {
    const int n = b - a;
    if (n <= 0) return;
    int cut[5];
    cut[0] = a;
    cut[4] = b;
    for (int q = 1; q < 4; ++q) {
        int c = std::max(a + (int)((long long)q * n / 4), cut[q - 1]);
        while (c > a && c < b && (key[c] >> 6) == (key[c - 1] >> 6)) ++c;
        cut[q] = c;
    }
    int len = n;
    for (int q = 0; q < 4; ++q) len = std::min(len, cut[q + 1] - cut[q]);
    unsigned cl[4] = {~0u, ~0u, ~0u, ~0u};
    unsigned long long cm[4] = {0, 0, 0, 0};
    auto step = [&](int q, int i) {
        const unsigned kj = key[i], l = kj >> 6;
        const unsigned long long bit = 1ull << (kj & 63);
        cm[q] = l == cl[q] ? (cm[q] | bit) : bit;
        cl[q] = l;
        // (relaxed atomic: two chunks store the same landmark only when its observations are not
        // one run, which the bit count rejects)
        __atomic_store_n(m2 + l, cm[q], __ATOMIC_RELAXED);
    };
    for (int j = 0; j < len; ++j) {
        step(0, cut[0] + j);
        step(1, cut[1] + j);
        step(2, cut[2] + j);
        step(3, cut[3] + j);
    }
    for (int q = 0; q < 4; ++q)
        for (int i = cut[q] + len; i < cut[q + 1]; ++i) step(q, i);
}

__attribute__((target("popcnt"))) static long long mask_bits(int n_lm, const unsigned long long* m2) {
    long long bits = 0;
    for (int l = 0; l < n_lm; ++l) bits += __builtin_popcountll(m2[l]);
    return bits;
}

// Per-landmark (keyframe, camera) masks from the keys when each landmark's observations are
// contiguous (a landmark-major list, as SlidingWindow builds it).  True iff the masks hold n_obs
// bits in total -- no duplicate observation and no landmark in two runs; otherwise the exact pass
// rebuilds them (and reports a duplicate).
static bool obs_masks_runs(int n_obs, const unsigned* key, int n_lm, unsigned long long* m2) {
    std::memset(m2, 0, sizeof(unsigned long long) * (size_t)n_lm);
    masks_of_runs(0, n_obs, key, m2);
    return mask_bits(n_lm, m2) == n_obs;
}

// ======================================================================================
// HostPool: the calling thread plus `helpers` threads run fn(ctx, chunk) for chunk 0 .. n-1.  One
// 64-bit word holds (generation, n, next): a thread claims chunk `next` by a CAS that also checks the
// generation, so a late thread can neither claim a finished job's chunk nor run a new job with the
// old job's function (the function and context are read before the claim and used only when it
// succeeds: a job cannot be replaced before all its chunks are claimed and done).  Helpers spin
// for spin_us after their last chunk, then park on a condition variable; run() wakes parked ones
// and takes chunks itself meanwhile.  run() is for one caller at a time (try_run: false if busy).
class HostPool {
  public:
    using Fn = void (*)(void*, int);

    HostPool(int helpers, int spin_us) : spin_ns_((long long)spin_us * 1000) {
        for (int i = 0; i < helpers; ++i) threads_.emplace_back([this] { helper(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_.store(true, std::memory_order_seq_cst);
        }
        cv_.notify_all();
        for (auto& t : threads_) t.join();
    }
    int helpers() const { return (int)threads_.size(); }

    // false (nothing run) when another caller holds the pool
    bool try_run(int n, Fn fn, void* ctx) {
        std::unique_lock<std::mutex> own(run_m_, std::try_to_lock);
        if (!own.owns_lock()) return false;
        if (n <= 0) return true;
        fn_.store(fn, std::memory_order_relaxed);
        ctx_.store(ctx, std::memory_order_relaxed);
        done_.store(0, std::memory_order_relaxed);
        gen_ = (gen_ + 1) & 0xffffffffu;
        word_.store(pack(gen_, (unsigned)n, 0), std::memory_order_seq_cst);
        if (parked_.load(std::memory_order_seq_cst) > 0) {
            std::lock_guard<std::mutex> lk(m_);
            cv_.notify_all();
        }
        work(gen_);
        while (done_.load(std::memory_order_acquire) < n) _mm_pause();
        return true;
    }

  private:
    static uint64_t pack(uint32_t g, unsigned n, unsigned next) {
        return (uint64_t)g << 32 | (uint64_t)(n & 0xffff) << 16 | (next & 0xffff);
    }
    static uint32_t gen_of(uint64_t v) { return (uint32_t)(v >> 32); }
    static unsigned n_of(uint64_t v) { return (unsigned)(v >> 16) & 0xffff; }
    static unsigned next_of(uint64_t v) { return (unsigned)v & 0xffff; }

    // claims and runs chunks of generation g until none is left; false if the word moved on
    void work(uint32_t g) {
        uint64_t v = word_.load(std::memory_order_acquire);
        while (gen_of(v) == g && next_of(v) < n_of(v)) {
            Fn fn = fn_.load(std::memory_order_relaxed);
            void* ctx = ctx_.load(std::memory_order_relaxed);
            if (word_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel, std::memory_order_acquire)) {
                fn(ctx, (int)next_of(v));
                done_.fetch_add(1, std::memory_order_release);
                v = word_.load(std::memory_order_acquire);
            }
        }
    }

    void helper() {
        uint32_t seen = 0;
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            uint64_t v;
            for (;;) {  // spin for new work
                if (stop_.load(std::memory_order_relaxed)) return;
                v = word_.load(std::memory_order_acquire);
                if (gen_of(v) != seen) break;
                _mm_pause();
                if (std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                        .count() > spin_ns_) {
                    std::unique_lock<std::mutex> lk(m_);
                    parked_.fetch_add(1, std::memory_order_seq_cst);
                    cv_.wait(lk, [&] {
                        return stop_.load(std::memory_order_seq_cst) ||
                               gen_of(word_.load(std::memory_order_seq_cst)) != seen;
                    });
                    parked_.fetch_sub(1, std::memory_order_seq_cst);
                    if (stop_.load(std::memory_order_relaxed)) return;
                }
            }
            seen = gen_of(v);
            work(seen);
        }
    }

    std::vector<std::thread> threads_;
    std::atomic<uint64_t> word_{0};
    std::atomic<Fn> fn_{nullptr};
    std::atomic<void*> ctx_{nullptr};
    std::atomic<int> done_{0};
    std::atomic<int> parked_{0};
    std::atomic<bool> stop_{false};
    std::mutex m_, run_m_;
    std::condition_variable cv_;
    uint32_t gen_ = 0;
    long long spin_ns_;
};

// ======================================================================================
// The chunked pass: keys (+ validation), run masks and the narrowed (u, v) of each chunk.
struct ObsJob {
    const int32_t *lm, *kf;
    const uint8_t* cam;
    const double* uv;
    int n_lm, n_kf;
    unsigned* key;
    unsigned long long* m2;
    float* uv32;                 // null: (u, v) not narrowed here
    const int* cut;              // n_chunk + 1 run-aligned boundaries
    std::atomic<int> bad{0};     // an index out of range in some chunk
    std::atomic<int> wide{0};    // a (u, v) not exactly an f32 in some chunk

    static void chunk(void* p, int c) {
        ObsJob& J = *static_cast<ObsJob*>(p);
        const int a = J.cut[c], b = J.cut[c + 1];
        if (!obs_keys(b - a, J.lm + a, J.kf + a, J.cam + a, J.n_lm, J.n_kf, J.key + a))
            J.bad.store(1, std::memory_order_relaxed);
        else
            masks_of_runs(a, b, J.key, J.m2);
        if (J.uv32 && !uv_narrow(2 * (size_t)(b - a), J.uv + 2 * (size_t)a, J.uv32 + 2 * (size_t)a))
            J.wide.store(1, std::memory_order_relaxed);
    }
};

// The pool shared by every handle of the process (created on first use): RSVIO_BA_HOST_THREADS
// helpers (default 0: off -- on the MI355X box's host the pass did not get shorter with 3 helpers,
// 17.5 vs 14.7-20.7 us, the window's arrays being in the calling core's cache and the helpers'
// spinning costing CPU time, profiles/r06n_host_pool_cu_order_ab.txt), spinning
// RSVIO_BA_HOST_SPIN_US (default 2000) before parking.
static HostPool* shared_pool() {
    static HostPool* pool = [] {
        const char* tv = std::getenv("RSVIO_BA_HOST_THREADS");
        const char* sv = std::getenv("RSVIO_BA_HOST_SPIN_US");
        const int nt = tv ? std::max(0, std::min(15, std::atoi(tv))) : 0;
        const int sp = sv ? std::max(0, std::atoi(sv)) : 2000;
        return nt > 0 ? new HostPool(nt, sp) : nullptr;  // (lives to the process's end)
    }();
    return pool;
}

#ifndef RSVIO_OBS_CHUNK
#define RSVIO_OBS_CHUNK 3072
#endif
constexpr int kObsChunk = RSVIO_OBS_CHUNK;  // observations per chunk (~75 KB of input)

// The observation pass: keys, masks (m2, n_lm entries) and, when uv32 is not null, the narrowed
// (u, v).  Returns false when the fast path does not apply (an index out of range, a duplicate, a
// landmark in two runs): the caller then runs its exact pass.  *narrowed = every (u, v) fit f32.
static bool observation_pass(int n_obs, const int32_t* lm, const int32_t* kf, const uint8_t* cam,
                             const double* uv, int n_lm, int n_kf, unsigned* key, unsigned long long* m2,
                             float* uv32, bool* narrowed) {
    if (n_lm <= 0 || n_kf <= 0) return false;
    HostPool* pool = n_obs >= 2 * kObsChunk ? shared_pool() : nullptr;
    std::memset(m2, 0, sizeof(unsigned long long) * (size_t)n_lm);
    if (pool) {
        const int nc = std::min((n_obs + kObsChunk - 1) / kObsChunk, 0xffff);
        int cut_s[64];
        std::vector<int> cut_v;
        int* cut = cut_s;
        if (nc + 1 > 64) {
            cut_v.resize(nc + 1);
            cut = cut_v.data();
        }
        cut[0] = 0;
        cut[nc] = n_obs;
        for (int q = 1; q < nc; ++q) {  // run-aligned: a landmark's run stays in one chunk
            int c = std::max((int)((long long)q * n_obs / nc), cut[q - 1]);
            while (c > 0 && c < n_obs && lm[c] == lm[c - 1]) ++c;
            cut[q] = c;
        }
        ObsJob J;
        J.lm = lm; J.kf = kf; J.cam = cam; J.uv = uv; J.n_lm = n_lm; J.n_kf = n_kf;
        J.key = key; J.m2 = m2; J.uv32 = uv32; J.cut = cut;
        if (pool->try_run(nc, &ObsJob::chunk, &J)) {
            *narrowed = uv32 && !J.wide.load(std::memory_order_relaxed);
            if (J.bad.load(std::memory_order_relaxed)) return false;
            return mask_bits(n_lm, m2) == n_obs;
        }
    }
    *narrowed = uv32 && uv_narrow(2 * (size_t)n_obs, uv, uv32);
    if (!obs_keys(n_obs, lm, kf, cam, n_lm, n_kf, key)) return false;
    masks_of_runs(0, n_obs, key, m2);
    return mask_bits(n_lm, m2) == n_obs;
}

}  // namespace rsvio_obs
