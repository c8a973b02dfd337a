// CPU micro-benchmark + equality check of set_problem's observation pass (obs_pass.hpp): the
// single-threaded pass vs the chunked one over the helper pool (RSVIO_BA_HOST_THREADS, default 0: set it), on a config-3-shaped window
// (2,000 landmarks x 12 observations, landmark-major, (u, v) exact f32 values).
//   g++ -O2 -std=c++17 -pthread -I rs-vio_amd/csrc tools/obs_pass_bench.cpp -o /tmp/obs_pass_bench
#include <chrono>
#include <cstdio>
#include <random>

#include "obs_pass.hpp"

int main(int argc, char** argv) {
    const int n_lm = argc > 1 ? atoi(argv[1]) : 2000, per = 12, n_kf = 10, reps = argc > 2 ? atoi(argv[2]) : 2000;
    const int n_obs = n_lm * per;
    std::vector<int32_t> lm(n_obs), kf(n_obs);
    std::vector<uint8_t> cam(n_obs);
    std::vector<double> uv(2 * n_obs);
    std::mt19937 rng(7);
    for (int l = 0, i = 0; l < n_lm; ++l)
        for (int k = 0; k < 6; ++k)
            for (int c = 0; c < 2; ++c, ++i) {
                lm[i] = l;
                kf[i] = (l + k) % n_kf;
                cam[i] = (uint8_t)c;
                uv[2 * i] = (float)(rng() * 1e-9);
                uv[2 * i + 1] = (float)(rng() * 1e-9);
            }
    std::vector<unsigned> k1(n_obs), k2(n_obs);
    std::vector<unsigned long long> m1(n_lm), m2(n_lm);
    std::vector<float> u1(2 * n_obs), u2(2 * n_obs);
    double best[2] = {1e9, 1e9}, sum[2] = {0, 0};
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        bool n1 = rsvio_obs::uv_narrow(2 * (size_t)n_obs, uv.data(), u1.data());
        bool f1 = rsvio_obs::obs_keys(n_obs, lm.data(), kf.data(), cam.data(), n_lm, n_kf, k1.data()) &&
                  rsvio_obs::obs_masks_runs(n_obs, k1.data(), n_lm, m1.data());
        auto t1 = std::chrono::steady_clock::now();
        bool n2 = false;
        bool f2 = rsvio_obs::observation_pass(n_obs, lm.data(), kf.data(), cam.data(), uv.data(), n_lm, n_kf,
                                              k2.data(), m2.data(), u2.data(), &n2);
        auto t2 = std::chrono::steady_clock::now();
        const double a = std::chrono::duration<double, std::micro>(t1 - t0).count();
        const double b = std::chrono::duration<double, std::micro>(t2 - t1).count();
        best[0] = std::min(best[0], a); best[1] = std::min(best[1], b);
        sum[0] += a; sum[1] += b;
        ok &= n1 && n2 && f1 && f2 && k1 == k2 && m1 == m2 && u1 == u2;
    }
    // a landmark in two runs and a duplicate must be rejected
    std::swap(lm[5], lm[n_obs - 5]);
    bool n3;
    const bool split = rsvio_obs::observation_pass(n_obs, lm.data(), kf.data(), cam.data(), uv.data(), n_lm, n_kf,
                                                   k2.data(), m2.data(), u2.data(), &n3);
    std::swap(lm[5], lm[n_obs - 5]);
    kf[1] = kf[3];
    cam[1] = cam[3];
    const bool dup = rsvio_obs::observation_pass(n_obs, lm.data(), kf.data(), cam.data(), uv.data(), n_lm, n_kf,
                                                 k2.data(), m2.data(), u2.data(), &n3);
    printf("n_obs %d helpers %d: single %.1f us (mean %.1f), pool %.1f us (mean %.1f); equal %d; split rejected %d, "
           "duplicate rejected %d\n",
           n_obs, rsvio_obs::shared_pool() ? rsvio_obs::shared_pool()->helpers() : 0, best[0], sum[0] / reps, best[1],
           sum[1] / reps, (int)ok, (int)!split, (int)!dup);
    return ok && !split && !dup ? 0 : 1;
}
