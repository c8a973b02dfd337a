// trig_exhaustive.cpp -- proves rs-vio_amd/csrc/trig.hpp (the device's restatement of glibc
// sinf/cosf) bit-equal to this machine's libm over all 2^32 f32 inputs, and glibc's sincosf equal
// to the separate sinf/cosf (Rust may reach either).  Host build of the same header the kernels
// include; libm is the reference's trig (Rust f32::sin/cos -> glibc on x86-64 Linux).
//   g++ -O2 -mfma -ffp-contract=off -fno-builtin -I rs-vio_amd/csrc tools/trig_exhaustive.cpp \
//       -o /tmp/trig_exhaustive -lm -lpthread && /tmp/trig_exhaustive [lo hi]
#include "trig.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

extern "C" void sincosf(float, float*, float*);

namespace {
float (*volatile libm_sinf)(float) = ::sinf;
float (*volatile libm_cosf)(float) = ::cosf;

bool same(float a, float b) {
    return rsvio::libm_trig::f32_bits(a) == rsvio::libm_trig::f32_bits(b) || (a != a && b != b);
}

struct Count {
    uint64_t sin_bad = 0, cos_bad = 0, pair_bad = 0;
    uint32_t first = 0;
};
}  // namespace

int main(int argc, char** argv) {
    const uint64_t lo = argc > 1 ? strtoull(argv[1], nullptr, 0) : 0;
    const uint64_t hi = argc > 2 ? strtoull(argv[2], nullptr, 0) : (1ull << 32);
    const unsigned nt = std::max(1u, std::thread::hardware_concurrency());
    std::vector<Count> cnt(nt);
    std::vector<std::thread> th;
    for (unsigned k = 0; k < nt; ++k)
        th.emplace_back([&, k] {
            Count& c = cnt[k];
            const uint64_t a = lo + (hi - lo) * k / nt, b = lo + (hi - lo) * (k + 1) / nt;
            for (uint64_t i = a; i < b; ++i) {
                const uint32_t u = (uint32_t)i;
                float y;
                memcpy(&y, &u, 4);
                float ds, dc, ps, pc;
                rsvio::libm_trig::sincosf(y, &ds, &dc);
                const float ls = libm_sinf(y), lc = libm_cosf(y);
                ::sincosf(y, &ps, &pc);
                const bool bs = !same(ds, ls), bc = !same(dc, lc);
                if ((bs || bc) && !c.sin_bad && !c.cos_bad) c.first = u;
                c.sin_bad += bs;
                c.cos_bad += bc;
                c.pair_bad += !same(ps, ls) || !same(pc, lc);
            }
        });
    Count t;
    for (unsigned k = 0; k < nt; ++k) {
        th[k].join();
        if ((cnt[k].sin_bad || cnt[k].cos_bad) && !t.sin_bad && !t.cos_bad) t.first = cnt[k].first;
        t.sin_bad += cnt[k].sin_bad;
        t.cos_bad += cnt[k].cos_bad;
        t.pair_bad += cnt[k].pair_bad;
    }
    printf("inputs [%#llx, %#llx): %llu; trig.hpp vs libm sinf mismatches %llu, cosf %llu; "
           "libm sincosf vs sinf/cosf %llu%s\n",
           (unsigned long long)lo, (unsigned long long)hi, (unsigned long long)(hi - lo),
           (unsigned long long)t.sin_bad, (unsigned long long)t.cos_bad, (unsigned long long)t.pair_bad,
           (t.sin_bad || t.cos_bad) ? "" : " -- bit-equal");
    if (t.sin_bad || t.cos_bad) printf("first mismatch bits %08x\n", t.first);
    return (t.sin_bad || t.cos_bad) ? 1 : 0;
}
