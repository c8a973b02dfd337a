// ba.hip -- HP-B: sliding-window bundle adjustment on gfx950 (f64), landmark-sharded over ranks.
//
// Replaces SlidingWindow::optimize's solver call (src/estimator/sliding_window.rs:159-381):
// BundleAdjustmentFactor::linearize (src/optimization/factors.rs:350-447) for every observation,
// Huber(2.0) (sliding_window.rs:295-296), and apex-solver's LevenbergMarquardt with
// SparseSchurComplement (sliding_window.rs:126-135,325) -- restated as DESIGN.md "BA LM".
//
// Layout (landmark-major, built once per problem on the host):
//   obs   sorted by (landmark, keyframe, camera)
//   slot  = (landmark, keyframe) group of 1-2 observations, sorted like obs
//   wave  = a run of whole landmarks with <= 64 slots: one lane per slot (padded to 64 per wave)
//   chunk = <= 64 (slot_a, slot_b) pairs of one upper-triangular 6x6 camera block (fa <= fb)
// A linearisation (lambda-independent) of a state is stored per slot -- W, U, g_c -- and per
// landmark -- V, g_p -- in the raw buffers of that state (double-buffered like the state).
// Per solve: K0 ba_reset, K4 ba_linearize (the initial state), then per LM iteration (one HIP
// stream; the host reads the LM state once per chunk of iterations):
//   K4c ba_schur_chunks         wave / 64 pairs: (V + lambda I)^-1, Y = W V^-1 on the fly,
//                               -Y_a W_b^T (+ U, Y g_p - g_c on the diagonal), lane-ordered sums
//   K4d ba_schur_combine        wave / camera block: chunk partials in chunk order -> S, b, g_c
//   [RCCL all-reduce of the per-rank reduced system when sharded]
//   K5  ba_camera_solve         1 workgroup: S, b in LDS; pipelined 4-wave LDL^T (n <= 60) or
//                               blocked Cholesky; substitutions, SE3 (+) trial poses
//   K6  ba_backsub_relinearize  wave / landmark group: dp = V^-1 (-g_p - W^T dc), trial point,
//                               and the speculative linearisation of the trial state (residual,
//                               Jacobian, Huber) into the other raw buffers -- its cost is the
//                               trial cost; an accepted step needs no further linearisation
//   [sharded: K6r per-rank trial scalars + RCCL all-reduce, K7 ba_lm_decide]
//   single rank: the last K6 wave to arrive takes the LM decision (gain ratio, accept / reject
//   = buffer flip, lambda, termination)
// Every reduction has a fixed order (no floating-point atomics): results are run-to-run identical.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/resource.h>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "common.hpp"

#include "obs_pass.hpp"  // host: set_problem's observation pass
#include "se3.hpp"
#include "wave.hpp"

// HP-B is f64 with tolerance parity: multiply-adds contract to FMAs
// here, unlike the tracker's bit-exact f32 code (built with -ffp-contract=off)
#pragma clang fp contract(fast)

namespace rsvio {

namespace {

RSVIO_DBG_DECL
RSVIO_RT_DECL

constexpr int kMaxFree = 20;            // camera system up to 120 x 120 in LDS
constexpr int kMaxN = 6 * kMaxFree;
// Raw linearisation per slot, one contiguous 224-B record (AoS).  factors.rs:437-441: the
// translation columns of the 2x9 Jacobian equal the point columns (J = [Jp | Jp | Jr]), so of a
// slot's W = Jc^T Jp (6x3), U = Jc^T Jc (6x6) and g_c = Jc^T r only the rotation parts are new:
//   W = [Vs; Wr],  U = [[Vs, Wr^T], [Wr, Ur]],  g_c = [gp_s; gr]
// with Vs, gp_s the slot's own landmark-block contribution.  Record: Vs (3x3 packed upper, 6),
// gp_s (3), Wr (3x3, rotation row x point column, 9), Ur (3x3 packed upper, 6), gr (3), pad --
// 27 values instead of 48, and half the multiply-adds of the linearisation.  Per landmark
// (96 B): V (3x3 packed upper), g_p (3), pad.
enum { RV = 0, RGP = 6, RWR = 9, RUR = 18, RGR = 24, kRawF = 28 };
enum { LV = 0, LG = 6, kLmF = 12 };
constexpr int kBlockF = 48;             // 36 S + 6 b + 6 g_c per camera block workgroup
constexpr int kPartA = 2;               // cost of the initial linearisation, 0 (per wave)
constexpr int kPartD = 4;               // trial cost, |dp|^2, g_p.dp, |p|^2 per wave
// Landmark groups of the Schur reduction: wave w (K4 / K6 workgroup w, dispatched round robin to
// XCD w % 8) belongs to group w % kGrp, and K4c workgroup 8 pb + g (on XCD g) reduces block pb
// over group g -- each slot record is fetched into one XCD's L2 per launch; K5 sums the kGrp
// partial systems.  (4 groups of 512-thread workgroups: 42 vs 39 us per LM iteration -- two
// waves per SIMD then share the FP64 pipe -- although K5's combine moved half the bytes.)
constexpr int kGrp = 8;
constexpr int kSchurThreads = 256;      // K4c workgroup: one pair per thread per pass
constexpr int kK5Threads = 256;         // K5 (n_free <= 10): 4 waves (8 pulling the partials measured no faster)

struct Mat4 {
    double m[16];
};

// factors.rs:350-447 -- residual and the 2x9 Jacobian [dp_W | dt | dw]; false on cheirality failure
__device__ __forceinline__ bool linearize(const double* pW, const Pose& P, const double* TCB, const double* uv,
                                          double r[2], double J[2][9], bool want_j) {
    double RCB[3][3] = {{TCB[0], TCB[1], TCB[2]}, {TCB[4], TCB[5], TCB[6]}, {TCB[8], TCB[9], TCB[10]}};
    double pB[3], pC[3], tmp[3];
    mat3vec(P.R, pW, tmp);
#pragma unroll
    for (int i = 0; i < 3; ++i) pB[i] = tmp[i] + P.t[i];
    mat3vec(RCB, pB, tmp);
    pC[0] = tmp[0] + TCB[3];
    pC[1] = tmp[1] + TCB[7];
    pC[2] = tmp[2] + TCB[11];
    if (pC[2] <= 0.0) {  // cheirality (factors.rs:391-403)
        r[0] = 1e6;
        r[1] = 1e6;
        if (want_j)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 9; ++b) J[a][b] = 0.0;
        return false;
    }
    r[0] = pC[0] / pC[2] - uv[0];
    r[1] = pC[1] / pC[2] - uv[1];
    if (!want_j) return true;
    double iz = 1.0 / pC[2];
    double iz2 = iz * iz;
    double Jp[2][3] = {{iz, 0.0, -pC[0] * iz2}, {0.0, iz, -pC[1] * iz2}};
    double A[2][3], M[3][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) A[i][j] = (Jp[i][0] * RCB[0][j] + Jp[i][1] * RCB[1][j]) + Jp[i][2] * RCB[2][j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double v = (A[i][0] * P.R[0][j] + A[i][1] * P.R[1][j]) + A[i][2] * P.R[2][j];
            J[i][j] = v;
            J[i][3 + j] = v;
        }
    double S[3][3] = {{0.0, -pW[2], pW[1]}, {pW[2], 0.0, -pW[0]}, {-pW[1], pW[0], 0.0}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            M[i][j] = ((-P.R[i][0]) * S[0][j] + (-P.R[i][1]) * S[1][j]) + (-P.R[i][2]) * S[2][j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) J[i][6 + j] = (A[i][0] * M[0][j] + A[i][1] * M[1][j]) + A[i][2] * M[2][j];
    return true;
}

__device__ __forceinline__ bool inv3(const double A[3][3], double X[3][3]) {
    double c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
    double c01 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
    double c02 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
    double det = A[0][0] * c00 + A[0][1] * c01 + A[0][2] * c02;
    if (!(det > 0.0) || !isfinite(det)) return false;
    double id = 1.0 / det;
    X[0][0] = c00 * id;
    X[1][0] = c01 * id;
    X[2][0] = c02 * id;
    X[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) * id;
    X[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) * id;
    X[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) * id;
    X[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) * id;
    X[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) * id;
    X[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) * id;
    return true;
}

__device__ __forceinline__ int utri(int a, int c) {  // index of (min, max) in a packed 6x6 upper triangle
    int i = a < c ? a : c, j = a < c ? c : a;
    return i * 6 - i * (i - 1) / 2 + (j - i);
}

// LM bookkeeping that lives on the device.  Two copies alternate by iteration: iteration i's
// K4c reads copy i & 1 (the state left by iteration i-1, with its trial pending), takes the
// pending decision and writes the decided state to copy (i+1) & 1, which K5 / K6 of iteration i
// then use -- so no workgroup ever reads a copy another workgroup of the same launch writes.
struct LmState {
    double lambda, nu, cost, initial_cost;
    double dc2, gcdc;
    double new_cost, dp2, gpdp, x2;
    int iter, status, done, solve_ok;
    int accepted, cur;                      // cur: which of the two state buffers is current
    int pending;                            // K5 produced a step (or failed) not yet decided
    int p2p_err;                            // K7 (sharded over P2P): a peer did not arrive
};

struct Geometry {
    int n_kf, n_free, n_lm, n_obs, n_slot, n_pb, n_wave, n_chunk, pair_stride;
    Mat4 TCB[2];
    double huber_delta;
    int chol;  // linear solver: 0 Schur (inv3 landmark blocks), 1 the SparseCholesky fallback (LL^T)
    // the symbolic envelope of the camera system: env[k] = the last free keyframe whose rows of
    // column block k may be nonzero in L (>= k; a window of landmarks over consecutive keyframes
    // gives a band), set_problem from the landmarks' keyframe masks
    unsigned char env[kMaxFree];
    int env_on;  // env is the landmarks' (past 10 free keyframes); else env[k] = n_free - 1, unused
};

// Structure-of-arrays problem description (device pointers)
// Slot header, padded layout: slot (wave w, lane i) is entry 64 w + i, two int4 per slot
//   {kf, landmark, lane of the landmark's first slot, slots of the landmark}
//   {free block of kf or -1, observations (0 = padding, <= 2), camera bits, 0}
// and its observations' normalised coordinates inline (2 double2): everything a lane needs
// before the pose / point loads arrives in one round trip.
// Schur chunks: chunk c = 8 pb + x (workgroup c of K4c, dispatched to XCD c % 8 = x) holds all
// slot pairs of camera block pb among the landmarks of XCD group x (the landmarks of the K6 / K4
// waves w with w % 8 == x, which run on that XCD too).  Its partial goes to slot x of the
// partial systems (cpart: 8 copies of the sys layout), which K5 sums in slot order.
struct Prob {
    const int* free_idx;     // kf -> free block or -1
    const int4* slot_hdr;    // 2 per padded slot
    const double2* slot_uv;  // 2 per padded slot
    const int4* pairs;       // n_chunk x pair_stride: {slot a, slot b, landmark, 0}, padding a = -1
    const int* pb_fa;
    const int* pb_fb;
    const int* dmap;         // MFMA camera solve: packed-system entry -> dense LDS position (see kMfMap*)
};

struct Work {
    double* pose[2];         // n_kf x 7, current / trial (LmState::cur)
    double* pw[2];           // n_lm x 3
    const double* pose_init;
    const double* pw_init;
    double* raws[2];         // n_slot x kRawF per state buffer
    double* rawl[2];         // n_lm x kLmF per state buffer
    int* singular;           // set by K4c when a landmark block (V + lambda I) is singular
    const int* p2p_err;      // sharded over P2P: the exchange kernels' error flag (else null)
    double* partA;           // n_wave x kPartA
    double* partD;           // n_wave x kPartD
    double* cpart;           // kGrp x sys_len partial systems (slot g: landmark group g)
    double* sys;             // n_pb * 36 + 12 n_free + 2
    double* dc;              // 6 n_free
    double* trial4;          // 4 (sharded: reduced trial scalars)
    const LmState* st_prev;  // K4c: the state left by the previous iteration (read only)
    LmState* st;             // this iteration's state (K4c's owner block writes it; K5, K6 use it)
    unsigned long long* tick;  // [0] decisions published to the host, [1] solve start (wall clock)
};

__device__ __forceinline__ size_t sys_len(const Geometry& G) { return (size_t)G.n_pb * 36 + 12 * G.n_free + 2; }

// ---------------------------------------------------------------------------------------
// Landmark sharding over the P2P one-shot exchange
// ---------------------------------------------------------------------------------------
constexpr int kP2PMax = 8;       // ranks
constexpr int kP2PMsg = 8192;    // doubles per slot (>= 36 * 210 + 12 * 20 + 2)

struct P2P {
    double* peer[kP2PMax];       // exchange buffer of each rank (own one included)
    int nranks, rank;
    int* xnw;                    // (local) every rank's wave count, as K5's exchange carried it
    int ll;                      // K5's system exchange flag-in-word (RSVIO_P2P_LL=1, A/B) instead of data + flags
};

// The trial-scalar exchange folded into K6 and the next decision (RSVIO_P2P_FOLD=2): after the
// system's message slots and their flags, each buffer holds per parity, per source rank and per
// wave that rank's K6 wave partial (4 doubles) and its generation flag.
constexpr int kP2PWaves = 16384;  // waves per rank (a larger shard takes the X2 path)
constexpr size_t kP2PTval = (size_t)2 * kP2PMax * kP2PMsg + 2 * kP2PMax;  // doubles before the trial values
constexpr size_t kP2PTflag = kP2PTval + (size_t)2 * kP2PMax * kP2PWaves * 4;
// Small messages (n <= kP2PLLMax doubles: the trial scalars, the attach self-test) take the
// flag-in-word protocol: every double travels as two 8-byte words {32 data bits, 32-bit
// generation}, each an atomic store, so a reader knows a word has arrived when it carries the
// exchange's generation -- no fence and no separate flag between the data and its readiness
// (the flag protocol's writer waits for its data writes to be acknowledged before it may raise
// the flag: one more xGMI round trip per exchange).  Per parity and source rank, 2 kP2PLLMax words.
constexpr int kP2PLLMax = 16;
constexpr size_t kP2PLL = kP2PTflag + (size_t)2 * kP2PMax * kP2PWaves;  // (in doubles / words)
// K5's system exchange in flag-in-word form (A/B): per parity and source rank 2 kP2PMsg words
constexpr size_t kP2PLLSys = kP2PLL + (size_t)2 * kP2PMax * 2 * kP2PLLMax;
constexpr size_t kP2PBytes = sizeof(double) * (kP2PLLSys + (size_t)2 * kP2PMax * 2 * kP2PMsg);

__device__ __forceinline__ unsigned long long* p2p_flags(double* xbuf) {
    return reinterpret_cast<unsigned long long*>(xbuf + (size_t)2 * kP2PMax * kP2PMsg);
}

// P2P exchange buffer slot [parity][rank] of a peer's buffer, and the generation flags
__device__ __forceinline__ double* p2p_slot(double* xbuf, int par, int r) {
    return xbuf + (size_t)(par * kP2PMax + r) * kP2PMsg;
}
// trial exchange: wave w of source rank r, parity par (value quad and its flag)
__device__ __forceinline__ double* p2p_tval(double* xbuf, int par, int r, int w) {
    return xbuf + kP2PTval + (((size_t)par * kP2PMax + r) * kP2PWaves + w) * 4;
}
__device__ __forceinline__ unsigned long long* p2p_tflag(double* xbuf, int par, int r, int w) {
    return reinterpret_cast<unsigned long long*>(xbuf + kP2PTflag) + ((size_t)par * kP2PMax + r) * kP2PWaves + w;
}
// One value of every rank's slot, summed in rank order (identical bits on every rank): the
// nranks loads are issued together (a clamped index past nranks, its value not added), so the
// sum costs one round trip to the exchange buffer, not one per rank -- a runtime rank loop of
// load + add put a full wait on every load (nranks round trips per value; at 4 ranks that was
// the largest part of K5's exchange).
__device__ __forceinline__ void p2p_rank_sum(const double* mine, int nr, int e, double& acc) {
    double v[kP2PMax];
#pragma unroll
    for (int r = 0; r < kP2PMax; ++r)
        v[r] = __hip_atomic_load(mine + (size_t)min(r, nr - 1) * kP2PMsg + e, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
    for (int r = 0; r < kP2PMax; ++r)
        if (r < nr) acc += v[r];
}

// sums[i] += every rank's entry tid + T i, in rank order: ranks in groups of W whose loads are in
// flight together (a clamped index past the last rank, not added)
template <int KE, int W>
__device__ __forceinline__ void p2p_group_sums(const double* mine, int nr, int ne, int tid, int T, double (&sums)[KE]) {
    for (int r0 = 0; r0 < nr; r0 += W) {
        double v[KE][W];
#pragma unroll
        for (int i = 0; i < KE; ++i)
#pragma unroll
            for (int q = 0; q < W; ++q)
                v[i][q] = __hip_atomic_load(mine + (size_t)min(r0 + q, nr - 1) * kP2PMsg + min(tid + T * i, ne - 1),
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
        for (int i = 0; i < KE; ++i)
#pragma unroll
            for (int q = 0; q < W; ++q)
                if (r0 + q < nr) sums[i] += v[i][q];
    }
}

// p2p_group_sums with this rank's own contribution taken from registers (own[i], substituted at
// rank `me` in the rank order: the same adds, the same bits): only the PEERS' slots are read
// from the uncached exchange buffer, and at one rank nothing is
template <int KE, int W>
__device__ __forceinline__ void p2p_group_sums_own(const double* mine, int nr, int me, int ne, int tid, int T,
                                                   const double (&own)[KE], double (&sums)[KE]) {
    for (int r0 = 0; r0 < nr; r0 += W) {
        double v[KE][W];
#pragma unroll
        for (int i = 0; i < KE; ++i)
#pragma unroll
            for (int q = 0; q < W; ++q) {
                const int r = r0 + q;
                v[i][q] = (r < nr && r != me)
                              ? __hip_atomic_load(mine + (size_t)r * kP2PMsg + min(tid + T * i, ne - 1),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                              : own[i];
            }
#pragma unroll
        for (int i = 0; i < KE; ++i)
#pragma unroll
            for (int q = 0; q < W; ++q)
                if (r0 + q < nr) sums[i] += v[i][q];
    }
}

// flag-in-word slot [parity][source rank] (2 kP2PLLMax words)
__device__ __forceinline__ unsigned long long* p2p_ll(double* xbuf, int par, int r) {
    return reinterpret_cast<unsigned long long*>(xbuf + kP2PLL) + ((size_t)par * kP2PMax + r) * 2 * kP2PLLMax;
}
__device__ __forceinline__ unsigned long long* p2p_llsys(double* xbuf, int par, int r) {
    return reinterpret_cast<unsigned long long*>(xbuf + kP2PLLSys) + ((size_t)par * kP2PMax + r) * 2 * kP2PMsg;
}
// acc[i] += every rank's tagged entry tid + T i, in rank order: ranks in groups of W, each group's
// words polled together until all carry tag g; true if a peer never arrived (bounded)
template <int KE, int W>
__device__ __forceinline__ bool ll_group_sums(const unsigned long long* mine, int nr, int ne, int tid, int T,
                                              unsigned g, double (&acc)[KE]) {
    bool late = false;
    for (int r0 = 0; r0 < nr; r0 += W) {
        unsigned long long w[KE][W][2];
        long long spins = 0;
        for (;;) {
#pragma unroll
            for (int i = 0; i < KE; ++i)
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    const unsigned long long* a =
                        mine + (size_t)min(r0 + q, nr - 1) * 2 * kP2PMsg + 2 * (size_t)min(tid + T * i, ne - 1);
                    w[i][q][0] = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    w[i][q][1] = __hip_atomic_load(a + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            bool ok = true;
#pragma unroll
            for (int i = 0; i < KE; ++i)
#pragma unroll
                for (int q = 0; q < W; ++q) ok &= (unsigned)(w[i][q][0] >> 32) == g && (unsigned)(w[i][q][1] >> 32) == g;
            if (ok) break;
            if (++spins > (1ll << 25)) {
                late = true;
                break;
            }
            // back off after the first polls: every re-poll reads all KE x W x 2 words of every
            // thread from uncached memory, and on a GPU the ranks share (the rehearsals) a tight
            // loop starves the late rank whose words it waits for
            if (spins > 4)
                __builtin_amdgcn_s_sleep(16);
            else
                __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int i = 0; i < KE; ++i)
#pragma unroll
            for (int q = 0; q < W; ++q)
                if (r0 + q < nr)
                    acc[i] += __longlong_as_double((long long)((w[i][q][0] & 0xffffffffull) | (w[i][q][1] << 32)));
    }
    return late;
}

// s_waitcnt immediate (gfx9 encoding) for vmcnt(0) with expcnt / lgkmcnt left at their maxima: this
// wave's outstanding memory operations -- its stores included -- have completed.  The encoding (and
// stores counted by vmcnt, no separate store counter) is gfx9's: the build targets gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "kWaitStores is the gfx9 s_waitcnt encoding: build for gfx950 (ARCH=gfx950)"
#endif
constexpr int kWaitStores = 0x0F70;

template <int SCOPE>
__device__ __forceinline__ void ll_put_scope(unsigned long long* w, double v, unsigned g) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v), t = (unsigned long long)g << 32;
    __hip_atomic_store(w, (b & 0xffffffffull) | t, __ATOMIC_RELAXED, SCOPE);
    __hip_atomic_store(w + 1, (b >> 32) | t, __ATOMIC_RELAXED, SCOPE);
}

__device__ __forceinline__ void ll_put(unsigned long long* w, double v, unsigned g) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v), t = (unsigned long long)g << 32;
    __hip_atomic_store(w, (b & 0xffffffffull) | t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(w + 1, (b >> 32) | t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


// ---------------------------------------------------------------------------------------
__global__ void ba_reset(Geometry G, Work Wk, double lambda0) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 7 * G.n_kf) {
        Wk.pose[0][i] = Wk.pose_init[i];
        Wk.pose[1][i] = Wk.pose_init[i];
    }
    if (i < 3 * G.n_lm) {
        Wk.pw[0][i] = Wk.pw_init[i];
        Wk.pw[1][i] = Wk.pw_init[i];
    }
    if (i == 0) {
        Wk.tick[1] = wall_clock64();
        *Wk.singular = 0;
        LmState s{};
        s.lambda = lambda0;
        s.nu = 2.0;
        *Wk.st = s;
    }
}

// ---------------------------------------------------------------------------------------
// Linearisation of one slot (lane) and of the wave's landmarks, shared by K4 (initial state)
// and K6 (the trial state): factors.rs:350-447 residual + 2x9 Jacobian per observation,
// Huber IRLS weight, and the slot's contributions V, g_p (landmark block), W, U, g_c
// (camera blocks, free keyframes only), cost.
// ---------------------------------------------------------------------------------------
struct SlotLin {
    double V[6], gp[3], Wr[9], Ur[6], gr[3], cost;
};

__device__ __forceinline__ void slot_linearize(const Geometry& G, const Pose& P, const double p[3], int nobs,
                                               int cams, const double2 (&uvq)[2], bool fr, SlotLin& L) {
#pragma unroll
    for (int i = 0; i < 6; ++i) L.V[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) L.gp[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) L.Wr[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) L.Ur[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) L.gr[i] = 0.0;
    L.cost = 0.0;
    // unrolled over the <= 2 observations of a slot: a runtime-indexed uvq[o] was lowered to a
    // scratch-memory array (a store + reload on the linearisation's critical path)
#pragma unroll
    for (int o = 0; o < 2; ++o) {
        if (o >= nobs) break;
        double r[2], J[2][9];
        const double uv[2] = {uvq[o].x, uvq[o].y};
        linearize(p, P, G.TCB[(cams >> o) & 1].m, uv, r, J, true);
        double sq = r[0] * r[0] + r[1] * r[1], rho, wt;
        huber(sq, G.huber_delta, &rho, &wt);
        L.cost += 0.5 * rho;
        const double wr0 = wt * r[0], wr1 = wt * r[1];
        int k = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
#pragma unroll
            for (int c = a; c < 3; ++c) L.V[k++] += wt * (J[0][a] * J[0][c] + J[1][a] * J[1][c]);
            L.gp[a] += J[0][a] * wr0 + J[1][a] * wr1;
        }
        if (fr) {
            int u = 0;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
#pragma unroll
                for (int c = 0; c < 3; ++c) L.Wr[a * 3 + c] += wt * (J[0][6 + a] * J[0][c] + J[1][6 + a] * J[1][c]);
#pragma unroll
                for (int c = a; c < 3; ++c) L.Ur[u++] += wt * (J[0][6 + a] * J[0][6 + c] + J[1][6 + a] * J[1][6 + c]);
                L.gr[a] += J[0][6 + a] * wr0 + J[1][6 + a] * wr1;
            }
        }
    }
}

// Store one wave's linearisation into raw buffer `buf`: the slot records (free keyframes), then
// the landmark sums V, g_p in slot order by each landmark's first lane.  Called by the whole
// wave (contains barriers); sh is a [10][64] LDS scratch.
// intra-wave LDS hand-off (a wave's LDS operations execute in order; this keeps the compiler
// from moving them across)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <bool WAVE = false>
__device__ void store_linearization(const Work& Wk, int buf, int s, int lane, bool act, bool fr, int first, int nk,
                                    int l, const SlotLin& L, double (*sh)[64]) {
    if (act && fr) {
        double rec[kRawF];
#pragma unroll
        for (int i = 0; i < 6; ++i) rec[RV + i] = L.V[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) rec[RGP + i] = L.gp[i];
#pragma unroll
        for (int i = 0; i < 9; ++i) rec[RWR + i] = L.Wr[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) rec[RUR + i] = L.Ur[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) rec[RGR + i] = L.gr[i];
        rec[27] = 0.0;
        double2* dst = reinterpret_cast<double2*>(Wk.raws[buf] + (size_t)s * kRawF);
#pragma unroll
        for (int i = 0; i < kRawF / 2; ++i) dst[i] = make_double2(rec[2 * i], rec[2 * i + 1]);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) sh[i][lane] = L.V[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) sh[6 + i][lane] = L.gp[i];
    if constexpr (WAVE) wave_sync(); else __syncthreads();
    if (act && lane == first) {  // landmark sums in slot order
        double Vl[6] = {0, 0, 0, 0, 0, 0}, gl[3] = {0, 0, 0};
        for (int k = 0; k < nk; ++k) {
#pragma unroll
            for (int i = 0; i < 6; ++i) Vl[i] += sh[i][first + k];
#pragma unroll
            for (int i = 0; i < 3; ++i) gl[i] += sh[6 + i][first + k];
        }
        double rec[kLmF] = {Vl[0], Vl[1], Vl[2], Vl[3], Vl[4], Vl[5], gl[0], gl[1], gl[2], 0.0, 0.0, 0.0};
        double2* dst = reinterpret_cast<double2*>(Wk.rawl[buf] + (size_t)l * kLmF);
#pragma unroll
        for (int i = 0; i < kLmF / 2; ++i) dst[i] = make_double2(rec[2 * i], rec[2 * i + 1]);
    }
}

// (V + lambda I)^-1 by its 3x3 Cholesky factor L: (L L^T)^-1 = L^-T L^-1.  This is the
// landmark block of the SparseCholesky fallback (sliding_window.rs:334-341) with the landmarks
// eliminated first -- the order a fill-reducing ordering gives the BA arrow matrix -- so the
// camera block it leaves is the same Schur complement; false unless every pivot is > 0.
__device__ __forceinline__ bool chol_inv3(const double A[3][3], double X[3][3]) {
    const double d0 = A[0][0];
    if (!(d0 > 0.0) || !isfinite(d0)) return false;
    const double l00 = sqrt(d0), l10 = A[1][0] / l00, l20 = A[2][0] / l00;
    const double d1 = A[1][1] - l10 * l10;
    if (!(d1 > 0.0) || !isfinite(d1)) return false;
    const double l11 = sqrt(d1), l21 = (A[2][1] - l20 * l10) / l11;
    const double d2 = (A[2][2] - l20 * l20) - l21 * l21;
    if (!(d2 > 0.0) || !isfinite(d2)) return false;
    const double l22 = sqrt(d2);
    const double m00 = 1.0 / l00, m11 = 1.0 / l11, m22 = 1.0 / l22;
    const double m10 = -(l10 * m00) * m11, m21 = -(l21 * m11) * m22;
    const double m20 = -(l20 * m00 + l21 * m10) * m22;
    X[0][0] = (m00 * m00 + m10 * m10) + m20 * m20;
    X[0][1] = X[1][0] = m10 * m11 + m20 * m21;
    X[0][2] = X[2][0] = m20 * m22;
    X[1][1] = m11 * m11 + m21 * m21;
    X[1][2] = X[2][1] = m21 * m22;
    X[2][2] = m22 * m22;
    return true;
}

// (V + lambda I)^-1 of a landmark from its raw record; the same f64 operations wherever it is
// needed (K4c lanes, K6 first lanes), so every user sees identical bits.  false if singular
// (then Vi = 0).  chol: the SparseCholesky fallback's LL^T form (chol_inv3).
__device__ __forceinline__ bool landmark_inverse(const double* Vp, double lambda, double Vi[3][3], int chol) {
    double A[3][3] = {{Vp[0] + lambda, Vp[1], Vp[2]}, {Vp[1], Vp[3] + lambda, Vp[4]}, {Vp[2], Vp[4], Vp[5] + lambda}};
    const bool ok = chol ? chol_inv3(A, Vi) : inv3(A, Vi);
    if (!ok)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int c = 0; c < 3; ++c) Vi[a][c] = 0.0;
    return ok;
}

// ---------------------------------------------------------------------------------------
// set_problem's device part (ba_build_layout, one launch): the padded slot layout and the pair
// lists of the Schur chunks -- chunk c = 8 pb + x lists, in ascending landmark order, every
// landmark of group x (the landmarks of the waves w % 8 == x) that has slots in both keyframes
// (fa, fb) of camera block pb (a landmark has at most one slot per keyframe, so at most one pair
// per chunk) as {slot a, slot b, landmark, 0}, and {-1, 0, 0, 0} past the count (the host sizes
// the stride by the largest group).
// ---------------------------------------------------------------------------------------
// The padded slot layout of a problem, built on the device from what set_problem uploads: per
// landmark the (keyframe, camera) bit mask (bit 2 kf + cam) and the padded position of its first
// slot (the host's greedy wave packing), per wave its real slot count, per observation its packed
// key and (u, v).  A landmark's slots are its keyframes in ascending order; a slot's observations
// are camera 0 then camera 1 -- the layout of a stable (landmark, keyframe, camera) sort.
struct SlotSrc {
    const unsigned long long* mask;  // n_lm
    const int* lm_base;              // n_lm: padded slot of the landmark's first slot, -1 unobserved
    const int* wave_fill;            // n_wave: real slots of the wave (the rest are padding lanes)
    const int* wave_lm;              // n_wave + 1: first landmark of each wave, then n_lm
    const unsigned* key;             // n_obs: landmark << 6 | kf << 1 | cam
    const double2* uv;               // n_obs, f64 -- or, when uv32 is set, the same values as f32 pairs
    int nb_lm, nb_pad;               // blocks of the landmark and padding parts of the grid
    int uv32;                        // the upload holds (u, v) as float2 (every value exact in f32)
};
constexpr unsigned long long kEvenBits = 0x5555555555555555ull;

// blocks [0, nb_lm): one thread per landmark -- its slot headers {kf, landmark, lane of the
// landmark's first slot, slots of the landmark} {free block of kf or -1, observations, camera
// bits, 0}; [nb_lm, nb_lm + nb_pad): one thread per padded slot -- the waves' padding lanes
// {0, 0, 0, 0} {-1, 0, 0, 0} with zero observations; the rest: one thread per observation -- its
// (u, v) into its slot (first = camera 0 if present, second = camera 1; an absent second zero).
__device__ void build_slots_body(const Geometry& G, const Prob& Pr, const SlotSrc& S, int4* hdr, double2* huv,
                                 int b) {
    const int t = threadIdx.x;
    const double2 z2 = make_double2(0.0, 0.0);
    if (b < S.nb_lm) {
        const int l = 256 * b + t;
        if (l >= G.n_lm) return;
        const int base = S.lm_base[l];
        if (base < 0) return;
        const unsigned long long m = S.mask[l];
        unsigned long long kb = (m | (m >> 1)) & kEvenBits;
        const int ns = __popcll(kb);
        for (size_t ps = (size_t)base; kb; kb &= kb - 1, ++ps) {
            const int k = (__ffsll((long long)kb) - 1) >> 1;
            const int c0 = (int)(m >> (2 * k)) & 1, c1 = (int)(m >> (2 * k + 1)) & 1;
            const int no = c0 + c1;
            hdr[2 * ps] = make_int4(k, l, base & 63, ns);
            hdr[2 * ps + 1] = make_int4(Pr.free_idx[k], no, no == 2 ? 2 : c1, 0);
            if (no == 1) huv[2 * ps + 1] = z2;
        }
    } else if (b < S.nb_lm + S.nb_pad) {
        const int ps = 256 * (b - S.nb_lm) + t;
        if (ps >= 64 * G.n_wave || (ps & 63) < S.wave_fill[ps >> 6]) return;
        hdr[2 * (size_t)ps] = make_int4(0, 0, 0, 0);
        hdr[2 * (size_t)ps + 1] = make_int4(-1, 0, 0, 0);
        huv[2 * (size_t)ps] = z2;
        huv[2 * (size_t)ps + 1] = z2;
    } else {
        const int i = 256 * (b - S.nb_lm - S.nb_pad) + t;
        if (i >= G.n_obs) return;
        const unsigned key = S.key[i];
        const int l = (int)(key >> 6), k = (int)(key >> 1) & 31, c = (int)(key & 1);
        const unsigned long long m = S.mask[l];
        const unsigned long long below = ((m | (m >> 1)) & kEvenBits) & ((1ull << (2 * k)) - 1ull);
        const size_t q = (size_t)S.lm_base[l] + __popcll(below);
        const int sub = (c == 1 && ((m >> (2 * k)) & 1)) ? 1 : 0;
        if (S.uv32) {  // widened exactly: the same f64 values as the caller's
            const float2 f = reinterpret_cast<const float2*>(S.uv)[i];
            huv[2 * q + sub] = make_double2((double)f.x, (double)f.y);
        } else {
            huv[2 * q + sub] = S.uv[i];
        }
    }
}

// The Schur pair list of chunk c = 8 pb + x straight from the landmark masks (no slot headers
// needed, so it runs in the same launch as the slot build): the landmarks of the group's waves
// w = x + 8 k, in (wave, landmark) order -- the order K4c's chunk sums have always used -- that have a
// slot in both keyframes of camera block pb give {slot a, slot b, landmark, 0}; {-1, 0, 0, 0}
// past the count.  Four waves, each a contiguous run of the group's waves: count, prefix, write.
constexpr int kPairU = 8;  // waves of a run whose landmark ranges and masks are in flight together

__device__ void build_pairs_body(const Geometry& G, const Prob& Pr, const SlotSrc& S, int4* pairs, int c) {
    __shared__ int cnt[4];
    const int pb = c / kGrp, x = c % kGrp;
    const int fa = Pr.pb_fa[pb], fb = Pr.pb_fb[pb];
    int kfa = 0, kfb = 0;
    for (int k = 0; k < G.n_kf; ++k) {
        const int f = Pr.free_idx[k];
        if (f == fa) kfa = k;
        if (f == fb) kfb = k;
    }
    const unsigned long long ma = 3ull << (2 * kfa), mb = 3ull << (2 * kfb);
    const unsigned long long below_a = (1ull << (2 * kfa)) - 1ull, below_b = (1ull << (2 * kfb)) - 1ull;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nw = G.n_wave > x ? (G.n_wave - x + kGrp - 1) / kGrp : 0;  // slot waves x + 8k of the group
    const int k0 = nw * wave / 4, k1 = nw * (wave + 1) / 4;
    int4* out = pairs + (size_t)c * G.pair_stride;
    // the run's waves kPairU at a time: their landmark ranges, then the first 64 landmarks' masks
    // and first slots of each, every load of a round in flight together (a wave of more than 64
    // landmarks -- unobserved ones between observed ones -- continues in a loop).  The run's first
    // round (the whole run at config-3 sizes) is loaded once and kept for both passes.
    struct Round {
        int l0[kPairU], l1[kPairU], lbs[kPairU];
        unsigned long long m[kPairU];
    };
    auto load = [&](int kb, Round& R) {
#pragma unroll
        for (int u = 0; u < kPairU; ++u) {
            const int w = x + kGrp * (kb + u);
            const bool in = kb + u < k1;
            R.l0[u] = in ? S.wave_lm[w] : 0;
            R.l1[u] = in ? S.wave_lm[w + 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < kPairU; ++u) {
            const bool in = R.l0[u] + lane < R.l1[u];
            R.m[u] = in ? S.mask[R.l0[u] + lane] : 0ull;
            R.lbs[u] = in ? S.lm_base[R.l0[u] + lane] : 0;
        }
    };
    auto scan = [&](const Round& R, bool write, int& acc) {
#pragma unroll
        for (int u = 0; u < kPairU; ++u) {
            for (int l = R.l0[u] + lane; l - lane < R.l1[u]; l += 64) {
                const bool first = l == R.l0[u] + lane;
                const unsigned long long mm = first ? R.m[u] : (l < R.l1[u] ? S.mask[l] : 0ull);
                const bool has = (mm & ma) && (mm & mb);
                const unsigned long long bal = __ballot(has);
                if (write && has) {
                    const unsigned long long kbits = (mm | (mm >> 1)) & kEvenBits;
                    const int lb = first ? R.lbs[u] : S.lm_base[l];
                    out[acc + __popcll(bal & ((1ull << lane) - 1ull))] =
                        make_int4(lb + __popcll(kbits & below_a), lb + __popcll(kbits & below_b), l, 0);
                }
                acc += __popcll(bal);
            }
        }
    };
    Round R0;
    load(k0, R0);
    int n = 0;  // pass 1: this run's pair count
    scan(R0, false, n);
    for (int kb = k0 + kPairU; kb < k1; kb += kPairU) {
        Round R;
        load(kb, R);
        scan(R, false, n);
    }
    if (lane == 0) cnt[wave] = n;
    __syncthreads();
    int base = 0;
    for (int v = 0; v < wave; ++v) base += cnt[v];
    const int total = cnt[0] + cnt[1] + cnt[2] + cnt[3];
    scan(R0, true, base);  // pass 2
    for (int kb = k0 + kPairU; kb < k1; kb += kPairU) {
        Round R;
        load(kb, R);
        scan(R, true, base);
    }
    for (int i = total + tid; i < G.pair_stride; i += 256) out[i] = make_int4(-1, 0, 0, 0);
}

// set_problem's staging image into the device arena, on the BA's own stream: this kernel reads the
// pinned image over PCIe (8-B system-scope loads: each goes to host memory, nothing stale from an
// earlier window can be served by a cache) instead of an SDMA copy, so ba_build_layout follows it
// in the same queue without the copy engine -> compute queue hand-off (≈ 12 µs between the copy's
// end and the next kernel's start in the traced step, profiles/r06n_traced_step_timeline.txt).
// 16-B words, two per thread (both loads in flight before the stores); the image is a multiple of
// 256 B.  (8-B atomic loads: 10.5 us for the 386 KB window, profiles/r06r_headline_kstats.txt.)
__global__ __launch_bounds__(256) void ba_stage_in(const uint4* src, uint4* __restrict__ dst, int n_words) {
    const int t = (int)(blockIdx.x * 256 + threadIdx.x), st = (int)(gridDim.x * 256);
    const int i0 = t, i1 = t + st;
    uint4 a, b;
    host_load2x16(src + min(i0, n_words - 1), src + min(i1, n_words - 1), a, b);
    if (i0 < n_words) dst[i0] = a;
    if (i1 < n_words) dst[i1] = b;
}

// set_problem's device part in one launch: blocks [0, nb_slots) build the slot layout, the next
// n_chunk blocks the Schur pair lists
__global__ __launch_bounds__(256) void ba_build_layout(Geometry G, Prob Pr, SlotSrc S, int nb_slots, int4* hdr,
                                                       double2* huv, int4* pairs) {
    const int b = blockIdx.x;
    if (b < nb_slots)
        build_slots_body(G, Pr, S, hdr, huv, b);
    else
        build_pairs_body(G, Pr, S, pairs, b - nb_slots);
}

// ---------------------------------------------------------------------------------------
// K4: linearisation of the initial state (buffer 0) -- one wave per landmark group, one lane
// per (landmark, keyframe) slot.  Its cost partials (partA) give the initial cost.
// ---------------------------------------------------------------------------------------
// with_reset: K0 folded in (one kernel boundary less per solve): the grid also copies the
// initial state into both state buffers and initialises the LM state; the linearisation reads
// the initial state directly (the same values K0 copies).
__device__ void linearize_body(const Geometry& G, const Prob& Pr, const Work& Wk, int w, int with_reset,
                               double lambda0) {
    __shared__ double sh[10][64];
    const int lane = threadIdx.x;
    const int s = 64 * w + lane;
    if (with_reset) {
        const int nt = G.n_wave * 64;  // the window's own waves (a batched grid may be wider)
        for (int i = s; i < 7 * G.n_kf; i += nt) {
            Wk.pose[0][i] = Wk.pose_init[i];
            Wk.pose[1][i] = Wk.pose_init[i];
        }
        for (int i = s; i < 3 * G.n_lm; i += nt) {
            Wk.pw[0][i] = Wk.pw_init[i];
            Wk.pw[1][i] = Wk.pw_init[i];
        }
        if (s == 0) {
            Wk.tick[1] = wall_clock64();
            *Wk.singular = 0;
            LmState st{};
            st.lambda = lambda0;
            st.nu = 2.0;
            *Wk.st = st;
        }
    }
    const double* pose0 = with_reset ? Wk.pose_init : Wk.pose[0];
    const double* pw0 = with_reset ? Wk.pw_init : Wk.pw[0];
    const int4 h0 = Pr.slot_hdr[2 * s], h1 = Pr.slot_hdr[2 * s + 1];
    const double2 uvq[2] = {Pr.slot_uv[2 * s], Pr.slot_uv[2 * s + 1]};
    STAMP(11);
    const bool act = h1.y > 0;
    const int kf = h0.x, l = h0.y, first = act ? h0.z : lane, nk = act ? h0.w : 1;
    const bool fr = h1.x >= 0;
    SlotLin L;
    if (act) {
        const Pose P = pose_from7(pose0 + 7 * kf);
        const double* pwp = pw0 + 3 * l;
        const double p[3] = {pwp[0], pwp[1], pwp[2]};
        slot_linearize(G, P, p, h1.y, h1.z, uvq, fr, L);
    } else {
        const Pose P{};
        const double p[3] = {0.0, 0.0, 1.0};
        slot_linearize(G, P, p, 0, 0, uvq, false, L);
    }
    STAMP(12);
    store_linearization(Wk, 0, s, lane, act, fr, first, nk, l, L, sh);
    const double c = wave_sum_det(L.cost);
    if (lane == 0) {
        Wk.partA[w * kPartA] = c;
        Wk.partA[w * kPartA + 1] = 0.0;
    }
    STAMP(14);
}

// (always with the reset folded in: a runtime flag here made the compiler keep 40 B of scratch)
__global__ __launch_bounds__(64) void ba_linearize(Geometry G, Prob Pr, Work Wk, double lambda0) {
    linearize_body(G, Pr, Wk, blockIdx.x, 1, lambda0);
}

// Trial scalars of this rank, one wave: the K6 wave partials (+ |x|^2 of the free poses on the
// owner rank), per-lane strided sums then a fixed-pairing wave reduction; every load is issued
// before the state is read (the free-pose squares of both buffers; the current one is picked
// afterwards).  Result on every lane.  Used by every decision (K4c blocks, K7, K6r), so the
// sharded and single-rank paths reduce in the same order.
__device__ void trial_scalars_wave(const Geometry& G, const Prob& Pr, const Work& Wk, const LmState& s,
                                   int include_poses, double out[4]) {
    const int lane = threadIdx.x & 63;
    // all loads in flight together, branch-free (clamped indices, zeroed after the load): up to
    // 8 wave partials per lane (a tail loop past 512 waves), then the <= 3 pose entries per
    // lane of both state buffers
    constexpr int kU = 8;
    double4 pv[kU];
    const int wl = max(G.n_wave - 1, 0), el = 7 * G.n_kf - 1;
#pragma unroll
    for (int k = 0; k < kU; ++k)
        pv[k] = *reinterpret_cast<const double4*>(Wk.partD + (size_t)min(lane + 64 * k, wl) * kPartD);
    double p0[3], p1[3];
    int fi[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int e = min(lane + 64 * k, el);
        fi[k] = Pr.free_idx[e / 7];
        p0[k] = Wk.pose[0][e];
        p1[k] = Wk.pose[1][e];
    }
#pragma unroll
    for (int k = 0; k < kU; ++k)
        if (lane + 64 * k >= G.n_wave) pv[k] = make_double4(0.0, 0.0, 0.0, 0.0);
    bool fr[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fr[k] = include_poses && lane + 64 * k <= el && fi[k] >= 0;
    double acc[kPartD] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < kU; ++k) {
        acc[0] += pv[k].x;
        acc[1] += pv[k].y;
        acc[2] += pv[k].z;
        acc[3] += pv[k].w;
    }
    for (int i = lane + 64 * kU; i < G.n_wave; i += 64) {
        const double4 v = *reinterpret_cast<const double4*>(Wk.partD + (size_t)i * kPartD);
        acc[0] += v.x;
        acc[1] += v.y;
        acc[2] += v.z;
        acc[3] += v.w;
    }
    double sq[2] = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (fr[k]) {
            sq[0] += p0[k] * p0[k];
            sq[1] += p1[k] * p1[k];
        }
    if (!s.solve_ok)
#pragma unroll
        for (int k = 0; k < kPartD; ++k) acc[k] = 0.0;
    acc[3] += sq[s.cur];
#pragma unroll
    for (int k = 0; k < kPartD; ++k) out[k] = wave_sum_det(acc[k]);
}

// trial_scalars_wave over ALL ranks of the P2P-sharded solve, from the wave partials every rank's
// K6 pushed into this rank's exchange buffer (RSVIO_P2P_FOLD=2): per source rank r, in rank order,
// exactly the per-lane strided sums and the fixed-pairing wave reduction rank r's X2 would have
// computed (+ |x|^2 of the free poses on rank 0, from this rank's identical pose buffers), then
// the rank-ordered sum from 0.0 the exchange would have formed -- the same bits as the X2 path.
// Each lane waits (bounded) for the generation flags of the slots it reads.
__device__ void trial_scalars_p2p(const Geometry& G, const Prob& Pr, const Work& Wk, const LmState& s, const P2P& P,
                                  unsigned long long gen, int* err, double out[4]) {
    const int lane = threadIdx.x & 63, par = (int)(gen & 1);
    double* own = P.peer[P.rank];
    const int el = 7 * G.n_kf - 1;
    double p0[3], p1[3];
    int fi[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int e = min(lane + 64 * k, el);
        fi[k] = Pr.free_idx[e / 7];
        p0[k] = Wk.pose[0][e];
        p1[k] = Wk.pose[1][e];
    }
    double sq[2] = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (lane + 64 * k <= el && fi[k] >= 0) {
            sq[0] += p0[k] * p0[k];
            sq[1] += p1[k] * p1[k];
        }
    for (int j = 0; j < 4; ++j) out[j] = 0.0;
    bool late = false;
    for (int r = 0; r < P.nranks; ++r) {
        const int nw = P.xnw[r];
        double acc[kPartD] = {0.0, 0.0, 0.0, 0.0};
        for (int w = lane; w < max(nw, 512); w += 64) {  // (>= 8 steps: the wave sum's order)
            double4 v = make_double4(0.0, 0.0, 0.0, 0.0);
            if (w < nw) {
                const unsigned long long* f = p2p_tflag(own, par, r, w);
                long long spins = 0;
                while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1ll << 25)) {
                        late = true;
                        break;
                    }
                }
                // relaxed polls (no L2 invalidate per poll), one acquire once the flag is seen
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                const double* q = p2p_tval(own, par, r, w);
                v.x = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                v.y = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                v.z = __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                v.w = __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            acc[0] += v.x;
            acc[1] += v.y;
            acc[2] += v.z;
            acc[3] += v.w;
        }
        if (r == 0) acc[3] += sq[s.cur];
#pragma unroll
        for (int k = 0; k < kPartD; ++k) out[k] += wave_sum_det(acc[k]);
    }
    if (late) atomicExch(err, 1);
}

// The build's LM decision for one iteration: cost = cost at the current
// state, tv = trial cost, |dp|^2, g_p.dp, |x|^2.  Flips the state buffers on acceptance.
__device__ void lm_update(LmState& s, double cost, const double tv[4], int max_iter, double cost_tol,
                          double param_tol) {
    if (s.iter == 0) s.initial_cost = cost;
    s.cost = cost;
    s.iter += 1;
    s.accepted = 0;
    if (!isfinite(cost)) {
        s.status = RSVIO_LM_NUMERICAL_FAILURE;
        s.done = 1;
    } else if (!s.solve_ok) {
        // a singular landmark block or camera system: apex's optimize returns
        // Err(LinearSolveFailed), which SlidingWindow::optimize answers with the SparseCholesky
        // retry, then a revert (sliding_window.rs:326-353)
        s.status = RSVIO_LM_LINEAR_SOLVE_FAILED;
        s.done = 1;
    } else {
        s.new_cost = tv[0];
        s.dp2 = tv[1];
        s.gpdp = tv[2];
        s.x2 = tv[3];
        const double dx2 = s.dc2 + s.dp2;
        const double dxn = sqrt(dx2), xn = sqrt(s.x2);
        if (dxn <= param_tol * (xn + param_tol)) {
            s.status = RSVIO_LM_PARAMETER_TOLERANCE;
            s.done = 1;
        } else {
            const double pred = 0.5 * (s.lambda * dx2 - (s.gcdc + s.gpdp));
            const double dcost = cost - s.new_cost;
            const double rho = dcost / pred;
            if (isfinite(s.new_cost) && fabs(dcost) <= cost_tol * cost) {
                // converged: the candidate's cost change is within the
                // tolerance, whatever its sign, and the candidate is not applied -- so a change
                // at rounding level, whose sign two summation orders may disagree on, decides
                // neither the outcome nor the state.  This build's rule, NOT apex-solver's (absent
                // offline, parity unpinned): a deliberate departure, DESIGN.md section 5
                s.status = RSVIO_LM_COST_TOLERANCE;
                s.done = 1;
            } else if (isfinite(s.new_cost) && rho > 0.0) {
                s.accepted = 1;
                s.cur = 1 - s.cur;  // the trial buffers become current
                const double f = 2.0 * rho - 1.0;
                s.lambda *= fmax(1.0 / 3.0, 1.0 - f * f * f);
                s.nu = 2.0;
                s.cost = s.new_cost;
            } else {
                s.lambda *= s.nu;
                s.nu *= 2.0;
                if (s.lambda > 1e32) {
                    s.status = RSVIO_LM_TRUST_REGION;
                    s.done = 1;
                }
            }
        }
    }
    if (!s.done && s.iter >= max_iter) {
        s.status = RSVIO_LM_MAX_ITERATIONS;
        s.done = 1;
    }
}

// LM configuration passed to the kernels that decide
struct LmArgs {
    int max_iter;
    double cost_tol, param_tol;
};

// The pending decision (the previous iteration's trial), by one whole wave: returns the decided
// state on every lane.  pre_reduced: the trial scalars come from trial4 (all-reduced over ranks),
// else they are this rank's.  The cost of the initial state is sys[SC0] (K5's combine, or the
// sharded combine + all-reduce, wrote it in iteration 0).  Every caller runs the same
// operations on the same data, so every workgroup that decides gets identical bits.
__device__ LmState lm_decide(const Geometry& G, const Prob& Pr, const Work& Wk, const LmState* src, int pre_reduced,
                             const LmArgs& la, const P2P* PP = nullptr, const unsigned long long* xgen = nullptr,
                             int* err = nullptr) {
    LmState s = *src;
    // the trial scalars are gathered whether or not a decision is pending, so their loads are
    // in flight together with the state's (one round trip) -- except from the P2P exchange
    // (pre_reduced 2), which waits for flags only a pending decision has
    double tv[4];
    if (pre_reduced == 4) {
        // fold 4: every rank's 4 scalars, flag-in-word in this rank's X2 slots (K6's last wave
        // pushed them): lane 4 r + i holds rank r's value i; the first read is issued with the
        // state's load, re-polled (bounded) only if a pending decision finds a tag not yet there
        const int lane = threadIdx.x & 63, r = lane >> 2, i = lane & 3, nr = PP->nranks;
        const unsigned long long gen = *xgen;
        const unsigned g32 = (unsigned)gen;
        const unsigned long long* wv = p2p_ll(PP->peer[PP->rank], (int)(gen & 1), min(r, nr - 1)) + 2 * i;
        unsigned long long a = __hip_atomic_load(wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        unsigned long long b = __hip_atomic_load(wv + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int k = 0; k < 4; ++k) tv[k] = 0.0;
        if (s.pending && !s.done && s.solve_ok) {
            long long spins = 0;
            bool late = false;
            while (r < nr && !((unsigned)(a >> 32) == g32 && (unsigned)(b >> 32) == g32)) {
                if (++spins > (1ll << 25)) {
                    late = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                a = __hip_atomic_load(wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                b = __hip_atomic_load(wv + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (late) atomicExch(err, 1);
            const double got = late ? 0.0 : __longlong_as_double((long long)((a & 0xffffffffull) | (b << 32)));
            for (int k = 0; k < 4; ++k) {
                double v = 0.0;
                for (int q = 0; q < nr; ++q) v += rl64(got, 4 * q + k);  // rank order from 0.0: X2's sum
                tv[k] = v;
            }
        }
    } else if (pre_reduced == 2) {
        const unsigned long long gen = *xgen;  // K5 of the iteration that produced the trial
        for (int k = 0; k < 4; ++k) tv[k] = 0.0;
        if (s.pending && !s.done && s.solve_ok) trial_scalars_p2p(G, Pr, Wk, s, *PP, gen, err, tv);
    } else if (pre_reduced) {
        for (int k = 0; k < 4; ++k) tv[k] = Wk.trial4[k];
    } else {
        trial_scalars_wave(G, Pr, Wk, s, 1, tv);
    }
    const double cost0 = Wk.sys[(size_t)G.n_pb * 36 + 12 * G.n_free];
    // keep the compiler from sinking the gathers under the branch below (the state's load and
    // theirs then overlap instead of running back to back)
    __asm__ volatile("" ::"v"(tv[0]), "v"(tv[1]), "v"(tv[2]), "v"(tv[3]), "v"(cost0));
    STAMP(29);
    if (s.pending && !s.done) {
        // cost at the current state: the initial linearisation's at the first iteration, then
        // the cost of the last accepted trial state (K6 evaluated it while linearising it)
        const double cost = s.iter == 0 ? cost0 : s.cost;
        lm_update(s, cost, tv, la.max_iter, la.cost_tol, la.param_tol);
        s.pending = 0;
    }
    return s;
}

// ---------------------------------------------------------------------------------------
// K4c: one 128-thread workgroup per (XCD group x, upper-triangular 6x6 camera block fa <= fb),
// one slot pair per thread (more passes past 128 pairs).  It first takes the pending LM
// decision (every wave redundantly, identical bits; block 0 stores it as this iteration's
// state), then per pair  S_ab -= Y_a W_b^T  with Y = W (V + lambda I)^-1 formed on the fly
// (+ U_a, b_a, g_c,a on diagonal blocks), reduce-scattered over each wave and summed over the
// two waves in a fixed order into slot x of the partial systems.  No atomics and no last
// arriver: K5 (or K4d when sharded) sums the 8 slots.
// ---------------------------------------------------------------------------------------
// One slot pair of a camera block.  DIAG: a diagonal block's pairs are (s, s) (a landmark has
// one slot per keyframe), so W is loaded once and U, g_c join; off-diagonal blocks touch only
// the 36 S entries -- two instantiations keep each one's register footprint to its own needs.
// W (6x3) of a slot from its record: rows 0-2 = Vs (symmetric), rows 3-5 = Wr
__device__ __forceinline__ void slot_w(const double* rec, double W[18]) {
    const double* v = rec + RV;
    const double Vs[9] = {v[0], v[1], v[2], v[1], v[3], v[4], v[2], v[4], v[5]};
#pragma unroll
    for (int i = 0; i < 9; ++i) W[i] = Vs[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) W[9 + i] = rec[RWR + i];
}

template <bool DIAG>
__device__ __forceinline__ void schur_pair(const Work& Wk, int cur, double lambda, int chol, int sa, int sb, int l,
                                           double (&acc)[kBlockF]) {
    const double2* ra = reinterpret_cast<const double2*>(Wk.raws[cur] + (size_t)sa * kRawF);
    const double2* rb = reinterpret_cast<const double2*>(Wk.raws[cur] + (size_t)sb * kRawF);
    const double2* rl = reinterpret_cast<const double2*>(Wk.rawl[cur] + (size_t)l * kLmF);
    // record a: all 28 values on a diagonal block (Ur, gp_s, gr join), else Vs, gp_s, Wr (18)
    constexpr int NA = DIAG ? kRawF / 2 : 9;
    double Ra[2 * NA], Rb[18], Lm[10];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const double2 x = ra[i];
        Ra[2 * i] = x.x; Ra[2 * i + 1] = x.y;
    }
    if constexpr (!DIAG)
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double2 y = rb[i];
            Rb[2 * i] = y.x; Rb[2 * i + 1] = y.y;
        }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const double2 x = rl[i];
        Lm[2 * i] = x.x; Lm[2 * i + 1] = x.y;
    }
    double Wa[18], Wb[18];
    slot_w(Ra, Wa);
    if constexpr (DIAG) {
#pragma unroll
        for (int i = 0; i < 18; ++i) Wb[i] = Wa[i];  // a diagonal block's pairs are (s, s)
    } else {
        slot_w(Rb, Wb);
    }
    double Vi[3][3];
    if (!landmark_inverse(Lm + LV, lambda, Vi, chol)) *Wk.singular = 1;
    double Ya[18];  // Y_a = W_a (V + lambda I)^-1
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            Ya[a * 3 + k] = fma(Wa[a * 3 + 2], Vi[2][k], fma(Wa[a * 3 + 1], Vi[1][k], Wa[a * 3] * Vi[0][k]));
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int k = 0; k < 6; ++k)
            acc[a * 6 + k] -= fma(Ya[a * 3 + 2], Wb[k * 3 + 2], fma(Ya[a * 3 + 1], Wb[k * 3 + 1], Ya[a * 3] * Wb[k * 3]));
    if constexpr (DIAG) {
        // U = [[Vs, Wr^T], [Wr, Ur]] and g_c = [gp_s; gr]
        double U[36];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                U[a * 6 + c] = Wa[a * 3 + c];              // Vs
                U[(3 + a) * 6 + c] = Wa[(3 + a) * 3 + c];  // Wr
                U[c * 6 + 3 + a] = Wa[(3 + a) * 3 + c];    // Wr^T
            }
        const double* ur = Ra + RUR;
        const double Ur[9] = {ur[0], ur[1], ur[2], ur[1], ur[3], ur[4], ur[2], ur[4], ur[5]};
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int c = 0; c < 3; ++c) U[(3 + a) * 6 + 3 + c] = Ur[a * 3 + c];
#pragma unroll
        for (int i = 0; i < 36; ++i) acc[i] += U[i];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double gca = a < 3 ? Ra[RGP + a] : Ra[RGR + a - 3];
            const double yg = fma(Ya[a * 3 + 2], Lm[LG + 2], fma(Ya[a * 3 + 1], Lm[LG + 1], Ya[a * 3] * Lm[LG]));
            acc[36 + a] += yg - gca;  // b = -g_c + sum Y g_p
            acc[42 + a] += gca;
        }
    }
}

template <bool DIAG>
__device__ __forceinline__ void schur_chunk_pairs(const Geometry& G, const Work& Wk, const LmState& s, const int4* pr,
                                                  int4 p1, int tid, double (&acc)[kBlockF]) {
    if (p1.x >= 0) schur_pair<DIAG>(Wk, s.cur, s.lambda, G.chol, p1.x, p1.y, p1.z, acc);
    for (int p = tid + kSchurThreads; p < G.pair_stride; p += kSchurThreads) {  // > 512 pairs per group
        const int4 q = pr[p];
        if (q.x >= 0) schur_pair<DIAG>(Wk, s.cur, s.lambda, G.chol, q.x, q.y, q.z, acc);
    }
}

__device__ void schur_chunks_body(const Geometry& G, const Prob& Pr, const Work& Wk, const LmArgs& la,
                                  int pre_reduced, int c, const P2P* PP = nullptr,
                                  const unsigned long long* xgen = nullptr, int* err = nullptr) {
    __shared__ double red[kSchurThreads / 64][kBlockF];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int pb = c / kGrp, x = c % kGrp;
    RTSTAMP(0);
    STAMP(26);
    if (G.env_on) {
        // a camera block outside the system's envelope (no landmark sees both keyframes: a window
        // of landmarks over consecutive keyframes, config 5) has no pair: its partial is zero and
        // needs no decision -- a third of config 5's 1,520 chunks.  (fa, fb) from pb by the host's
        // enumeration (pb_fa / pb_fb: a-major, b >= a), without a load
        int a = 0, r = pb;
        while (a < G.n_free && r >= G.n_free - a) {
            r -= G.n_free - a;
            ++a;
        }
        if (a < G.n_free && a + r > (int)G.env[a]) {
            if (tid < 36) Wk.cpart[(size_t)x * sys_len(G) + pb * 36 + tid] = 0.0;
            return;
        }
    }
    // this chunk's pairs sit at a fixed stride: the first pair of every thread is one load,
    // issued together with the decision's loads
    const int4* pr = Pr.pairs + (size_t)c * G.pair_stride;
    const int4 p1 = tid < G.pair_stride ? pr[tid] : make_int4(-1, 0, 0, 0);
    const int fa = Pr.pb_fa[pb];
    const bool diag = fa == Pr.pb_fb[pb];
    // the decision by wave 0, handed to the other waves through LDS (a quarter of the loads)
    __shared__ LmState sd;
    STAMP(27);
    if (wave == 0) {
        const LmState d = lm_decide(G, Pr, Wk, Wk.st_prev, pre_reduced, la, PP, xgen, err);
        STAMP(28);
        if (lane == 0) {
            sd = d;
            if (c == 0) *Wk.st = d;
        }
    }
    __syncthreads();
    const LmState s = sd;
    if (s.done) return;
    STAMP(16);
    RTSTAMP(1);
    double acc[kBlockF];
#pragma unroll
    for (int i = 0; i < kBlockF; ++i) acc[i] = 0.0;
    if (diag)
        schur_chunk_pairs<true>(G, Wk, s, pr, p1, tid, acc);
    else
        schur_chunk_pairs<false>(G, Wk, s, pr, p1, tid, acc);
    STAMP(17);
    wave_reduce_scatter<3>(acc, lane);
    if ((lane & 3) == 0)
#pragma unroll
        for (int j = 0; j < 3; ++j) red[wave][3 * (lane >> 2) + j] = acc[j];
    __syncthreads();
    if (tid < (diag ? kBlockF : 36)) {
        double v = red[0][tid];
#pragma unroll
        for (int w = 1; w < kSchurThreads / 64; ++w) v += red[w][tid];
        const int SB0 = G.n_pb * 36, SG0 = SB0 + 6 * G.n_free;
        const int e = tid < 36 ? pb * 36 + tid : (tid < 42 ? SB0 + 6 * fa + tid - 36 : SG0 + 6 * fa + tid - 42);
        Wk.cpart[(size_t)x * sys_len(G) + e] = v;
    }
    STAMP(18);
    RTSTAMP(2);
}

__global__ __launch_bounds__(kSchurThreads) void ba_schur_chunks(Geometry G, Prob Pr, Work Wk, LmArgs la,
                                                                  int pre_reduced) {
    schur_chunks_body(G, Pr, Wk, la, pre_reduced, blockIdx.x);
}

// K4c of the P2P-sharded iteration with the trial-scalar exchange folded in (RSVIO_P2P_FOLD=2):
// the pending decision from every rank's K6 wave partials in this rank's exchange buffer
// (mode 4, fold 4: from the 4 scalars per rank K6's last wave pushed)
__global__ __launch_bounds__(kSchurThreads) void ba_schur_chunks_p2p(Geometry G, Prob Pr, Work Wk, LmArgs la, P2P P,
                                                                      const unsigned long long* xgen, int* err,
                                                                      int mode) {
    schur_chunks_body(G, Pr, Wk, la, mode, blockIdx.x, &P, xgen, err);
}

// The reduced system of this rank into dst (sys layout): S, b, g_c summed over the kGrp partial
// systems in slot order (+ lambda on the diagonal of diagonal blocks when add_lambda), then the
// cost of the initial linearisation (K4 wave partials, fixed order) and the singular-landmark
// flag of this iteration's K4c.  Every load is coalesced and independent of any other.  Whole
// block (T threads).
template <int T>
__device__ void combine_system(const Geometry& G, const Prob& Pr, const Work& Wk, double* dst, double lambda,
                               bool add_lambda) {
    const int n_e = G.n_pb * 36 + 12 * G.n_free;
    const size_t L = sys_len(G);
    // the K4 wave partials (initial cost) and the singular flag are loaded first, with the
    // partial systems: one round trip for everything
    constexpr int kU = 16;  // all in flight (a tail loop past 1024 waves)
    const int lane = threadIdx.x;
    double pa[kU];
    int sing = 0;
    if (lane < 64) {
#pragma unroll
        for (int k = 0; k < kU; ++k) pa[k] = lane + 64 * k < G.n_wave ? Wk.partA[(lane + 64 * k) * kPartA] : 0.0;
        sing = *Wk.singular;
    }
    // rounds of kE entries per thread, every load of a round issued before any is consumed
    constexpr int kE = 8;
    for (int e0 = 0; e0 < n_e; e0 += T * kE) {
        double v[kE][kGrp];
#pragma unroll
        for (int i = 0; i < kE; ++i) {
            const int e = e0 + threadIdx.x + T * i;
#pragma unroll
            for (int x = 0; x < kGrp; ++x) v[i][x] = e < n_e ? Wk.cpart[(size_t)x * L + e] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < kE; ++i) {
            const int e = e0 + threadIdx.x + T * i;
            if (e >= n_e) break;
            double a = v[i][0];
#pragma unroll
            for (int x = 1; x < kGrp; ++x) a += v[i][x];
            dst[e] = a;
        }
    }
    if (add_lambda) {  // + lambda on the diagonal of each diagonal block (f, f), after its sum
        __syncthreads();
        for (int t = threadIdx.x; t < 6 * G.n_free; t += T) {
            const int f = t / 6, k = t % 6;
            dst[(f * G.n_free - f * (f - 1) / 2) * 36 + 7 * k] += lambda;
        }
    }
    if (lane < 64) {
        double c = 0.0;
#pragma unroll
        for (int k = 0; k < kU; ++k) c += pa[k];
        for (int w = lane + 64 * kU; w < G.n_wave; w += 64) c += Wk.partA[w * kPartA];
        c = wave_sum_det(c);
        if (lane == 0) {
            dst[n_e] = c;
            dst[n_e + 1] = sing ? 1.0 : 0.0;
            Wk.sys[n_e] = c;  // the decision of iteration 0 reads the initial cost here
        }
    }
}

// K4d (sharded path, and build_system): the rank's reduced system into sys (+ lambda on the
// owner rank), ready for the all-reduce; clears the singular flag.
__global__ __launch_bounds__(256) void ba_schur_combine(Geometry G, Prob Pr, Work Wk, int lambda_owner) {
    const LmState* st = Wk.st;
    if (st->done) return;
    STAMP(19);
    combine_system<256>(G, Pr, Wk, Wk.sys, st->lambda, lambda_owner != 0);
    __syncthreads();
    if (threadIdx.x == 0) *Wk.singular = 0;
}

// K4d-wide (single rank, 11..20 free keyframes, round 6): the 8 partial systems summed into sys
// by many workgroups -- one entry per thread, the partials in slot order then + lambda on the
// diagonal, exactly combine_system's operations -- so the camera solve's one workgroup pulls one
// system (55 KB at W=20) instead of eight (440 KB: 28k of K5's 128k cycles, one CU's bandwidth,
// profiles/r06c_c5_k5_stamps.txt).  Block 0 also sums the initial cost (K4's wave partials, as
// combine_system) and copies the singular flag; K5 then reads sys through the map (combine = 0).
__global__ __launch_bounds__(256) void ba_schur_combine_wide(Geometry G, Prob Pr, Work Wk) {
    const LmState* st = Wk.st;
    if (st->done) return;
    const int n_e = G.n_pb * 36 + 12 * G.n_free;
    const size_t L = sys_len(G);
    const int e = blockIdx.x * 256 + threadIdx.x;
    constexpr int kU = 16;
    const int lane = threadIdx.x;
    double pa[kU];
    int sing = 0;
    if (blockIdx.x == 0 && lane < 64) {
#pragma unroll
        for (int k = 0; k < kU; ++k) pa[k] = lane + 64 * k < G.n_wave ? Wk.partA[(lane + 64 * k) * kPartA] : 0.0;
        sing = *Wk.singular;
    }
    const double lambda = st->lambda;
    if (e < n_e) {
        double v[kGrp];
#pragma unroll
        for (int x = 0; x < kGrp; ++x) v[x] = Wk.cpart[(size_t)x * L + e];
        double a = v[0];
#pragma unroll
        for (int x = 1; x < kGrp; ++x) a += v[x];
        // a diagonal entry (k, k) of a diagonal camera block (f, f): pb = f n - f (f - 1) / 2
        const int pb = e / 36, k = e % 36;
        if (pb < G.n_pb && k % 7 == 0 && Pr.pb_fa[pb] == Pr.pb_fb[pb]) a += lambda;
        Wk.sys[e] = a;
    }
    if (blockIdx.x == 0 && lane < 64) {
        double c = 0.0;
#pragma unroll
        for (int k = 0; k < kU; ++k) c += pa[k];
        for (int w = lane + 64 * kU; w < G.n_wave; w += 64) c += Wk.partA[w * kPartA];
        c = wave_sum_det(c);
        if (lane == 0) {
            Wk.sys[n_e] = c;  // the decision of iteration 0 reads the initial cost here
            Wk.sys[n_e + 1] = sing ? 1.0 : 0.0;
        }
    }
}

// ---------------------------------------------------------------------------------------
// K5: camera system solve (one workgroup of 256):
//   n <= 60 (<= 10 free keyframes): pipelined 4-wave register LDL^T of [S; b^T] (chol_pipe)
//     straight from sys, unit-L back substitution by wave 0; |dc|^2, g_c.dc; SE3 (+) trial poses.
//   n > 60: ba_camera_solve_x2 below (two rows per lane, 8 waves).
// ---------------------------------------------------------------------------------------




// Pipelined 4-wave LDL^T of the augmented system [S; b^T]: wave WV owns the contiguous columns
// [WV*CW, WV*CW + CW) of every row (lane = row; lane NP = b).  A wave first consumes the
// columns of the waves before it (waits on an LDS progress counter, then rank-1 updates its own
// columns) and then factors its own columns, publishing each finished column to LDS: the unit
// L column (Lc, kept for the back substitution) and the unscaled column D L (Uc, which the
// updates use).  No barrier: one wave's serial pivot chain (pivot -> 1/d -> next pivot, from
// registers) overlaps the trailing updates of the waves after it.  LDL^T needs no square root,
// which shortens that chain; row NP ends as z = D^-1 L^-1 b.
constexpr int kLcLd = 65;

template <int NP, int CW, int WV, int K>
__device__ __forceinline__ void chol_pipe_step(double (&a)[CW], int lane, double* Lc, double* Uc, int* progress,
                                               int& seen, bool& bad, double inv, double (&uq)[CW], double lp) {
    constexpr int c0 = WV * CW;
    constexpr int c1 = (c0 + CW < NP) ? c0 + CW : NP;
    constexpr int KN = (K + 1 < c0) ? K + 2 : K + 1;  // consume columns in pairs
    if constexpr (K < c0) {
        // consume columns K (.. KN-1) of earlier waves (the LDS counter is re-read only when behind)
        if (seen < KN) {
            do {
                seen = __hip_atomic_load(progress, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (seen >= KN) break;
                __builtin_amdgcn_s_sleep(1);
            } while (true);
        }
        const double lr = Lc[K * kLcLd + lane];
        const double* u = Uc + K * kLcLd;
        if constexpr (KN == K + 2) {
            const double lr2 = Lc[(K + 1) * kLcLd + lane];
            const double* u2 = Uc + (K + 1) * kLcLd;
            double v1[CW], v2[CW];
#pragma unroll
            for (int jj = 0; jj < CW; ++jj) {
                v1[jj] = u[c0 + jj];
                v2[jj] = u2[c0 + jj];
            }
#pragma unroll
            for (int jj = 0; jj < CW; ++jj)
                if (c0 + jj < NP) a[jj] = fma(-lr2, v2[jj], fma(-lr, v1[jj], a[jj]));
        } else {
#pragma unroll
            for (int jj = 0; jj < CW; ++jj)
                if (c0 + jj < NP) a[jj] = fma(-lr, u[c0 + jj], a[jj]);
        }
        if constexpr (KN == c0) {  // first own pivot
            const double piv = rl64(a[0], c0);
            bad |= !(piv > 0.0) || !isfinite(piv);
            inv = rcp_f64(piv);
        }
    } else if constexpr (K < c1) {
        // own column K (inv = 1/d_K ready); the next pivot comes straight from registers (on
        // lane K+1, L[K+1][K] and (DL)[K+1][K] are its own values), so its 1/d chain overlaps
        // this column's trailing FMAs
        constexpr int j = K - c0;
#ifdef RSVIO_STAMPS
        if (K == c0 && lane == 0) g_dbg[28 + WV] = (unsigned long long)clock64();
#endif
        // publish column K-1: a relaxed store behind a compiler barrier -- a wave's LDS operations
        // are performed in order, so a consumer that reads the counter reads the column after
        // it, and no wait for this wave's outstanding LDS operations stalls the pivot chain
        if constexpr (K > c0) {
            __asm__ volatile("" ::: "memory");
            __hip_atomic_store(progress, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const double uk = a[j];
        const double l = uk * inv;
        a[j] = l;
        Lc[K * kLcLd + lane] = l;
        Uc[K * kLcLd + lane] = uk;
        double piv = 1.0;
        if constexpr (j + 1 < CW && K + 1 < NP) {
            // column K+1 by readlane (no LDS round trip on the pivot chain)
            a[j + 1] = fma(-l, rl64(uk, K + 1), a[j + 1]);
            piv = rl64(a[j + 1], K + 1);
        }
        // column K+2 by readlane too: it is the next step's pivot-path column
        if constexpr (j + 2 < CW && K + 2 < NP) a[j + 2] = fma(-l, rl64(uk, K + 2), a[j + 2]);
        if constexpr (j + 1 < CW && K + 1 < NP) {
            bad |= !(piv > 0.0) || !isfinite(piv);
            inv = rcp_f64(piv);
        }
        // the next reciprocal is issued before anything below touches LDS results
        __builtin_amdgcn_sched_barrier(0);
        // software-pipelined rest of the own block: the previous column's updates of columns
        // >= j + 2, from U values read from LDS one step ago (landed by now), then this column's
        // U values for columns >= j + 3 are read for the next step -- a readlane pair per value
        // plus its SGPR hazard wait cost ~4x the issue slots, and an LDS read consumed in the
        // same step puts its latency on the chain
        if constexpr (K > c0) {
#pragma unroll
            for (int jj = j + 2; jj < CW; ++jj)
                if (c0 + jj < NP) a[jj] = fma(-lp, uq[jj], a[jj]);
        }
        {
            const double* uK = Uc + K * kLcLd;
#pragma unroll
            for (int jj = j + 3; jj < CW; ++jj) uq[jj] = c0 + jj < NP ? uK[c0 + jj] : 0.0;
        }
        lp = l;
        if constexpr (K + 1 == c1) {
            __asm__ volatile("" ::: "memory");
            __hip_atomic_store(progress, K + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    // consume steps: materialise the updates here (keeps the compiler from sinking the FMAs
    // past the next wait loop, which would keep every loaded column alive)
    if constexpr (K < c0) {
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) __asm__ volatile("" : "+v"(a[jj]));
    }
    constexpr int KNEXT = (K < c0) ? KN : K + 1;
    if constexpr (KNEXT < c1) chol_pipe_step<NP, CW, WV, KNEXT>(a, lane, Lc, Uc, progress, seen, bad, inv, uq, lp);
}

// Element (r, c), c <= r < n, of the lower triangle of S in the packed block layout of sys
// (upper camera blocks fa <= fb, block-major a-then-b; a diagonal block keeps its own lower
// triangle, an off-diagonal one is read transposed).  row == n: b.
template <int NF>
__device__ __forceinline__ const double* sys_lower(const double* sys, int r, int c) {
    constexpr int n = 6 * NF;
    if (r == n) return sys + (NF * (NF + 1) / 2) * 36 + c;
    const int a = c / 6, b = r / 6;
    const int pb = a * NF - a * (a - 1) / 2 + (b - a);
    const int k = (a == b) ? (r % 6) * 6 + (c % 6) : (c % 6) * 6 + (r % 6);
    return sys + pb * 36 + k;
}

template <int NP, int CW, int WV>
__device__ void chol_pipe(const double* sys, double* Lc, double* Uc, int* progress, int* badw, int lane) {
    constexpr int c0 = WV * CW;
    double a[CW];
    // this wave's columns of every row straight from sys (one round trip): row lane < NP of S,
    // row NP = b, the rest zero
#pragma unroll
    for (int jj = 0; jj < CW; ++jj) {
        const int c = c0 + jj;
        a[jj] = (c < NP && lane <= NP && (c <= lane || lane == NP)) ? *sys_lower<NP / 6>(sys, lane, c) : 0.0;
    }
    bool bad = false;
    if constexpr (c0 < NP) {
        double inv = 0.0;
        if constexpr (c0 == 0) {
            const double piv = rl64(a[0], 0);
            bad = !(piv > 0.0) || !isfinite(piv);
            inv = rcp_f64(piv);
        }
        int seen = 0;
        double uq[CW];
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) uq[jj] = 0.0;
        chol_pipe_step<NP, CW, WV, 0>(a, lane, Lc, Uc, progress, seen, bad, inv, uq, 0.0);
    }
    if (lane == 0) badw[WV] = bad ? 1 : 0;
#ifdef RSVIO_STAMPS
    if (lane == 0) g_dbg[24 + WV] = (unsigned long long)clock64();
#endif
}

// K5's result in this iteration's state: the step (or its failure) is pending a decision
__device__ __forceinline__ void k5_result(LmState* st, int ok, double d2, double gd) {
    st->solve_ok = ok;
    st->dc2 = d2;
    st->gcdc = gd;
    st->pending = 1;
}

// K5's tail (wave 0): dc = x, |dc|^2, g_c.dc, trial poses by SE3 (+) from the prefetched
// current poses, the state's step fields.  A[0..n) is LDS scratch for dc.
template <int NF>
__device__ void k5_finish(const Geometry& G, const Work& Wk, double* A, double x, double gcl_v, int n, int lane,
                          const double (&p7)[7], int fidx) {
    LmState* st = Wk.st;
    const double d2 = wave_sum_det(x * x);
    const double gd = wave_sum_det(lane < n ? gcl_v * x : 0.0);
    __builtin_amdgcn_wave_barrier();
    if (lane < n) {
        Wk.dc[lane] = x;
        A[lane] = x;
    }
    // the LDS copy visible to the wave (lgkmcnt only: waiting for the dc store's acknowledgement
    // as well, s_waitcnt 0, put a memory round trip before the trial poses)
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    STAMP(4);
    if (lane < G.n_kf) {  // trial poses from the prefetched current poses
        double* q = Wk.pose[1 - st->cur] + 7 * lane;
        if (fidx < 0) {
#pragma unroll
            for (int i = 0; i < 7; ++i) q[i] = p7[i];
        } else {
            double qv[7];
            se3_plus(p7, A + 6 * fidx, qv);
#pragma unroll
            for (int i = 0; i < 7; ++i) q[i] = qv[i];
        }
    }
    STAMP(5);
    if (lane == 0) k5_result(st, 1, d2, gd);
    STAMP(6);
}

template <int NF>
__device__ void camera_solve_w4(const Geometry& G, const Prob& Pr, const Work& Wk, const double* sys, double* A,
                                int* badw, int* progress, int n, int tid, const double (&p7)[7], int fidx) {
    constexpr int NP = 6 * NF, CW = (NP + 3) / 4;
    const int lane = tid & 63, wave = tid >> 6;
    LmState* st = Wk.st;
    const double gcl_v = (wave == 0 && lane < n) ? sys[(NF * (NF + 1) / 2) * 36 + 6 * NF + lane] : 0.0;  // g_c
    // Lc / Uc in A's LDS past its first 128 doubles (A[0..n) holds dc for the pose updates)
    double* Lc = A + 128;
    double* Uc = Lc + NP * kLcLd;
    switch (wave) {
        case 0: chol_pipe<NP, CW, 0>(sys, Lc, Uc, progress, badw, lane); break;
        case 1: chol_pipe<NP, CW, 1>(sys, Lc, Uc, progress, badw, lane); break;
        case 2: chol_pipe<NP, CW, 2>(sys, Lc, Uc, progress, badw, lane); break;
        default: chol_pipe<NP, CW, 3>(sys, Lc, Uc, progress, badw, lane); break;
    }
    __syncthreads();
    if (wave != 0) return;
    if (badw[0] | badw[1] | badw[2] | badw[3]) {
        if (lane == 0) k5_result(st, 0, 0.0, 0.0);
        return;
    }
    STAMP(7);
    const int li = lane < NP ? lane : 0;
    const double* Li = Lc + li * kLcLd;  // column li of L: L[j][li] for j >= li, y_li at row NP
    double yv = Li[NP];
    double lt[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) lt[j] = Li[j];
#pragma unroll
    for (int j = NP - 1; j >= 0; --j) {  // L^T x = z (unit diagonal)
        const double xj = rl64(yv, j);
        const double upd = fma(-lt[j], xj, yv);
        yv = lane < j ? upd : yv;
    }
    STAMP(3);
    k5_finish<NF>(G, Wk, A, lane < n ? yv : 0.0, gcl_v, n, lane, p7, fidx);
}

// K5 alternative (A/B, RSVIO_K5=gj1): one wave, Gauss-Jordan on [S | b] with lane = row and
// the full symmetric rows in registers -- no inter-wave hand-off and no back substitution (each
// pivot also eliminates upward; x_i = b'_i / d_i at the end).  Pivot K: l_i = a_iK / d_K (0 on
// the pivot row), a_ij -= l_i A[j][K] for j > K (the trailing block is symmetric, so the pivot
// row's entries are column K's, written to LDS by every lane in one store and read back as
// broadcasts), b_i -= l_i b_K.  The next pivot's column uses readlanes (no LDS round trip on
// the 1/d chain); the other columns get the previous pivot's update one step late, from LDS
// reads issued a step earlier.  (Tolerance parity like the pipelined LDL^T: same pivots, a
// different elimination order.)
constexpr int kGjLd = 65;

template <int NP, int K>
__device__ __forceinline__ void gj1_pivot(double (&a)[NP + 1], double (&uq)[NP], double* U, int lane, bool& bad,
                                          double inv, double lp) {
    if constexpr (K >= 1 && K + 1 < NP) a[K + 1] = fma(-lp, uq[K + 1], a[K + 1]);  // pivot K-1, deferred
    const double aK = a[K];
    const double l = lane == K ? 0.0 : aK * inv;
    U[K * kGjLd + lane] = aK;
    const double ub = rl64(a[NP], K);
    double inv_next = 1.0;
    if constexpr (K + 1 < NP) {
        a[K + 1] = fma(-l, rl64(aK, K + 1), a[K + 1]);
        const double piv = rl64(a[K + 1], K + 1);
        bad |= !(piv > 0.0) || !isfinite(piv);
        inv_next = rcp_f64(piv);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (K >= 1)
#pragma unroll
        for (int j = K + 2; j < NP; ++j) a[j] = fma(-lp, uq[j], a[j]);
    {
        const double* uK = U + K * kGjLd;
#pragma unroll
        for (int j = K + 2; j < NP; ++j) uq[j] = uK[j];
    }
    a[NP] = fma(-l, ub, a[NP]);
    if constexpr (K + 1 < NP) gj1_pivot<NP, K + 1>(a, uq, U, lane, bad, inv_next, l);
}

// wave 0 of the K5 block; U: NP x kGjLd doubles of LDS.  Returns x_lane (0 past n); bad if a
// pivot is not > 0.
template <int NF>
__device__ double camera_solve_gj1(const double* sys, double* U, int lane, bool& bad) {
    constexpr int NP = 6 * NF;
    double a[NP + 1];
#pragma unroll
    for (int j = 0; j < NP; ++j)
        a[j] = lane < NP ? (j <= lane ? *sys_lower<NF>(sys, lane, j) : *sys_lower<NF>(sys, j, lane)) : 0.0;
    a[NP] = lane < NP ? *sys_lower<NF>(sys, NP, lane) : 0.0;
    double uq[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) uq[j] = 0.0;
    const double piv0 = rl64(a[0], 0);
    bad = !(piv0 > 0.0) || !isfinite(piv0);
    gj1_pivot<NP, 0>(a, uq, U, lane, bad, rcp_f64(piv0), 0.0);
    __builtin_amdgcn_wave_barrier();
    return lane < NP ? a[NP] / U[lane * kGjLd + lane] : 0.0;
}

template <int NF>
constexpr size_t k5_lds_doubles() { return 128 + 2 * 6 * NF * kLcLd; }
template <int NF>
constexpr size_t k5_sys_doubles() { return (size_t)(NF * (NF + 1) / 2) * 36 + 12 * NF + 2; }

// K5 body (one 256-thread block); A: k5_lds_doubles<NF>() of LDS, Ls: k5_sys_doubles<NF>().
// combine (single rank): the reduced system is first summed from K4c's chunk partials into Ls
// (+ lambda on the diagonal); sharded: it is the all-reduced sys.  Every write of its results
// (dc, trial poses, the state's solve_ok/dc2/gcdc/pending) is made by wave 0.
template <int NF>
__device__ void k5_body(const Geometry& G, const Prob& Pr, const Work& Wk, double* A, double* Ls, int combine,
                        int variant) {
    static_assert(NF >= 1 && NF <= 10, "one row per lane: n <= 60");
    __shared__ int badw[4];
    __shared__ int progress;
    __shared__ int fail;
    LmState* st = Wk.st;
    if (st->done) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nF = G.n_free, n = 6 * nF;
    const int SC0 = G.n_pb * 36 + 12 * nF;
    const int cur = st->cur;
    // the trial-pose inputs of wave 0 are fetched now, behind the fill
    double p7[7] = {0, 0, 0, 1, 0, 0, 0};
    int fidx = -1;
    if (wave == 0 && lane < G.n_kf) {
        fidx = Pr.free_idx[lane];
#pragma unroll
        for (int i = 0; i < 7; ++i) p7[i] = Wk.pose[cur][7 * lane + i];
    }
    STAMP(0);
    const double* sys = Wk.sys;
    if (combine) {  // all kK5Threads threads pull the partial systems (more loads in flight)
        combine_system<kK5Threads>(G, Pr, Wk, Ls, st->lambda, true);
        sys = Ls;
    }
    __syncthreads();
    if (tid == 0) {
        // a landmark block was singular (sharded: summed over ranks by K4d + all-reduce;
        // single rank: K4c's flag, cleared here for the next iteration)
        fail = (sys[SC0 + 1] != 0.0 || *Wk.singular) ? 1 : 0;
        *Wk.singular = 0;
        progress = 0;
    }
    __syncthreads();
    STAMP(1);
    if (wave >= 4) return;  // the solve is the first 4 waves' (exited waves leave the barriers)
    if (fail) {
        if (tid == 0) k5_result(st, 0, 0.0, 0.0);
        return;
    }
    STAMP(2);
    // the one-wave variant is instantiated up to 9 free keyframes (config 3): at 10 its full
    // rows no longer fit the register file
    if (NF > 9 || variant == 0) {
        camera_solve_w4<NF>(G, Pr, Wk, sys, A, badw, &progress, n, tid, p7, fidx);
        return;
    }
    if constexpr (NF <= 9) {
        if (wave != 0) return;
        const double gcl_v = lane < n ? sys[(NF * (NF + 1) / 2) * 36 + 6 * NF + lane] : 0.0;  // g_c
        bool bad = false;
        const double x = camera_solve_gj1<NF>(sys, A + 128, lane, bad);
        STAMP(7);
        if (bad) {
            if (lane == 0) k5_result(st, 0, 0.0, 0.0);
            return;
        }
        k5_finish<NF>(G, Wk, A, x, gcl_v, n, lane, p7, fidx);
    }
}

template <int NF>
__global__ __launch_bounds__(kK5Threads) void ba_camera_solve(Geometry G, Prob Pr, Work Wk, int combine, int variant) {
    // A[0..128): dc for the pose updates; then the L and D L columns of chol_pipe
    __shared__ __attribute__((aligned(16))) double A[k5_lds_doubles<NF>()];
    __shared__ double Ls[k5_sys_doubles<NF>()];
    RTSTAMP(4);
    k5_body<NF>(G, Pr, Wk, A, Ls, combine, variant);
    RTSTAMP(5);
}

// ---------------------------------------------------------------------------------------
// K5 on the matrix cores (n <= 60; RSVIO_K5=mfma): blocked right-looking
// LDL^T of the camera system with 16-column panels.  The system (padded to NPP = 16 ceil(n/16)
// with identity rows / columns, which couple to nothing) sits column-major in LDS.  Per panel:
//   * wave 0 (lane = row) factors the panel's columns in registers -- per pivot K the 1/d_K
//     chain (v_rcp_f64 + the folded Newton step), l = u / d_K, the in-panel updates from
//     readlanes of the unscaled column, and b_i -= l_iK b_K (so b ends as L^-1 b) -- and writes
//     L into the panel's columns of M, U = D L into Up;
//   * every wave then updates its share of the trailing lower tiles (I, J > panel) with
//     v_mfma_f64_16x16x4_f64: C_IJ += (-U_I) L_J^T over the panel's 16 columns (4 MFMAs per
//     tile, accumulator in registers, C loaded from / stored to M).
// The serial chain is the pivots inside the panels; the O(n^3) trailing work runs on the matrix
// cores, off wave 0's chain.  z = D^-1 L^-1 b, then L^T x = z by wave 0 (readlanes, as pipe4).
// Tolerance parity like pipe4 (same pivots; the trailing sums reassociated by the MFMA).
// ---------------------------------------------------------------------------------------
typedef double mf_dbl4 __attribute__((ext_vector_type(4)));
constexpr int kMfLd = 65;  // f64 leading dimension of the LDS matrices (odd: column reads spread banks)
constexpr int kBkLd = 129;  // the same for the 6x6-block solver past 10 free keyframes (up to 121 rows)
// the block solver's instantiations past 10 free keyframes (a window pads up to the next one)
inline int bk_template_nf(int n_free) { return n_free <= 13 ? 13 : n_free <= 16 ? 16 : 20; }
constexpr int kMfPanel = 8;  // panel width: 8 pivots of in-panel VALU work between matrix-core updates

// The augmented system [[S, .], [b^T, .]] padded to NPP = 16 NT >= NP + 1 rows: row NP is b, so
// eliminating the augmented matrix turns row NP into z^T = (D^-1 L^-1 b)^T on the fly (one more
// row of every panel).  Rows past NP are never initialised: elimination is row-local (a row's
// update uses its own multiplier and the pivot rows' values), so they cannot leak into the
// result; the same holds for the upper halves of the diagonal tiles.
template <int NF>
struct MfDims {
    static constexpr int NP = 6 * NF;
    static constexpr int NT = NP / 16 + 1;
    static constexpr int NPP = 16 * NT;
    static constexpr int NH = (NP + kMfPanel - 1) / kMfPanel;  // panels
};

// Per packed-system entry (sys layout: n_pb x 36 S | 6 n_free b | 6 n_free g_c) its destination
// in K5's LDS: >= 0 a column-major position of M (bit 30: + lambda after the sum), -1 none (the
// upper half of a diagonal block), -2 - i the i-th g_c.  Built on the host per problem.
constexpr int kMfMapLambda = 1 << 30;
inline void mf_dense_map(int nf, int n_pb, const int* pb_fa, const int* pb_fb, int* map, int np_target = 0,
                         int ld = kMfLd) {
    const int np = np_target > 0 ? np_target : 6 * nf;  // the b row (the template's NP)
    for (int pb = 0; pb < n_pb; ++pb)
        for (int k = 0; k < 36; ++k) {
            const int ra = k / 6, ca = k % 6, fa = pb_fa[pb], fb = pb_fb[pb];
            int v;
            if (fa == fb)
                v = ra >= ca ? ((6 * fa + ca) * ld + 6 * fa + ra) | (ra == ca ? kMfMapLambda : 0) : -1;
            else
                v = (6 * fa + ra) * ld + 6 * fb + ca;  // S[6fa+ra][6fb+ca] -> its lower mirror
            map[36 * pb + k] = v;
        }
    for (int i = 0; i < 6 * nf; ++i) map[36 * n_pb + i] = i * ld + np;  // b_i -> row NP, column i
    for (int i = 0; i < 6 * nf; ++i) map[36 * n_pb + 6 * nf + i] = -2 - i;
}

// combine_system with the sums scattered straight into M (and g_c into gsh) by the map
// The partial systems' loads are issued before the LM state's (whose done flag decides whether
// anything is stored and whose lambda joins the diagonal), so the state's round trip overlaps
// theirs.  Returns the state's done flag (nothing stored then).
template <int NF>
__device__ bool combine_mapped(const Geometry& G, const Prob& Pr, const Work& Wk, double* M, double* gsh,
                               const LmState* st, int* fail) {
    constexpr int NE = (NF * (NF + 1) / 2) * 36 + 12 * NF;  // the template's (upper bound)
    constexpr int T = kK5Threads, kE = (NE + T - 1) / T;
    const size_t L = sys_len(G);
    const int ne = G.n_pb * 36 + 12 * G.n_free;  // this window's entries (batched: may be fewer)
    const int tid = threadIdx.x;
    double v[kE][kGrp];
    int dst[kE];
#pragma unroll
    for (int i = 0; i < kE; ++i) {  // (branch-free: clamped loads; an entry past ne is never stored)
        const int e = tid + T * i, ec = min(e, ne - 1);
        const int d = Pr.dmap[ec];
        dst[i] = e < ne ? d : -1;
#pragma unroll
        for (int x = 0; x < kGrp; ++x) v[i][x] = Wk.cpart[(size_t)x * L + ec];
    }
    // then the K4 wave partials (initial cost) and the singular flag, behind them (branch-free:
    // clamped loads, the ones past the last wave dropped at the sum -- a zeroing select here made
    // the compiler wait for these loads before issuing the partial systems')
    double pa[16];
    int sing = 0;
    if (tid < 64) {
        const int wl = max(G.n_wave - 1, 0);
#pragma unroll
        for (int k = 0; k < 16; ++k) pa[k] = Wk.partA[min(tid + 64 * k, wl) * kPartA];
        sing = *Wk.singular;
    }
    const int done = st->done;
    const double lambda = st->lambda;
    // keep the compiler from sinking the partial systems' loads under the done branch
#pragma unroll
    for (int i = 0; i < kE; ++i)
#pragma unroll
        for (int x = 0; x < kGrp; ++x) __asm__ volatile("" ::"v"(v[i][x]));
    if (done) return true;
#pragma unroll
    for (int i = 0; i < kE; ++i) {
        double a = v[i][0];
#pragma unroll
        for (int x = 1; x < kGrp; ++x) a += v[i][x];
        const int d = dst[i];
        if (d >= 0) {
            if (d & kMfMapLambda) a += lambda;
            M[d & (kMfMapLambda - 1)] = a;
        } else if (d <= -2) {
            gsh[-2 - d] = a;
        }
    }
    if (tid < 64) {
        double c = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) c += tid + 64 * k < G.n_wave ? pa[k] : 0.0;
        for (int w = tid + 64 * 16; w < G.n_wave; w += 64) c += Wk.partA[w * kPartA];
        c = wave_sum_det(c);
        if (tid == 0) {
            Wk.sys[G.n_pb * 36 + 12 * G.n_free] = c;  // the decision of iteration 0 reads the initial cost here
            *fail = sing;
        }
    }
    return false;
}

// combine_p2p's exchange in flag-in-word form (RSVIO_P2P_LL=1, A/B): every entry (and the three
// scalars: initial cost, singular flag, wave count) goes to every rank as two tagged 8-byte words
// -- no fence, no flags -- and the reader polls the words themselves, every rank's words of its
// entries in flight together (ranks in two groups of 4), re-reading until all carry this
// exchange's tag.  Same sums in the same rank order as the flag protocol: the same bits.
template <int NF>
__device__ bool combine_p2p_ll(const Geometry& G, const Work& Wk, double* M, double* gsh, int* fail, const P2P& P,
                               unsigned long long* xgen, int* err,
                               const double (&v)[((NF * (NF + 1) / 2) * 36 + 12 * NF + kK5Threads - 1) / kK5Threads][kGrp],
                               const int (&dst)[((NF * (NF + 1) / 2) * 36 + 12 * NF + kK5Threads - 1) / kK5Threads],
                               const double (&pa)[16], int sing, double lambda, unsigned long long gen) {
    constexpr int NE = (NF * (NF + 1) / 2) * 36 + 12 * NF;
    constexpr int T = kK5Threads, kE = (NE + T - 1) / T;
    const int ne = G.n_pb * 36 + 12 * G.n_free;
    const int tid = threadIdx.x, nr = P.nranks, me = P.rank, par = (int)(gen & 1);
    const unsigned g32 = (unsigned)gen;
#pragma unroll
    for (int i = 0; i < kE; ++i) {
        const int e = tid + T * i;
        if (e >= ne) break;
        double a = v[i][0];
#pragma unroll
        for (int x = 1; x < kGrp; ++x) a += v[i][x];
        if (me == 0 && dst[i] >= 0 && (dst[i] & kMfMapLambda)) a += lambda;
        for (int r = 0; r < nr; ++r) ll_put(p2p_llsys(P.peer[r], par, me) + 2 * (size_t)e, a, g32);
    }
    double c = 0.0;
    if (tid < 64) {
#pragma unroll
        for (int k = 0; k < 16; ++k) c += tid + 64 * k < G.n_wave ? pa[k] : 0.0;
        for (int w = tid + 64 * 16; w < G.n_wave; w += 64) c += Wk.partA[w * kPartA];
        c = wave_sum_det(c);
    }
    // the scalars go last, once every thread's entry stores have completed (vmcnt(0), then the
    // barrier), so a reader that sees a rank's scalars finds its entries there too: the readers
    // poll the 6 scalar words of each rank and read the entries once (still tag-checked), instead
    // of every thread re-reading all its entries' words of every rank until they arrive -- traffic
    // that, with four ranks on one GPU, starved the last rank's own progress until the spin bound
    __builtin_amdgcn_s_waitcnt(kWaitStores);
    __syncthreads();
    if (tid < nr) {  // lane r pushes the scalars to rank r
        unsigned long long* d = p2p_llsys(P.peer[tid], par, me) + 2 * (size_t)ne;
        ll_put(d, c, g32);
        ll_put(d + 2, sing ? 1.0 : 0.0, g32);
        ll_put(d + 4, (double)G.n_wave, g32);
    }
    const unsigned long long* mine = p2p_llsys(P.peer[me], par, 0);
    // scalars: lane r of wave 0 reads rank r's three (the sums in rank order by lane 0, below)
    __shared__ double sc[kP2PMax][3];
    if (tid < nr) {
        const unsigned long long* a = mine + (size_t)tid * 2 * kP2PMsg + 2 * (size_t)ne;
        unsigned long long ws[6];
        long long spins = 0;
        for (;;) {
#pragma unroll
            for (int k = 0; k < 6; ++k) ws[k] = __hip_atomic_load(a + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            bool ok = true;
#pragma unroll
            for (int k = 0; k < 6; ++k) ok &= (unsigned)(ws[k] >> 32) == g32;
            if (ok) break;
            if (++spins > (1ll << 25)) {
                atomicExch(err, 1);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k)
            sc[tid][k] = __longlong_as_double((long long)((ws[2 * k] & 0xffffffffull) | (ws[2 * k + 1] << 32)));
    }
    __syncthreads();
    // entries: every rank's two words of this thread's entries, ranks in groups of 2 or 4
    double acc[kE];
#pragma unroll
    for (int i = 0; i < kE; ++i) acc[i] = 0.0;
    const bool late = nr <= 2 ? ll_group_sums<kE, 2>(mine, nr, ne, tid, T, g32, acc)
                              : ll_group_sums<kE, 4>(mine, nr, ne, tid, T, g32, acc);
    if (late) atomicExch(err, 1);
#pragma unroll
    for (int i = 0; i < kE; ++i) {
        const int e = tid + T * i;
        if (e >= ne) break;
        const int d = dst[i];
        if (d >= 0)
            M[d & (kMfMapLambda - 1)] = acc[i];
        else if (d <= -2)
            gsh[-2 - d] = acc[i];
    }
    if (tid == 0) {
        double cs = 0.0, f = 0.0;
        for (int r = 0; r < nr; ++r) {
            cs += sc[r][0];
            f += sc[r][1];
        }
        Wk.sys[ne] = cs;  // the decision of iteration 0 reads the (all-reduced) initial cost here
        *fail = f != 0.0;
        *xgen = gen;
    }
    if (tid < nr && P.xnw) P.xnw[tid] = (int)sc[tid][2];
    return false;
}

// combine_mapped for the landmark-sharded path over the P2P exchange (X1 folded into K5): this
// rank's reduced system is summed from its partials as combine_mapped does (+ lambda on rank 0,
// after the sum, as K4d), each entry pushed from its register into slot [parity][rank] of every
// peer's exchange buffer together with the rank's initial cost and singular flag; after the
// system-scope flags of every rank have arrived, each thread sums its entries over the slots in
// RANK ORDER (identical bits on every rank, and the same bits as X1's exchange into sys followed
// by K5's read of sys) and scatters them into M / gsh by the map.  Returns the state's done flag:
// every rank takes the same decision, so either all exchange or none does.  LL: the flag-in-word
// form (combine_p2p_ll) -- a kernel of its own, so that its polling loops' registers do not
// inflate the flag protocol's (one kernel holding both took 399 VGPRs, AGPR copies on the
// prologue's path, +1.3 us per K5 at one rank against the unsharded combine)
template <int NF, bool LL>
__device__ bool combine_p2p(const Geometry& G, const Prob& Pr, const Work& Wk, double* M, double* gsh,
                            const LmState* st, int* fail, const P2P& P, unsigned long long* xgen, int* err) {
    constexpr int NE = (NF * (NF + 1) / 2) * 36 + 12 * NF;
    constexpr int T = kK5Threads, kE = (NE + T - 1) / T;
    const size_t L = sys_len(G);
    const int ne = G.n_pb * 36 + 12 * G.n_free;
    const int tid = threadIdx.x, nr = P.nranks, me = P.rank;
    // the exchange's generation: loaded by every thread (one address), waited for at its first
    // use after the partial systems' loads are in flight -- not an LDS broadcast by one thread,
    // whose store made wave 0 wait a whole round trip (with the pose loads ahead of it) before
    // issuing its share of those loads, and cost a barrier
    const unsigned long long gen0 = *xgen;
    double v[kE][kGrp];
    int dst[kE];
#pragma unroll
    for (int i = 0; i < kE; ++i) {  // (branch-free: clamped loads; an entry past ne is never stored)
        const int e = tid + T * i, ec = min(e, ne - 1);
        const int d = Pr.dmap[ec];
        dst[i] = e < ne ? d : -1;
#pragma unroll
        for (int x = 0; x < kGrp; ++x) v[i][x] = Wk.cpart[(size_t)x * L + ec];
    }
    // then the K4 wave partials (initial cost) and the singular flag, behind them (branch-free:
    // clamped loads, the ones past the last wave dropped at the sum -- a zeroing select here made
    // the compiler wait for these loads before issuing the partial systems')
    double pa[16];
    int sing = 0;
    if (tid < 64) {
        const int wl = max(G.n_wave - 1, 0);
#pragma unroll
        for (int k = 0; k < 16; ++k) pa[k] = Wk.partA[min(tid + 64 * k, wl) * kPartA];
        sing = *Wk.singular;
    }
    const int done = st->done;
    const double lambda = st->lambda;
#pragma unroll
    for (int i = 0; i < kE; ++i)
#pragma unroll
        for (int x = 0; x < kGrp; ++x) __asm__ volatile("" ::"v"(v[i][x]));
    if (done) return true;
    const unsigned long long gen = (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)gen0) +
                                   ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(gen0 >> 32)) << 32) + 1;
    const int par = (int)(gen & 1);
    if constexpr (LL) return combine_p2p_ll<NF>(G, Wk, M, gsh, fail, P, xgen, err, v, dst, pa, sing, lambda, gen);
    // this rank's entries stay in registers (own): only the peers' slots are written, flagged,
    // waited for and read back (round 5; the own slot's uncached write, flag and re-read were the
    // exchange's whole cost at one rank)
    double own[kE];
#pragma unroll
    for (int i = 0; i < kE; ++i) {
        const int e = tid + T * i;
        double a = v[i][0];
#pragma unroll
        for (int x = 1; x < kGrp; ++x) a += v[i][x];
        if (me == 0 && dst[i] >= 0 && (dst[i] & kMfMapLambda)) a += lambda;
        own[i] = a;
        if (e < ne)
            for (int r = 0; r < nr; ++r)
                if (r != me) p2p_slot(P.peer[r], par, me)[e] = a;
    }
    __shared__ double osc[2];  // this rank's initial cost and singular flag
    if (tid < 64) {
        double c = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) c += tid + 64 * k < G.n_wave ? pa[k] : 0.0;
        for (int w = tid + 64 * 16; w < G.n_wave; w += 64) c += Wk.partA[w * kPartA];
        c = wave_sum_det(c);
        if (tid == 0) {
            osc[0] = c;
            osc[1] = sing ? 1.0 : 0.0;
        }
        if (tid < nr && tid != me) {  // lane r pushes the scalars to rank r
            double* d = p2p_slot(P.peer[tid], par, me);
            d[ne] = c;
            d[ne + 1] = sing ? 1.0 : 0.0;
            d[ne + 2] = (double)G.n_wave;  // (per rank, not summed: the folded trial exchange's bound)
        }
    }
    if (nr > 1) __threadfence_system();
    __syncthreads();
    if (tid < nr && tid != me)
        __hip_atomic_store(p2p_flags(P.peer[tid]) + par * kP2PMax + me, gen, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid < nr && tid != me) {
        const unsigned long long* f = p2p_flags(P.peer[me]) + par * kP2PMax + tid;
        long long spins = 0;
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1ll << 25)) {  // a peer never arrived: report, do not hang
                atomicExch(err, 1);
                break;
            }
        }
        // relaxed polls (no L2 invalidate per poll), one acquire once the flag is seen
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    const double* mine = p2p_slot(P.peer[me], par, 0);
    // this thread's values from a group of ranks in flight together (own from registers, peers'
    // from their slots), groups in rank order: one round trip per group of 2 (two ranks), 4 (three
    // or four) or 8 ranks, then the rank-ordered sums
    double sums[kE];
#pragma unroll
    for (int i = 0; i < kE; ++i) sums[i] = 0.0;
    if (nr <= 2)
        p2p_group_sums_own<kE, 2>(mine, nr, me, ne, tid, T, own, sums);
    else if (nr <= 4)
        p2p_group_sums_own<kE, 4>(mine, nr, me, ne, tid, T, own, sums);
    else  // 5..8 ranks: every peer's slot in flight together -- one round trip, not two groups of 4
        p2p_group_sums_own<kE, 8>(mine, nr, me, ne, tid, T, own, sums);
#pragma unroll
    for (int i = 0; i < kE; ++i) {
        const int e = tid + T * i;
        if (e >= ne) break;
        const double a = sums[i];
        const int d = dst[i];
        if (d >= 0)
            M[d & (kMfMapLambda - 1)] = a;
        else if (d <= -2)
            gsh[-2 - d] = a;
    }
    if (tid == 0) {
        // every peer's two scalars in flight together (unrolled over the rank bound), then the
        // rank-ordered sums with this rank's own values substituted
        double cv[kP2PMax], fv[kP2PMax];
#pragma unroll
        for (int r = 0; r < kP2PMax; ++r) {
            const bool peer = r < nr && r != me;
            cv[r] = peer ? __hip_atomic_load(mine + (size_t)r * kP2PMsg + ne, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                         : osc[0];
            fv[r] = peer ? __hip_atomic_load(mine + (size_t)r * kP2PMsg + ne + 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM)
                         : osc[1];
        }
        double c = 0.0, f = 0.0;
#pragma unroll
        for (int r = 0; r < kP2PMax; ++r)
            if (r < nr) {
                c += cv[r];
                f += fv[r];
            }
        Wk.sys[ne] = c;  // the decision of iteration 0 reads the (all-reduced) initial cost here
        *fail = f != 0.0;
        *xgen = gen;
    }
    if (tid < nr && P.xnw)
        P.xnw[tid] = tid == me ? G.n_wave
                               : (int)__hip_atomic_load(mine + (size_t)tid * kP2PMsg + ne + 2, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_SYSTEM);
    return false;
}

// pivot J of panel H (width PW) by wave 0: inv = 1 / d_K ready.  Column J+1 (the next pivot's)
// and column J+2 are updated from readlanes of the unscaled column u; columns >= J+3 from values
// of u read this step and consumed one step later (uq, with the pivot's l as lp) -- by readlane
// since round 6 (LDS broadcasts before: their wait sat between two pivots' chains).
template <int H, int J, int PW>
__device__ __forceinline__ void mf_pivot(double (&a)[kMfPanel], double (&uq)[kMfPanel], double lp, double inv,
                                         double* Lf, double* Up, int lane, bool& bad) {
    constexpr int K = kMfPanel * H + J;
    const double u = a[J];
    double inv_next = 1.0;
    double uk1 = 0.0;
    if constexpr (J + 1 < PW) {
        // the next pivot on the shortest chain: d_{K+1} = a_{K+1,K+1} - u_{K+1,K}^2 / d_K, with
        // u_{K+1,K} and a_{K+1,K+1} read before 1/d_K is known -- inv -> fma -> rcp (+ Newton),
        // uniform on every lane, no readlane on the chain
        uk1 = rl64(u, K + 1);
        const double piv = fma(-(uk1 * uk1), inv, rl64(a[J + 1], K + 1));
        bad |= !(piv > 0.0) || !isfinite(piv);
#ifndef RSVIO_K5_RCP_LATE
        // the hardware reciprocal issued here, before the barrier (round 6): left to the
        // compiler, IR code sinking moved it past this pivot's other updates, so ~12 issue slots
        // sat between the pivot and its reciprocal on the 1/d chain; the Newton steps follow where
        // the next pivot needs them (rcp_f64's operations, the same bits).  Measured neutral
        // (0.0302-0.0304 ms per LM iteration either way, profiles/r06i_rcp_ab.txt): the chain's
        // issue slots, not this placement, bound it
        double y0 = __builtin_amdgcn_rcp(piv);
        __asm__ volatile("" : "+v"(y0));
        const double e = fma(-piv, y0, 1.0);
        inv_next = fma(y0, fma(e, e, e), y0);
#else
        inv_next = rcp_f64(piv);
#endif
    }
    const double l = u * inv;
    if constexpr (J + 1 < PW) a[J + 1] = fma(-l, uk1, a[J + 1]);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (J > 0)
#pragma unroll
        for (int jj = J + 2; jj < PW; ++jj) a[jj] = fma(-lp, uq[jj], a[jj]);
    if constexpr (J + 2 < PW) a[J + 2] = fma(-l, rl64(u, K + 2), a[J + 2]);
    Lf[K * kMfLd + lane] = l;  // column K of L (rows > K; row NP: z_K); the upper part is never read
    Up[J * kMfLd + lane] = u;  // column J of the panel's U = D L
#ifndef RSVIO_K5_LDSQ
    // round 6: the later columns' multipliers by readlane too -- no LDS read and no wait on it
    // between this pivot's chain and the next (0.0305 -> 0.0302 ms per LM iteration, 3 of 3 A/B
    // pairs, profiles/r06h_rlq_ab.txt); -DRSVIO_K5_LDSQ: LDS broadcasts (round 3-5)
#pragma unroll
    for (int jj = J + 3; jj < PW; ++jj) uq[jj] = rl64(u, kMfPanel * H + jj);
#else
#pragma unroll
    for (int jj = J + 3; jj < PW; ++jj) uq[jj] = Up[J * kMfLd + kMfPanel * H + jj];  // broadcasts
#endif
    if constexpr (J + 1 < PW) mf_pivot<H, J + 1, PW>(a, uq, l, inv_next, Lf, Up, lane, bad);
}

// Panel H (columns 8H .. 8H + PW - 1) factored by wave 0 from M into Lf and its U buffer Uh.
template <int NF, int H>
__device__ __forceinline__ void mf_factor(const double* M, double* Lf, double* Uh, int lane, bool& bad) {
    constexpr int NP = MfDims<NF>::NP;
    constexpr int C0 = kMfPanel * H;
    constexpr int PW = (NP - C0) < kMfPanel ? (NP - C0) : kMfPanel;
    double a[kMfPanel], uq[kMfPanel];
#pragma unroll
    for (int jj = 0; jj < kMfPanel; ++jj) {
        a[jj] = jj < PW ? M[(C0 + jj) * kMfLd + lane] : 0.0;
        uq[jj] = 0.0;
    }
    const double piv = rl64(a[0], C0);
    bad |= !(piv > 0.0) || !isfinite(piv);
    mf_pivot<H, 0, PW>(a, uq, 0.0, rcp_f64(piv), Lf, Uh, lane, bad);
}

// The trailing update of panel H on the matrix cores: lower tiles (I, J), I >= J, of tile columns
// J0 <= J < J1, C_IJ += (-U_I) L_J^T over the panel's 8 columns (2 MFMAs per tile), tile t of the
// flattened list taken by wave `wid` of `nw`.  A tile holding factored columns gets garbage there
// (their L lives in Lf).
template <int NF, int H>
__device__ __forceinline__ void mf_update(double* M, const double* Lf, const double* Uh, int lane, int wid, int nw,
                                          int J0, int J1) {
    constexpr int NT = MfDims<NF>::NT;
    constexpr int C0 = kMfPanel * H;
    const int i16 = lane & 15, k4 = lane >> 4;
    int ntile = 0;
    for (int J = J0; J < J1; ++J) ntile += NT - J;
    for (int t = wid; t < ntile; t += nw) {
        int TJ = J0, rem = t;
        while (rem >= NT - TJ) {
            rem -= NT - TJ;
            ++TJ;
        }
        const int TI = TJ + rem;
        double av[2], bv[2];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int kk = 4 * m + k4;
            av[m] = -Uh[kk * kMfLd + 16 * TI + i16];
            bv[m] = Lf[(C0 + kk) * kMfLd + 16 * TJ + i16];
        }
        mf_dbl4 c;
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = M[(16 * TJ + i16) * kMfLd + 16 * TI + k4 + 4 * r];
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0], bv[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1], bv[1], c, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) M[(16 * TJ + i16) * kMfLd + 16 * TI + k4 + 4 * r] = c[r];
    }
}

// Panel H is factored (Lf, Up[H & 1]) and visible to every wave.  Look-ahead: wave 0 updates the
// tile column T0 that holds panel H + 1's columns and factors panel H + 1 straight away (into the
// other U buffer), while waves 1-3 update the tile columns past T0 -- disjoint columns of M, so
// the next pivot chain starts without waiting for the rest of the trailing update.
template <int NF, int H>
__device__ __forceinline__ void mf_panel(double* M, double* Lf, double* Up, int tid, bool& bad) {
    constexpr int NT = MfDims<NF>::NT, NH = MfDims<NF>::NH;
    constexpr int C0 = kMfPanel * H;
    const int lane = tid & 63, wave = tid >> 6;
    if constexpr (H == 0) STAMP(9); else if constexpr (H == 2) STAMP(15); else if constexpr (H == 4) STAMP(30);
    if constexpr (H + 1 == NH) STAMP(7);
    if constexpr (H + 1 < NH) {
        constexpr int T0 = (C0 + kMfPanel) / 16;  // the tile column of panel H + 1
        double* Uh = Up + (H & 1) * kMfPanel * kMfLd;
        if (wave == 0) {
            mf_update<NF, H>(M, Lf, Uh, lane, 0, 1, T0, T0 + 1);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the column's updates before its reads
            __builtin_amdgcn_wave_barrier();
            mf_factor<NF, H + 1>(M, Lf, Up + ((H + 1) & 1) * kMfPanel * kMfLd, lane, bad);
        } else {
            mf_update<NF, H>(M, Lf, Uh, lane, wave - 1, kK5Threads / 64 - 1, T0 + 1, NT);
        }
        __syncthreads();
        if constexpr (H == 0) STAMP(13); else if constexpr (H == 2) STAMP(19); else if constexpr (H == 4) STAMP(31);
        mf_panel<NF, H + 1>(M, Lf, Up, tid, bad);
    }
}

// ---------------------------------------------------------------------------------------
// K5 by 6x6 block pivots (round 5): the solver of 11..20 free keyframes (camera_solve_blk_body);
// for <= 10 the 8-column panels above stay the default (measured faster at config 3, 12.7 vs
// 13.9 us) and -DRSVIO_K5_BLOCK builds this one there (A/B).  The camera system's own blocks:
// step k factors keyframe k's diagonal block as a whole.
//   * Chain wave (wave 0, lane = row; rows lane and lane + 64 past 64 rows): it holds column
//     block k of its rows in registers, fully updated.  The diagonal block's 21 lower entries go
//     to every lane through LDS (one store by its 6 rows, one broadcast read), and every lane
//     factors it redundantly in registers -- 6 pivots, the 1/d chain with no readlane or LDS on
//     it.  Every row below then solves its 6 multipliers against it (t forward-substituted,
//     u = t = the row of D L, l = t D^-1), writes L in place into M's columns and U into a U
//     buffer, and -- the look-ahead -- updates its row of column block k + 1 with this block's
//     contribution in registers, so the next step's columns never go back through LDS.
//   * Update waves (waves 1..): the block's rank-6 update of the columns past block k + 1 on the
//     matrix cores, C_IJ += (-U_I) L_J^T per 16x16 tile (the 6 columns padded to 8: two
//     v_mfma_f64_16x16x4f64), lanes whose column lies before block k + 2 neither load nor store.
// One workgroup barrier per block: 9 block steps at config 3 instead of 54 pivots each with its
// readlanes and LDS stores.  Row NP is b, whose multipliers end as z = D^-1 L^-1 b.  Tolerance
// parity like the panel version (the same pivots, sums reassociated).
// ---------------------------------------------------------------------------------------
// phase stamps of the block steps (stamps build only): lane 0 of wave w, after its memory drains
#ifdef RSVIO_STAMPS
#define WSTAMP(w, k)                                                                           \
    do {                                                                                       \
        if (threadIdx.x == 64 * (w) && blockIdx.x < 4096) {                                    \
            __builtin_amdgcn_s_waitcnt(0);                                                     \
            g_dbg[blockIdx.x * 32 + (k)] = (unsigned long long)clock64();                      \
        }                                                                                      \
    } while (0)
#else
#define WSTAMP(w, k) \
    do {             \
    } while (0)
#endif

template <int NF>
struct BkDims {
    static constexpr int NP = 6 * NF;
    static constexpr int RPL = NP + 1 <= 64 ? 1 : 2;  // rows per lane of the chain wave
    static constexpr int NT = (NP + 1 + 15) / 16;     // 16-row tiles, the b row included
    static constexpr int NPP = 16 * NT;
    static constexpr int NTC = (NP + 15) / 16;        // 16-column tiles
    static constexpr int LD = NF <= 10 ? kMfLd : kBkLd; // odd leading dimension of M and U
};

// Step K's rank-6 update of the columns >= 6 (K + 2) by update wave `wid` of `nw`.  Uk: U of
// block K (6 columns of LD doubles, zero on the rows before block K + 1); L of block K lives in
// M's columns 6K .. 6K + 5.
// Round 6: only the tiles the step can change.  env = the last camera block whose rows of column
// block K may be nonzero (the symbolic envelope, BA::set_problem: a window whose landmarks each
// span a few consecutive keyframes gives a banded S, and LDL^T keeps the band), so the update
// covers tile columns up to that block's and tile rows up to it plus the b row's tile; the other
// tiles of the dense count are skipped (no loads, no MFMAs).  The same tiles get the same MFMAs
// as before, the skipped ones would have added exact zeros: the same bits.
template <int NF, int K, int NWU>
__device__ __forceinline__ void bk_update(double* M, const double* Uk, int lane, int wid, int env) {
    using D = BkDims<NF>;
    constexpr int c0 = 6 * K, cmin = c0 + 12;
    if constexpr (cmin < D::NP) {
        constexpr int TJ0 = cmin / 16;
        constexpr int ntile_dense = (D::NTC - TJ0) * D::NT - (D::NTC - 1 + TJ0) * (D::NTC - TJ0) / 2;
        constexpr int Q = (ntile_dense + NWU - 1) / NWU;  // tiles per update wave (at most)
        constexpr int TIb = D::NP / 16;                   // the tile row of b (row NP)
        const int rlast = min(6 * (env + 1), D::NP) - 1;  // the band's last row
        const int TIe = rlast / 16;
        const int TJe = env >= K + 2 ? min(TIe, D::NTC - 1) : TJ0 - 1;  // no column in the band: nothing
        const int extra = TIb > TIe ? 1 : 0;              // the b row's tile below the band's
        // tiles of tile column TJ: rows TJ .. TIe, then TIb
        int ntile = 0;
        for (int TJ = TJ0; TJ <= TJe; ++TJ) ntile += TIe - TJ + 1 + extra;
        const int i16 = lane & 15, k4 = lane >> 4;
        // every tile's operands and accumulator loaded first, then the MFMAs, then the stores:
        // one LDS round trip per step instead of one per tile
        double av[Q][2], bv[Q][2];
        mf_dbl4 c[Q];
        int base[Q];
        bool live[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int t = wid + NWU * q;
            int TJ = TJ0, rem = t < ntile ? t : 0;
            while (rem >= TIe - TJ + 1 + extra) {
                rem -= TIe - TJ + 1 + extra;
                ++TJ;
            }
            const int TI = rem <= TIe - TJ ? TJ + rem : TIb;
            const int col = 16 * TJ + i16;  // this lane's column of the C tile (= a row of L)
            live[q] = t < ntile && col >= cmin && col < D::NP;
            base[q] = col * D::LD + 16 * TI + k4;
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const int kk = 4 * m + k4;
                av[q][m] = kk < 6 ? -Uk[kk * D::LD + 16 * TI + i16] : 0.0;
                bv[q][m] = (kk < 6 && live[q]) ? M[(c0 + kk) * D::LD + col] : 0.0;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) c[q][r] = live[q] ? M[base[q] + 4 * r] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (wid + NWU * q < ntile) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q][0], bv[q][0], c[q], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (wid + NWU * q < ntile) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q][1], bv[q][1], c[q], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (live[q])
#pragma unroll
                for (int r = 0; r < 4; ++r) M[base[q] + 4 * r] = c[q][r];
    }
}

// Block step K.  a: column block K of the chain wave's rows (updated); U: 2 x 6 x LD doubles
// (blocks alternate); Dsc / Lsc: 36 doubles each of chain-wave scratch.  Every wave of the block
// runs every step (one barrier each).
template <int NF, int K, int NW>
__device__ __forceinline__ void bk_steps(double* M, double* U, double* Dsc, double* Lsc,
                                         double (&a)[BkDims<NF>::RPL][6], int tid, bool& bad,
                                         const unsigned char* env) {
    using D = BkDims<NF>;
    constexpr int RPL = D::RPL, LD = D::LD, c0 = 6 * K;
    const int lane = tid & 63, wave = tid >> 6;
    double u[RPL][6];
    if constexpr (K < 9) WSTAMP(0, 8 + K);  // slots 8..16: wave 0 at the step's start
    WSTAMP(0, 32 + K);                       // slots 32..51: the same for every step (NF <= 20)
    WSTAMP(1, 64 + K);                       // slots 64..83: wave 1 done with step K - 1's update
    WSTAMP(7, 160 + K);                      // slots 160..179: wave 7 (the last update wave) the same
    if (wave == 0) {
        double Dg[6][6], Lg[6][6], inv[6];
#ifdef RSVIO_BK_DIAG_LDS
        // the diagonal block to every lane: its 6 rows store, every lane reads the lower 21
#pragma unroll
        for (int h = 0; h < RPL; ++h) {
            const int i = lane + 64 * h - c0;
            if (i >= 0 && i < 6)
#pragma unroll
                for (int j = 0; j < 6; ++j) Dsc[6 * i + j] = a[h][j];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) Dg[i][j] = Dsc[6 * i + j];
#else
        // the diagonal block to every lane by readlane: row c0 + i is lane (c0 + i) % 64's register
        // set (c0 + i) / 64, both compile-time -- no LDS store, wave barrier and read on the chain
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) Dg[i][j] = rl64(a[(c0 + i) >> 6][j], (c0 + i) & 63);
#endif
        // its LDL^T, redundantly on every lane: Dg[i][j] (i > j) ends as U = (D L)[i][j], Lg = L
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const double piv = Dg[j][j];
            bad |= !(piv > 0.0) || !isfinite(piv);
            inv[j] = rcp_f64(piv);
#pragma unroll
            for (int i = j + 1; i < 6; ++i) Lg[i][j] = Dg[i][j] * inv[j];
#pragma unroll
            for (int i = j + 1; i < 6; ++i)
#pragma unroll
                for (int i2 = j + 1; i2 <= i; ++i2) Dg[i][i2] = fma(-Lg[i][j], Dg[i2][j], Dg[i][i2]);
        }
        // the rows' multipliers, L and U stores, the next block's L rows to Lsc
#pragma unroll
        for (int h = 0; h < RPL; ++h) {
            const int r = lane + 64 * h, i = r - c0;
            double t[6], l[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) t[j] = a[h][j];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                u[h][j] = t[j];
                l[j] = t[j] * inv[j];
#pragma unroll
                for (int j2 = j + 1; j2 < 6; ++j2) t[j2] = fma(-l[j], Dg[j2][j], t[j2]);
            }
            // (a row i of the diagonal block gets l_j = Lg[i][j] bit for bit for j < i: the same
            // operations on the same values as the factor's; its entries j >= i land on M's
            // diagonal and upper part, which nothing reads)
            const bool below = i >= 6 && r <= D::NP;
            if (i >= 0 && r <= D::NP)
#pragma unroll
                for (int j = 0; j < 6; ++j) M[(c0 + j) * LD + r] = l[j];
            if (r < D::NPP)
#pragma unroll
                for (int j = 0; j < 6; ++j) U[(K & 1) * 6 * LD + j * LD + r] = below ? u[h][j] : 0.0;
            if constexpr (K + 1 < NF)
                if (i >= 6 && i < 12)
#pragma unroll
                    for (int j = 0; j < 6; ++j) Lsc[6 * (i - 6) + j] = l[j];
        }
    }
    if constexpr (K == 0) WSTAMP(0, 30);  // wave 0's part A of step 0 done
    if constexpr (K == 4) WSTAMP(0, 31);
    if constexpr (K >= 1 && K <= 4) WSTAMP(1, 25 + K);  // slots 26..29: wave 1 done with step K - 1
    WSTAMP(0, 128 + K);  // slots 128..147: wave 0 at barrier K (its part A done)
    __syncthreads();  // L and U of block K visible; the update waves finished block K - 1's update
    if constexpr (K < 8) WSTAMP(0, 17 + K);  // slots 17..24: wave 0 released by barrier K
    WSTAMP(0, 96 + K);                          // slots 96..115: the same for every step
    if (wave == 0) {
        if constexpr (K + 1 < NF) {
            // the look-ahead: column block K + 1 (block K - 1's update applied by the update
            // waves) minus this block's contribution, in registers
            double Ls[6][6];
#pragma unroll
            for (int j = 0; j < 6; ++j)
#pragma unroll
                for (int m = 0; m < 6; ++m) Ls[j][m] = Lsc[6 * j + m];
#pragma unroll
            for (int h = 0; h < RPL; ++h) {
                const int r = lane + 64 * h < D::NPP ? lane + 64 * h : D::NPP - 1;
#pragma unroll
                for (int j = 0; j < 6; ++j) a[h][j] = M[(c0 + 6 + j) * LD + r];
            }
#pragma unroll
            for (int h = 0; h < RPL; ++h)
#pragma unroll
                for (int j = 0; j < 6; ++j)
#pragma unroll
                    for (int m = 0; m < 6; ++m) a[h][j] = fma(-u[h][m], Ls[j][m], a[h][j]);
        }
    } else {
        bk_update<NF, K, NW - 1>(M, U + (K & 1) * 6 * LD, lane, wave - 1, env[K]);
    }
    if constexpr (K + 1 < NF) bk_steps<NF, K + 1, NW>(M, U, Dsc, Lsc, a, tid, bad, env);
}

// The whole factorisation (every wave of the block); afterwards M's columns hold L (unit lower)
// and row NP holds z.  U: 2 x 6 x LD doubles, S: 72 doubles of scratch.  (A rolled loop over
// the steps -- one step's code reused instead of ~37 KB of straight-line code -- measured
// slower: 17.1 vs 13.9 us per K5 launch at config 3, profiles/r05d_k5_stamps.txt.)
template <int NF, int NW>
__device__ __forceinline__ void bk_factor(double* M, double* U, double* S, int tid, bool& bad,
                                          const unsigned char* env) {
    using D = BkDims<NF>;
    double a[D::RPL][6];
    if ((tid >> 6) == 0) {
        const int lane = tid & 63;
#pragma unroll
        for (int h = 0; h < D::RPL; ++h) {
            const int r = lane + 64 * h < D::NPP ? lane + 64 * h : D::NPP - 1;
#pragma unroll
            for (int j = 0; j < 6; ++j) a[h][j] = M[j * D::LD + r];
        }
    }
    bk_steps<NF, 0, NW>(M, U, S, S + 36, a, tid, bad, env);
}

template <int NF, bool LL = false>
__device__ void camera_solve_mfma_body(const Geometry& G, const Prob& Pr, const Work& Wk, int combine,
                                       const P2P* P = nullptr, unsigned long long* xgen = nullptr, int* err = nullptr) {
    static_assert(NF >= 1 && NF <= 10, "one row per lane: n <= 60");
    constexpr int NP = MfDims<NF>::NP, NPP = MfDims<NF>::NPP;
    __shared__ __attribute__((aligned(16))) double M[NPP * kMfLd];
    __shared__ __attribute__((aligned(16))) double Lf[NPP * kMfLd];
    __shared__ __attribute__((aligned(16))) double Up[2 * kMfPanel * kMfLd];  // U of panels H & 1
    __shared__ double gsh[NP];
    __shared__ int fail;
    RTSTAMP(4);
    LmState* st = Wk.st;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nF = G.n_free, n = 6 * nF;
    const int SC0 = G.n_pb * 36 + 12 * nF;
    // both pose buffers (the state's cur picks one), loaded with the partial systems, before the
    // state itself
    double p7b[2][7];
    int fidx = -1;
    if (wave == 0 && lane < G.n_kf) {
        fidx = Pr.free_idx[lane];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 7; ++i) p7b[b][i] = Wk.pose[b][7 * lane + i];
    } else {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 7; ++i) p7b[b][i] = i == 3 ? 1.0 : 0.0;
    }
    STAMP(0);
    if (combine == 2) {  // sharded over P2P: this rank's system exchanged in the prologue (X1 folded in)
        if (combine_p2p<NF, LL>(G, Pr, Wk, M, gsh, st, &fail, *P, xgen, err)) return;
    } else if (combine) {
        if (combine_mapped<NF>(G, Pr, Wk, M, gsh, st, &fail)) return;
    } else {  // sharded: the all-reduced system (+ lambda on the owner rank) from sys, by the map
        if (st->done) return;
        const double* sys = Wk.sys;
        const int ne = G.n_pb * 36 + 12 * nF;
        for (int e = tid; e < ne; e += kK5Threads) {
            const int d = Pr.dmap[e];
            if (d >= 0)
                M[d & (kMfMapLambda - 1)] = sys[e];
            else if (d <= -2)
                gsh[-2 - d] = sys[e];
        }
        if (tid == 0) fail = sys[SC0 + 1] != 0.0;
    }
    const int cur = st->cur;
    double p7[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) p7[i] = cur ? p7b[1][i] : p7b[0][i];
    if (n < NP) {
        // a window with fewer free keyframes than the template (batched mode): its rows and
        // columns [n, NP) are identity padding, and the b row is zero there
        for (int e = tid; e < NP * (NP + 1); e += kK5Threads) {
            const int c = e / (NP + 1), r = e - c * (NP + 1);
            if (r >= c && ((r >= n && r < NP) || (c >= n && c < NP))) M[c * kMfLd + r] = r == c ? 1.0 : 0.0;
        }
    }
    __syncthreads();
    STAMP(1);
    // the singular flag of this iteration's K4c is already in fail (combine_mapped / combine_p2p
    // load it with the partial systems; the sys path's K4d / X1 carried it and cleared it): only
    // its reset for the next iteration here (re-reading it cost a round trip on the chain)
    if (tid == 0) *Wk.singular = 0;
    const double gcl_v = (wave == 0 && lane < n) ? gsh[lane] : 0.0;
    __syncthreads();
    STAMP(2);
    if (fail) {
        if (tid == 0) k5_result(st, 0, 0.0, 0.0);
        return;
    }
    bool bad = false;
#ifndef RSVIO_K5_BLOCK
    if (wave == 0) mf_factor<NF, 0>(M, Lf, Up, lane, bad);
    __syncthreads();
    mf_panel<NF, 0>(M, Lf, Up, tid, bad);
    double* const Lres = Lf;
#else
    static_assert(BkDims<NF>::NPP == NPP && BkDims<NF>::LD == kMfLd, "one M layout for both factorisations");
    bk_factor<NF, kK5Threads / 64>(M, Up, Lf, tid, bad, G.env);
    double* const Lres = M;  // L in place in M's columns
#endif
    if (wave != 0) return;
    if (bad) {
        if (lane == 0) k5_result(st, 0, 0.0, 0.0);
        return;
    }
    // z_j = L[NP][j] (row NP of the eliminated augmented matrix); L^T x = z (unit diagonal):
    // lane j, L[i][j] = Lf[j][i] column-major, zero for i <= j so the update needs no select
    const int lj = lane < NP ? lane : 0;
    double yv = lane < NP ? Lres[lj * kMfLd + NP] : 0.0;
    double lt[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const double m = Lres[lj * kMfLd + j];
        lt[j] = lane < j ? m : 0.0;
    }
#pragma unroll
    for (int j = NP - 1; j >= 0; --j) yv = fma(-lt[j], rl64(yv, j), yv);
    STAMP(3);
    k5_finish<NF>(G, Wk, Up, lane < n ? yv : 0.0, gcl_v, n, lane, p7, fidx);
    RTSTAMP(5);
}

template <int NF>
__global__ __launch_bounds__(kK5Threads) void ba_camera_solve_mfma(Geometry G, Prob Pr, Work Wk, int combine) {
    camera_solve_mfma_body<NF>(G, Pr, Wk, combine);
}

// K5 of the landmark-sharded iteration over the P2P exchange: the exchange of the reduced system
// (X1: combine + push + flags + rank-ordered sum) in the prologue, then the same factorisation
template <int NF, bool LL>
__global__ __launch_bounds__(kK5Threads) void ba_camera_solve_mfma_p2p(Geometry G, Prob Pr, Work Wk, P2P P,
                                                                        unsigned long long* xgen, int* err) {
    camera_solve_mfma_body<NF, LL>(G, Pr, Wk, 2, &P, xgen, err);
}

// ---------------------------------------------------------------------------------------
// K5 for 11..20 free keyframes (config 5's 19): the 6x6-block LDL^T above with MFMA trailing
// updates, 8 waves (the chain wave holds rows lane and lane + 64; 7 update waves), the system
// padded to NF in {13, 16, 20} with identity rows / columns (pivot 1, no coupling: every real
// entry sees the unpadded factorisation's operations).  The partial systems are summed in rounds
// (4 entries of 8 partials per thread in flight) and scattered into M by the window's map
// (leading dimension kBkLd).  The default past 10 free keyframes; RSVIO_K5=pipe4 / gj1 keep the
// VALU ba_camera_solve_x2 below.
// ---------------------------------------------------------------------------------------
constexpr int kBkWaves = 8;

template <int NF>
__device__ __forceinline__ void camera_solve_blk_body(const Geometry& G, const Prob& Pr, const Work& Wk, int combine) {
    using D = BkDims<NF>;
    constexpr int NP = D::NP, LD = D::LD;
    static_assert(NF > 10 && D::RPL == 2 && D::NPP <= LD, "the 11..20 free-keyframe solver");
    constexpr int T = 64 * kBkWaves;
    __shared__ __attribute__((aligned(16))) double M[16 * D::NTC * LD];
    __shared__ __attribute__((aligned(16))) double U[2 * 6 * LD];
    __shared__ __attribute__((aligned(16))) double S[72];
    __shared__ double gsh[NP];
    __shared__ double dcs[128];
    __shared__ int fail;
    LmState* st = Wk.st;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nF = G.n_free, n = 6 * nF;
    const int ne = G.n_pb * 36 + 12 * nF;
    STAMP(0);
    double p7b[2][7];
    int fidx = -1;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 7; ++i) p7b[b][i] = i == 3 ? 1.0 : 0.0;
    if (wave == 0 && lane < G.n_kf) {
        fidx = Pr.free_idx[lane];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 7; ++i) p7b[b][i] = Wk.pose[b][7 * lane + i];
    }
    if (combine) {
        // single rank: the cost of the initial linearisation (K4 wave partials) and the singular
        // flag with the first round's loads; then the partial systems in rounds
        double pa[16];
        int sing = 0;
        if (tid < 64) {
#pragma unroll
            for (int k = 0; k < 16; ++k) pa[k] = tid + 64 * k < G.n_wave ? Wk.partA[(tid + 64 * k) * kPartA] : 0.0;
            sing = *Wk.singular;
        }
        const int done = st->done;
        const double lambda = st->lambda;
        if (done) return;
        const size_t L = sys_len(G);
        constexpr int kR = 4;
        for (int e0 = 0; e0 < ne; e0 += T * kR) {
            double v[kR][kGrp];
            int dst[kR];
#pragma unroll
            for (int i = 0; i < kR; ++i) {
                const int e = e0 + tid + T * i;
                dst[i] = e < ne ? Pr.dmap[e] : -1;
#pragma unroll
                for (int x = 0; x < kGrp; ++x) v[i][x] = e < ne ? Wk.cpart[(size_t)x * L + e] : 0.0;
            }
#pragma unroll
            for (int i = 0; i < kR; ++i) {
                double a = v[i][0];
#pragma unroll
                for (int x = 1; x < kGrp; ++x) a += v[i][x];
                const int d = dst[i];
                if (d >= 0) {
                    if (d & kMfMapLambda) a += lambda;
                    M[d & (kMfMapLambda - 1)] = a;
                } else if (d <= -2) {
                    gsh[-2 - d] = a;
                }
            }
        }
        if (tid < 64) {
            double c = 0.0;
#pragma unroll
            for (int k = 0; k < 16; ++k) c += pa[k];
            for (int w = tid + 64 * 16; w < G.n_wave; w += 64) c += Wk.partA[w * kPartA];
            c = wave_sum_det(c);
            if (tid == 0) {
                Wk.sys[ne] = c;  // the decision of iteration 0 reads the initial cost here
                fail = sing;
            }
        }
    } else {  // sharded, or pre-summed (ba_schur_combine_wide): the system from sys, by the map
        // every entry's map and value loads in flight together (16 per thread covers W = 20:
        // 7,068 entries / 512 threads), then the scatter -- one round trip, not one per entry
        const double* sys = Wk.sys;
        constexpr int kE = 16;
        int dst[kE];
        double val[kE];
#pragma unroll
        for (int i = 0; i < kE; ++i) {
            const int e = tid + T * i;
            dst[i] = e < ne ? Pr.dmap[e] : -1;
            val[i] = e < ne ? sys[e] : 0.0;
        }
        const double sfail = sys[ne + 1];
        if (st->done) return;
        for (int e = tid + T * kE; e < ne; e += T) {  // (none at W <= 20)
            const int d = Pr.dmap[e];
            if (d >= 0)
                M[d & (kMfMapLambda - 1)] = sys[e];
            else if (d <= -2)
                gsh[-2 - d] = sys[e];
        }
#pragma unroll
        for (int i = 0; i < kE; ++i) {
            const int d = dst[i];
            if (d >= 0)
                M[d & (kMfMapLambda - 1)] = val[i];
            else if (d <= -2)
                gsh[-2 - d] = val[i];
        }
        if (tid == 0) fail = sfail != 0.0;
    }
    const int cur = st->cur;
    double p7[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) p7[i] = cur ? p7b[1][i] : p7b[0][i];
    if (n < NP) {  // identity padding: rows / columns [n, NP), the b row zero there
        // only the padded entries (round 6: the loop over every NP x (NP + 1) entry with a
        // division each was ~4k cycles at config 5): the padded columns' lower part (b row
        // included), then the real columns' padded rows
        const int np = NP - n;
        for (int e = tid; e < np * (np + 1); e += T) {
            const int c = n + e / (np + 1), r = n + e % (np + 1);
            if (r >= c) M[c * LD + r] = r == c ? 1.0 : 0.0;
        }
        for (int e = tid; e < n * np; e += T) {
            const int c = e / np, r = n + e % np;
            M[c * LD + r] = 0.0;
        }
    }
    __syncthreads();
    STAMP(1);
    if (tid == 0) *Wk.singular = 0;
    double gcl[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) gcl[q] = (wave == 0 && lane + 64 * q < n) ? gsh[lane + 64 * q] : 0.0;
    __syncthreads();
    STAMP(2);
    if (fail) {
        if (tid == 0) k5_result(st, 0, 0.0, 0.0);
        return;
    }
    bool bad = false;
    bk_factor<NF, kBkWaves>(M, U, S, tid, bad, G.env);
    STAMP(3);
    if (wave != 0) return;
    if (bad) {
        if (lane == 0) k5_result(st, 0, 0.0, 0.0);
        return;
    }
    // L^T x = z (unit diagonal), z = row NP: lane holds the unknowns i = lane, lane + 64, L[j][i] =
    // M[i LD + j] (zero for j <= i by the select); the padded unknowns have z = 0: start at n - 1
    // Unrolled over the template's NP unknowns (round 6): every readlane's lane and half are
    // compile-time constants (no runtime select of the half, no loop), the next 8 columns' L
    // entries are loaded while the current 8 steps run, and the padded unknowns (j >= n: z = 0,
    // no coupling) are skipped by a uniform test.  The same fmas in the same order as the
    // runtime loop it replaces (22k cycles at config 5, profiles/r06e_c5_k5_stamps.txt).
    double yv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) yv[q] = M[min(lane + 64 * q, NP - 1) * LD + NP];
    {
        constexpr int kBs = 8, NB = (NP + kBs - 1) / kBs;
        double lt[2][kBs][2];
#pragma unroll
        for (int t = 0; t < kBs; ++t)
#pragma unroll
            for (int q = 0; q < 2; ++q) lt[0][t][q] = M[min(lane + 64 * q, NP - 1) * LD + (NP - 1 - t)];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (b + 1 < NB)
#pragma unroll
                for (int t = 0; t < kBs; ++t) {
                    const int j = NP - 1 - (b + 1) * kBs - t;
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        lt[(b + 1) & 1][t][q] = M[min(lane + 64 * q, NP - 1) * LD + (j > 0 ? j : 0)];
                }
#pragma unroll
            for (int t = 0; t < kBs; ++t) {
                const int j = NP - 1 - b * kBs - t;
                if (j >= 0 && j < n) {
                    const double xj = rl64(yv[j >> 6], j & 63);
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const double upd = fma(-lt[b & 1][t][q], xj, yv[q]);
                        yv[q] = lane + 64 * q < j ? upd : yv[q];
                    }
                }
            }
        }
    }
    STAMP(4);
    double x[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) x[q] = lane + 64 * q < n ? yv[q] : 0.0;
    const double d2 = wave_sum_det(x[0] * x[0] + x[1] * x[1]);
    const double gd = wave_sum_det(gcl[0] * x[0] + gcl[1] * x[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int i = lane + 64 * q;
        if (i < n) {
            Wk.dc[i] = x[q];
            dcs[i] = x[q];
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // the LDS copy (not the dc store's acknowledgement)
    __builtin_amdgcn_wave_barrier();
    if (lane < G.n_kf) {
        double* qd = Wk.pose[1 - cur] + 7 * lane;
        if (fidx < 0) {
#pragma unroll
            for (int i = 0; i < 7; ++i) qd[i] = p7[i];
        } else {
            double qv[7];
            se3_plus(p7, dcs + 6 * fidx, qv);
#pragma unroll
            for (int i = 0; i < 7; ++i) qd[i] = qv[i];
        }
    }
    if (lane == 0) k5_result(st, 1, d2, gd);
    STAMP(5);
}

template <int NF>
__global__ __launch_bounds__(64 * kBkWaves) void ba_camera_solve_blk(Geometry G, Prob Pr, Work Wk, int combine) {
    camera_solve_blk_body<NF>(G, Pr, Wk, combine);
}

// ---------------------------------------------------------------------------------------
// K5 for 11..20 free keyframes (61 <= n <= 120): the pipelined register LDL^T with two rows per
// lane (rows lane and lane + 64) over 8 waves.  The system is padded to NP = 6 NF (NF in
// {13, 16, 20}) with identity rows / columns after the real ones and b as row NP: a padded
// column has pivot 1 and zero couplings, so every real entry sees exactly the operations of
// the unpadded factorisation.  Wave WV owns columns [WV CW, WV CW + CW); a wave whose columns
// all lie at or past 64 skips the upper half of the rows (lower triangle only).  LDS keeps the
// unscaled columns U[.][K] = (D L)[.][K] and 1/d_K; L = U / d is re-formed with the owner's
// multiply (same bits), so one NP x 121 array serves the updates and the back substitution.
// ---------------------------------------------------------------------------------------
constexpr int kX2Waves = 8;
constexpr int kUcLd = kMaxN + 1;  // 121 (odd)

__device__ __forceinline__ const double* sys_lower_rt(const double* sys, int nf, int r, int c) {
    const int n = 6 * nf;
    if (r == n) return sys + (nf * (nf + 1) / 2) * 36 + c;
    const int a = c / 6, b = r / 6;
    const int pb = a * nf - a * (a - 1) / 2 + (b - a);
    const int k = (a == b) ? (r % 6) * 6 + (c % 6) : (c % 6) * 6 + (r % 6);
    return sys + pb * 36 + k;
}

template <int NP, int CW, int WV, int K>
__device__ __forceinline__ void chol2_step(double (&a)[2][CW], int lane, double* Uc, double* dinv, double* sink,
                                           int* progress, int& seen, bool& bad, double inv) {
    constexpr int c0 = WV * CW;
    constexpr int c1 = (c0 + CW < NP) ? c0 + CW : NP;
    constexpr int Q0 = (c0 < 64) ? 0 : 1;             // first active half of the rows
    constexpr int KN = (K + 1 < c0) ? K + 2 : K + 1;  // consume columns in pairs
    if constexpr (K < c0) {
        if (seen < KN) {
            do {
                seen = __hip_atomic_load(progress, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (seen >= KN) break;
                __builtin_amdgcn_s_sleep(1);
            } while (true);
        }
        const double* u = Uc + K * kUcLd;
        const double di = dinv[K];
        double lr[2];
#pragma unroll
        for (int q = Q0; q < 2; ++q) lr[q] = u[min(lane + 64 * q, NP)] * di;
        if constexpr (KN == K + 2) {
            const double* u2 = Uc + (K + 1) * kUcLd;
            const double di2 = dinv[K + 1];
            double lr2[2];
#pragma unroll
            for (int q = Q0; q < 2; ++q) lr2[q] = u2[min(lane + 64 * q, NP)] * di2;
            double v1[CW], v2[CW];
#pragma unroll
            for (int jj = 0; jj < CW; ++jj) {
                v1[jj] = u[c0 + jj];
                v2[jj] = u2[c0 + jj];
            }
#pragma unroll
            for (int q = Q0; q < 2; ++q)
#pragma unroll
                for (int jj = 0; jj < CW; ++jj)
                    if (c0 + jj < NP) a[q][jj] = fma(-lr2[q], v2[jj], fma(-lr[q], v1[jj], a[q][jj]));
        } else {
#pragma unroll
            for (int q = Q0; q < 2; ++q)
#pragma unroll
                for (int jj = 0; jj < CW; ++jj)
                    if (c0 + jj < NP) a[q][jj] = fma(-lr[q], u[c0 + jj], a[q][jj]);
        }
        if constexpr (KN == c0) {  // first own pivot
            const double piv = rl64(a[c0 >> 6][0], c0 & 63);
            bad |= !(piv > 0.0) || !isfinite(piv);
            inv = rcp_f64(piv);
        }
    } else if constexpr (K < c1) {
        constexpr int j = K - c0;
        if constexpr (K > c0) __hip_atomic_store(progress, K, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        double uk[2], l[2];
#pragma unroll
        for (int q = Q0; q < 2; ++q) {
            uk[q] = a[q][j];
            l[q] = uk[q] * inv;
            a[q][j] = l[q];
            // every lane stores (rows past NP into the sink): the release below is then ordered
            // after each lane's own writes (a lane-divergent store could be scheduled after
            // another lane's release)
            double* dst = (q == 0 || lane + 64 <= NP) ? Uc + K * kUcLd + lane + 64 * q : sink + lane;
            *dst = uk[q];
        }
        dinv[K] = inv;  // uniform value, written by every lane for the same reason
        double piv = 1.0;
        if constexpr (j + 1 < CW && K + 1 < NP) {
            constexpr int qn = (K + 1) >> 6, ln = (K + 1) & 63;
            const double ukn = rl64(uk[qn], ln);
#pragma unroll
            for (int q = Q0; q < 2; ++q) a[q][j + 1] = fma(-l[q], ukn, a[q][j + 1]);
            piv = rl64(a[qn][j + 1], ln);
        }
#pragma unroll
        for (int jj = j + 2; jj < CW; ++jj) {
            if (c0 + jj < NP) {
                const double v = rl64(uk[(c0 + jj) >> 6], (c0 + jj) & 63);  // U[c0 + jj][K] from its lane
#pragma unroll
                for (int q = Q0; q < 2; ++q) a[q][jj] = fma(-l[q], v, a[q][jj]);
            }
        }
        if constexpr (j + 1 < CW && K + 1 < NP) {
            bad |= !(piv > 0.0) || !isfinite(piv);
            inv = rcp_f64(piv);
        }
        if constexpr (K + 1 == c1) __hip_atomic_store(progress, K + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if constexpr (K < c0) {
#pragma unroll
        for (int q = Q0; q < 2; ++q)
#pragma unroll
            for (int jj = 0; jj < CW; ++jj) __asm__ volatile("" : "+v"(a[q][jj]));
    }
    constexpr int KNEXT = (K < c0) ? KN : K + 1;
    if constexpr (KNEXT < c1) chol2_step<NP, CW, WV, KNEXT>(a, lane, Uc, dinv, sink, progress, seen, bad, inv);
}

template <int NP, int CW, int WV>
__device__ __forceinline__ void chol2_pipe(const double* sys, int nf, double* Uc, double* dinv, double* sink, int* progress,
                                           int* badw, int lane) {
    constexpr int c0 = WV * CW;
    constexpr int Q0 = (c0 < 64) ? 0 : 1;
    const int n = 6 * nf;
    double a[2][CW];
    // this wave's columns of its rows straight from sys: real rows / columns from the packed
    // system, padded ones identity, row NP = b (zero in padded columns), upper triangle zero
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int r = lane + 64 * q;
#pragma unroll
        for (int jj = 0; jj < CW; ++jj) {
            const int c = c0 + jj;
            double v = 0.0;
            if (q >= Q0 && c < NP && r <= NP && (c <= r || r == NP)) {
                if (r == NP) v = c < n ? *sys_lower_rt(sys, nf, n, c) : 0.0;
                else if (r < n) v = *sys_lower_rt(sys, nf, r, c);
                else v = (r == c) ? 1.0 : 0.0;
            }
            a[q][jj] = v;
        }
    }
    bool bad = false;
    if constexpr (c0 < NP) {
        double inv = 0.0;
        if constexpr (c0 == 0) {
            const double piv = rl64(a[0][0], 0);
            bad = !(piv > 0.0) || !isfinite(piv);
            inv = rcp_f64(piv);
        }
        int seen = 0;
        chol2_step<NP, CW, WV, 0>(a, lane, Uc, dinv, sink + 64 * WV, progress, seen, bad, inv);
    }
    if (lane == 0) badw[WV] = bad ? 1 : 0;
}

template <int NF>
__global__ __launch_bounds__(64 * kX2Waves) void ba_camera_solve_x2(Geometry G, Prob Pr, Work Wk, int combine) {
    constexpr int NP = 6 * NF, CW = (NP + kX2Waves - 1) / kX2Waves;
    static_assert(NP <= kMaxN && NP + 1 <= kUcLd && NP < 128, "padded system too large");
    __shared__ double Uc[NP * kUcLd];
    __shared__ double dinv[NP];
    __shared__ double dcs[128];
    __shared__ double sink[64 * kX2Waves];  // stores of rows past NP (see chol2_step)
    __shared__ int badw[kX2Waves];
    __shared__ int progress;
    __shared__ int fail;
    LmState* st = Wk.st;
    if (st->done) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nF = G.n_free, n = 6 * nF;
    const double* sys = Wk.sys;
    const int SG0 = G.n_pb * 36 + 6 * nF, SC0 = SG0 + 6 * nF;
    const int cur = st->cur;
    double p7[7] = {0, 0, 0, 1, 0, 0, 0};
    int fidx = -1;
    double gcl[2] = {0.0, 0.0};
    if (wave == 0 && lane < G.n_kf) {
        fidx = Pr.free_idx[lane];
#pragma unroll
        for (int i = 0; i < 7; ++i) p7[i] = Wk.pose[cur][7 * lane + i];
    }
    if (combine) {  // single rank: the reduced system from K4c's chunk partials into sys
        combine_system<64 * kX2Waves>(G, Pr, Wk, Wk.sys, st->lambda, true);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }
    if (wave == 0)
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (lane + 64 * q < n) gcl[q] = sys[SG0 + lane + 64 * q];
    if (tid == 0) {
        fail = (sys[SC0 + 1] != 0.0 || *Wk.singular) ? 1 : 0;
        *Wk.singular = 0;
        progress = 0;
    }
    __syncthreads();
    if (fail) {
        if (tid == 0) k5_result(st, 0, 0.0, 0.0);
        return;
    }
    switch (wave) {
        case 0: chol2_pipe<NP, CW, 0>(sys, nF, Uc, dinv, sink, &progress, badw, lane); break;
        case 1: chol2_pipe<NP, CW, 1>(sys, nF, Uc, dinv, sink, &progress, badw, lane); break;
        case 2: chol2_pipe<NP, CW, 2>(sys, nF, Uc, dinv, sink, &progress, badw, lane); break;
        case 3: chol2_pipe<NP, CW, 3>(sys, nF, Uc, dinv, sink, &progress, badw, lane); break;
        case 4: chol2_pipe<NP, CW, 4>(sys, nF, Uc, dinv, sink, &progress, badw, lane); break;
        case 5: chol2_pipe<NP, CW, 5>(sys, nF, Uc, dinv, sink, &progress, badw, lane); break;
        case 6: chol2_pipe<NP, CW, 6>(sys, nF, Uc, dinv, sink, &progress, badw, lane); break;
        default: chol2_pipe<NP, CW, 7>(sys, nF, Uc, dinv, sink, &progress, badw, lane); break;
    }
    __syncthreads();
    if (wave != 0) return;
    bool anybad = false;
#pragma unroll
    for (int w = 0; w < kX2Waves; ++w) anybad |= badw[w] != 0;
    if (anybad) {
        if (lane == 0) k5_result(st, 0, 0.0, 0.0);
        return;
    }
    // L^T x = z (unit diagonal), z = row NP of the factor: lane holds rows i = lane, lane + 64;
    // L[j][i] = U[j][i] / d_i by the owner's multiply.  Padded rows have z = 0: start at n - 1.
    double yv[2], di[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int i = min(lane + 64 * q, NP - 1);
        di[q] = dinv[i];
        yv[q] = Uc[i * kUcLd + NP] * di[q];
    }
    constexpr int kBs = 8;
    for (int j0 = n - 1; j0 >= 0; j0 -= kBs) {
        double lt[kBs][2];
#pragma unroll
        for (int t = 0; t < kBs; ++t) {
            const int j = max(j0 - t, 0);
#pragma unroll
            for (int q = 0; q < 2; ++q) lt[t][q] = Uc[min(lane + 64 * q, NP - 1) * kUcLd + j];
        }
#pragma unroll
        for (int t = 0; t < kBs; ++t) {
            const int j = j0 - t;
            if (j < 0) break;
            const double xj = j >= 64 ? rl64(yv[1], j - 64) : rl64(yv[0], j);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const double l = lt[t][q] * di[q];
                const double upd = fma(-l, xj, yv[q]);
                yv[q] = lane + 64 * q < j ? upd : yv[q];
            }
        }
    }
    STAMP(4);
    double x[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) x[q] = lane + 64 * q < n ? yv[q] : 0.0;
    const double d2 = wave_sum_det(x[0] * x[0] + x[1] * x[1]);
    const double gd = wave_sum_det(gcl[0] * x[0] + gcl[1] * x[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int i = lane + 64 * q;
        if (i < n) {
            Wk.dc[i] = x[q];
            dcs[i] = x[q];
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // the LDS copy (not the dc store's acknowledgement)
    __builtin_amdgcn_wave_barrier();
    if (lane < G.n_kf) {
        double* qd = Wk.pose[1 - st->cur] + 7 * lane;
        if (fidx < 0) {
#pragma unroll
            for (int i = 0; i < 7; ++i) qd[i] = p7[i];
        } else {
            double qv[7];
            se3_plus(p7, dcs + 6 * fidx, qv);
#pragma unroll
            for (int i = 0; i < 7; ++i) qd[i] = qv[i];
        }
    }
    if (lane == 0) k5_result(st, 1, d2, gd);
    STAMP(5);
}

// ---------------------------------------------------------------------------------------
// K6: one wave per landmark group: back-substitution dp = V^-1 (-g_p - W^T dc), the trial
// point, and the linearisation of the trial state into the other raw buffers (its cost is
// the trial cost).  Accepted: the next iteration starts from that linearisation; rejected:
// from the current one, untouched.
// ---------------------------------------------------------------------------------------
// The wave partials (trial cost, |dp|^2, g_p.dp, |p|^2) go out as plain stores: the decision
// is taken by the next iteration's K4c blocks (or K7 at the end of a chunk), after the boundary.
template <bool FUSED>
__device__ void k6_body(const Geometry& G, const Prob& Pr, const Work& Wk, int w, int lane, double (*sh)[64],
                        double (*shp)[64], double (*shs)[64], const P2P* PP = nullptr,
                        unsigned long long gen = 0, unsigned long long* k6tag = nullptr,
                        unsigned long long* k6part = nullptr) {
    // sh: W_s^T dc_f per slot, then the linearisation scratch; shp: trial point at the
    // landmark's first lane; shs: per-slot trial cost; per-landmark |dp|^2, g_p.dp, |p|^2
    const int s = 64 * w + lane;
    const int4 h0 = Pr.slot_hdr[2 * s], h1 = Pr.slot_hdr[2 * s + 1];
    const double2 uvq[2] = {Pr.slot_uv[2 * s], Pr.slot_uv[2 * s + 1]};
    const LmState* st = Wk.st;
    const bool act = h1.y > 0;
    const int kf = h0.x, l = h0.y, first = act ? h0.z : lane, nk = act ? h0.w : 1;
    const bool fr = h1.x >= 0;
    // every global input of this lane in one round trip with the LM state's (indices clamped on
    // padding lanes): the slot's record, the landmark's record and point and the trial pose of
    // BOTH state buffers -- the state's cur picks one after they are in flight -- and the
    // camera step
    const int kfc = act ? kf : 0, lc = act ? l : 0, fc = (act && fr) ? h1.x : 0;
    double recb[2][18], Lmb[2][10], pcb[2][3], p7b[2][7], d6[6];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const double2* wr = reinterpret_cast<const double2*>(Wk.raws[b] + (size_t)s * kRawF);
#pragma unroll
        for (int i = 0; i < 9; ++i) {  // Vs, gp_s, Wr
            const double2 x = wr[i];
            recb[b][2 * i] = x.x; recb[b][2 * i + 1] = x.y;
        }
        const double2* lr = reinterpret_cast<const double2*>(Wk.rawl[b] + (size_t)lc * kLmF);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const double2 x = lr[i];
            Lmb[b][2 * i] = x.x; Lmb[b][2 * i + 1] = x.y;
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) pcb[b][i] = Wk.pw[b][3 * lc + i];
#pragma unroll
        for (int i = 0; i < 7; ++i) p7b[b][i] = Wk.pose[b][7 * kfc + i];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) d6[i] = Wk.dc[6 * fc + i];
    const int done = st->done, solve_ok = st->solve_ok, cur = st->cur;
    const double lambda = st->lambda;
    // keep the compiler from sinking the speculative loads under the branch below
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int i = 0; i < 18; ++i) __asm__ volatile("" ::"v"(recb[b][i]));
#pragma unroll
        for (int i = 0; i < 10; ++i) __asm__ volatile("" ::"v"(Lmb[b][i]));
#pragma unroll
        for (int i = 0; i < 3; ++i) __asm__ volatile("" ::"v"(pcb[b][i]));
#pragma unroll
        for (int i = 0; i < 7; ++i) __asm__ volatile("" ::"v"(p7b[b][i]));
    }
    if (done || !solve_ok) return;  // no step: the decision (lambda up) is all there is
    STAMP(20);
    RTSTAMP(7);
    double Wv[18], Lm[10], pc[3], p7[7];
    {
        double rec[18];
#pragma unroll
        for (int i = 0; i < 18; ++i) rec[i] = cur ? recb[1][i] : recb[0][i];
        slot_w(rec, Wv);
#pragma unroll
        for (int i = 0; i < 10; ++i) Lm[i] = cur ? Lmb[1][i] : Lmb[0][i];
#pragma unroll
        for (int i = 0; i < 3; ++i) pc[i] = cur ? pcb[1][i] : pcb[0][i];
#pragma unroll
        for (int i = 0; i < 7; ++i) p7[i] = cur ? p7b[0][i] : p7b[1][i];  // the trial pose: buffer 1 - cur
    }
    double t3[3] = {0.0, 0.0, 0.0};
    if (act && fr) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double acc = 0.0;
#pragma unroll
            for (int a = 0; a < 6; ++a) acc += Wv[a * 3 + c] * d6[a];
            t3[c] = acc;
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) sh[c][lane] = t3[c];
#pragma unroll
    for (int i = 0; i < 4; ++i) shs[i][lane] = 0.0;
    if constexpr (FUSED) wave_sync(); else __syncthreads();
    STAMP(22);
    if (act && lane == first) {
        double Vi[3][3];
        landmark_inverse(Lm + LV, lambda, Vi, G.chol);
        double rhs[3] = {-Lm[LG], -Lm[LG + 1], -Lm[LG + 2]};
        for (int k = 0; k < nk; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) rhs[c] -= sh[c][first + k];
        double* pt = Wk.pw[1 - cur] + 3 * l;
        double dp2 = 0.0, gpdp = 0.0, p2 = 0.0;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double dp = (Vi[c][0] * rhs[0] + Vi[c][1] * rhs[1]) + Vi[c][2] * rhs[2];
            const double p = pc[c];
            const double q = p + dp;
            shp[c][lane] = q;
            pt[c] = q;
            dp2 += dp * dp;
            gpdp += Lm[LG + c] * dp;
            p2 += p * p;
        }
        shs[1][lane] = dp2;
        shs[2][lane] = gpdp;
        shs[3][lane] = p2;
    }
    if constexpr (FUSED) wave_sync(); else __syncthreads();
    STAMP(23);
    // linearisation of the trial state
    SlotLin L;
    if (act) {
        const Pose P = pose_from7(p7);
        const double q[3] = {shp[0][first], shp[1][first], shp[2][first]};
        slot_linearize(G, P, q, h1.y, h1.z, uvq, fr, L);
    } else {
        const Pose P{};
        const double q[3] = {0.0, 0.0, 1.0};
        slot_linearize(G, P, q, 0, 0, uvq, false, L);
    }
    shs[0][lane] = L.cost;
    if constexpr (FUSED) wave_sync(); else __syncthreads();  // sh is reused below
    STAMP(24);
    store_linearization<FUSED>(Wk, 1 - cur, s, lane, act, fr, first, nk, l, L, sh);
    STAMP(25);
    {  // wave partials: fixed-pairing butterflies over the lanes
        double v[kPartD];
#pragma unroll
        for (int i = 0; i < kPartD; ++i) v[i] = wave_sum_det(shs[i][lane]);
        if (lane == 0)
#pragma unroll
            for (int i = 0; i < kPartD; ++i) Wk.partD[w * kPartD + i] = v[i];
        if (k6tag && lane < kPartD) {  // the reducer's copy, flag-in-word at device scope (fold 3):
            // word-major planes (word q of every wave contiguous), so the reducer's polls coalesce
            double vl = v[0];
#pragma unroll
            for (int i = 1; i < kPartD; ++i) vl = lane == i ? v[i] : vl;
            const unsigned long long b = (unsigned long long)__double_as_longlong(vl), t = gen << 32;
            const size_t nw = (size_t)G.n_wave;
            __hip_atomic_store(k6tag + (2 * lane) * nw + w, (b & 0xffffffffull) | t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(k6tag + (2 * lane + 1) * nw + w, (b >> 32) | t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (k6part && lane < kPartD) {  // fold 4: the last-arriving wave's copy, at device scope
            double vl = v[0];
#pragma unroll
            for (int i = 1; i < kPartD; ++i) vl = lane == i ? v[i] : vl;
            __hip_atomic_store(k6part + (size_t)w * kPartD + lane, (unsigned long long)__double_as_longlong(vl),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (PP && lane < PP->nranks) {  // folded trial exchange: lane r pushes this wave's partial to rank r
            const int par = (int)(gen & 1);
            double* q = p2p_tval(PP->peer[lane], par, PP->rank, w);
            q[0] = v[0]; q[1] = v[1]; q[2] = v[2]; q[3] = v[3];
            __threadfence_system();
            __hip_atomic_store(p2p_tflag(PP->peer[lane], par, PP->rank, w), gen, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    STAMP(21);
    RTSTAMP(8);
}

__global__ __launch_bounds__(64) void ba_backsub_relinearize(Geometry G, Prob Pr, Work Wk) {
    __shared__ double sh[10][64];
    __shared__ double shp[3][64];
    __shared__ double shs[4][64];
    RTSTAMP(6);
    k6_body<false>(G, Pr, Wk, blockIdx.x, threadIdx.x, sh, shp, shs);
    RTSTAMP(9);
}

// K6 of the P2P-sharded iteration with the trial-scalar exchange folded in (RSVIO_P2P_FOLD=2):
// every wave also pushes its partial to every rank, tagged with this iteration's generation (the
// one K5's exchange just used); the next decision (K4c or K7) sums them there
__global__ __launch_bounds__(64) void ba_backsub_relinearize_p2p(Geometry G, Prob Pr, Work Wk, P2P P,
                                                                 const unsigned long long* xgen) {
    __shared__ double sh[10][64];
    __shared__ double shp[3][64];
    __shared__ double shs[4][64];
    unsigned long long gen = *xgen;
    __asm__ volatile("" : "+s"(gen));  // loaded with the kernel's first loads, not at its end
    k6_body<false>(G, Pr, Wk, blockIdx.x, threadIdx.x, sh, shp, shs, &P, gen);
}

// Fold 3 (round 5, the default P2P iteration: K4c, K5 with the system exchange, K6 -- three
// launches, no X2): K6's workgroup n_wave is the REDUCER.  Every K6 wave writes its 4 partials
// flag-in-word at device scope (k6tag, tag = this trial exchange's generation); the reducer polls
// them, sums them exactly as trial_scalars_wave does (the same lane-strided accumulation and
// fixed-pairing wave sums, + |x|^2 of the free poses on rank 0), pushes the 4 scalars to every
// peer flag-in-word (the X2 exchange's slots and generation), polls the peers', and writes the
// rank-ordered sums to trial4 -- the same bits X2 wrote, read by the next K4c / K7 after the
// boundary.  Forward progress: the reducer waits inside the grid for the other n_wave workgroups,
// so it needs them all dispatched -- HIP does not promise in-order dispatch or co-residency, it
// relies on (a) the dispatcher handing out workgroups in index order (the reducer is the last
// index) and (b) the whole grid fitting the stream's CUs at once.  (b) is checked on the host:
// fold 3 is taken only while n_wave + 1 <= the resident capacity of this kernel on the stream's CU
// mask (occupancy x CUs, divided among the ranks sharing the device), else the iteration falls back
// to fold 1 (plain K6 + X2, the same exchange slots and generation: bit-identical, and ranks may
// differ in the choice); see BA::k6_fits.  Its spins are bounded like every exchange's (the error
// flag the host checks), so a broken assumption fails the solve instead of hanging it.
// KU: waves per lane and sweep (4 when n_wave <= 256: the sums of the waves past the last are
// zeros either way, so trial_scalars_wave's 8 give the same bits; half the uncached words per sweep)
template <int KU>
__device__ void k6_reduce_p2p(const Geometry& G, const Prob& Pr, const Work& Wk, const P2P& P,
                              unsigned long long* xgen, int* err, const unsigned long long* k6tag) {
    const int lane = threadIdx.x & 63;
    const LmState s = *Wk.st;
    const unsigned long long gen = *xgen + 1;  // (X2's: the exchange after K5's)
    if (s.done) return;
    const unsigned g32 = (unsigned)gen;
    const int nr = P.nranks, me = P.rank, par = (int)(gen & 1);
    // the poses' |x|^2 (trial_scalars_wave's loads and sums)
    const int el = 7 * G.n_kf - 1;
    double p0[3], p1[3];
    int fi[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int e = min(lane + 64 * k, el);
        fi[k] = Pr.free_idx[e / 7];
        p0[k] = Wk.pose[0][e];
        p1[k] = Wk.pose[1][e];
    }
    constexpr int kU = KU;
    double acc[kPartD] = {0.0, 0.0, 0.0, 0.0};
    bool late = false;
    if (s.solve_ok) {  // (no step: K6's waves returned early, the partials are zeros)
        for (int i0 = 0; i0 < max(G.n_wave, 64 * kU); i0 += 64 * kU) {
            // this lane's waves i0 + lane + 64 k: every pending one's 8 words loaded together, a wave
            // whose words all carry this exchange's tag is done and not re-read (later sweeps load
            // only the waves still missing, and lanes past the last wave load nothing)
            unsigned long long wd[kU][kPartD][2];
            unsigned pend = 0;
#pragma unroll
            for (int k = 0; k < kU; ++k)
                if (i0 + lane + 64 * k < G.n_wave) pend |= 1u << k;
            long long spins = 0;
            const size_t nw = (size_t)G.n_wave;
            for (;;) {
#pragma unroll
                for (int k = 0; k < kU; ++k)
                    if (pend & (1u << k)) {
                        const unsigned long long* a = k6tag + (i0 + lane + 64 * k);
#pragma unroll
                        for (int j = 0; j < kPartD; ++j) {
                            wd[k][j][0] = __hip_atomic_load(a + (2 * j) * nw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            wd[k][j][1] = __hip_atomic_load(a + (2 * j + 1) * nw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
#pragma unroll
                for (int k = 0; k < kU; ++k)
                    if (pend & (1u << k)) {
                        bool ok = true;
#pragma unroll
                        for (int j = 0; j < kPartD; ++j)
                            ok &= (unsigned)(wd[k][j][0] >> 32) == g32 && (unsigned)(wd[k][j][1] >> 32) == g32;
                        if (ok) pend &= ~(1u << k);
                    }
                if (__all(pend == 0)) break;
                if (++spins > (1ll << 25)) {
                    late = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int k = 0; k < kU; ++k)
                if (i0 + lane + 64 * k < G.n_wave)
#pragma unroll
                    for (int j = 0; j < kPartD; ++j)
                        acc[j] += __longlong_as_double((long long)((wd[k][j][0] & 0xffffffffull) | (wd[k][j][1] << 32)));
        }
    }
    double sq[2] = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (me == 0 && lane + 64 * k <= el && fi[k] >= 0) {
            sq[0] += p0[k] * p0[k];
            sq[1] += p1[k] * p1[k];
        }
    acc[3] += sq[s.cur];
    double out[kPartD];
#pragma unroll
    for (int k = 0; k < kPartD; ++k) out[k] = wave_sum_det(acc[k]);
    // the exchange (X2's flag-in-word protocol): lane 4 r + i pushes value i to rank r, then polls
    // rank r's value i in this rank's buffer; this rank's own from registers
    const int r = lane >> 2, i = lane & 3;
    double mv = out[0];
#pragma unroll
    for (int k = 1; k < kPartD; ++k) mv = i == k ? out[k] : mv;
    double got = mv;
    if (r < nr && r != me) {
        ll_put(p2p_ll(P.peer[r], par, me) + 2 * i, mv, g32);
        const unsigned long long* w = p2p_ll(P.peer[me], par, r) + 2 * i;
        long long spins = 0;
        for (;;) {
            const unsigned long long a = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const unsigned long long b = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((unsigned)(a >> 32) == g32 && (unsigned)(b >> 32) == g32) {
                got = __longlong_as_double((long long)((a & 0xffffffffull) | (b << 32)));
                break;
            }
            if (++spins > (1ll << 25)) {
                late = true;
                got = 0.0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (late) atomicExch(err, 1);
    double v4[kPartD];
#pragma unroll
    for (int k = 0; k < kPartD; ++k) {
        double v = 0.0;
        for (int q = 0; q < nr; ++q) v += rl64(got, 4 * q + k);  // rank order from 0.0: X2's sum
        v4[k] = v;
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kPartD; ++k) Wk.trial4[k] = v4[k];
        *xgen = gen;
    }
}

__global__ __launch_bounds__(64) void ba_backsub_relinearize_p2p3(Geometry G, Prob Pr, Work Wk, P2P P,
                                                                  unsigned long long* xgen, int* err,
                                                                  unsigned long long* k6tag) {
    __shared__ double sh[10][64];
    __shared__ double shp[3][64];
    __shared__ double shs[4][64];
    if ((int)blockIdx.x == G.n_wave) {
        if (G.n_wave <= 256)
            k6_reduce_p2p<4>(G, Pr, Wk, P, xgen, err, k6tag);
        else
            k6_reduce_p2p<8>(G, Pr, Wk, P, xgen, err, k6tag);
        return;
    }
    unsigned long long gen = *xgen + 1;
    __asm__ volatile("" : "+s"(gen));  // loaded with the kernel's first loads, not at its end
    k6_body<false>(G, Pr, Wk, blockIdx.x, threadIdx.x, sh, shp, shs, nullptr, gen, k6tag);
}

// Fold 4 (round 5): no reducer workgroup and no wait inside K6.  Every K6 wave stores its 4
// partials at device scope (k6part), waits for them to complete and takes a ticket (a relaxed
// device-scope counter); the wave that draws the last ticket sums the partials exactly as
// trial_scalars_wave does (+ |x|^2 of the free poses on rank 0), pushes the 4 scalars flag-in-word
// to every rank (itself included, X2's slots and generation) and returns -- it waits for nobody.
// The next decision (K4c's wave 0, or K7) polls the nranks x 4 tagged words and sums them in rank
// order: the same bits as X2 / fold 3.  A rank without landmarks (no K6 wave) pushes from
// workgroup 0 of a one-workgroup grid.
__device__ void k6_last_push(const Geometry& G, const Prob& Pr, const Work& Wk, const P2P& P,
                             unsigned long long* xgen, unsigned long long gen, const unsigned long long* k6part,
                             const LmState& s) {
    const int lane = threadIdx.x & 63;
    constexpr int kU = 8;
    const int wl = max(G.n_wave - 1, 0), el = 7 * G.n_kf - 1;
    unsigned long long pw[kU][kPartD];
#pragma unroll
    for (int k = 0; k < kU; ++k)
#pragma unroll
        for (int j = 0; j < kPartD; ++j)
            pw[k][j] = __hip_atomic_load(k6part + (size_t)min(lane + 64 * k, wl) * kPartD + j, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    double p0[3], p1[3];
    int fi[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int e = min(lane + 64 * k, el);
        fi[k] = Pr.free_idx[e / 7];
        p0[k] = Wk.pose[0][e];
        p1[k] = Wk.pose[1][e];
    }
    // trial_scalars_wave's order: per lane the waves lane + 64 k ascending (zeros past the last),
    // a tail loop past 512 waves, then the poses' squares, then the fixed-pairing wave sums
    double acc[kPartD] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < kU; ++k)
#pragma unroll
        for (int j = 0; j < kPartD; ++j)
            acc[j] += lane + 64 * k < G.n_wave ? __longlong_as_double((long long)pw[k][j]) : 0.0;
    for (int i = lane + 64 * kU; i < G.n_wave; i += 64)
#pragma unroll
        for (int j = 0; j < kPartD; ++j)
            acc[j] += __longlong_as_double((long long)__hip_atomic_load(k6part + (size_t)i * kPartD + j, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_AGENT));
    double sq[2] = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (P.rank == 0 && lane + 64 * k <= el && fi[k] >= 0) {
            sq[0] += p0[k] * p0[k];
            sq[1] += p1[k] * p1[k];
        }
    acc[3] += sq[s.cur];
    double out[kPartD];
#pragma unroll
    for (int k = 0; k < kPartD; ++k) out[k] = wave_sum_det(acc[k]);
    const int r = lane >> 2, i = lane & 3, par = (int)(gen & 1);
    double mv = out[0];
#pragma unroll
    for (int k = 1; k < kPartD; ++k) mv = i == k ? out[k] : mv;
    if (r < P.nranks) ll_put(p2p_ll(P.peer[r], par, P.rank) + 2 * i, mv, (unsigned)gen);
    if (lane == 0) *xgen = gen;
}

__global__ __launch_bounds__(64) void ba_backsub_relinearize_p2p4(Geometry G, Prob Pr, Work Wk, P2P P,
                                                                  unsigned long long* xgen, unsigned* k6cnt,
                                                                  unsigned long long* k6part) {
    __shared__ double sh[10][64];
    __shared__ double shp[3][64];
    __shared__ double shs[4][64];
    unsigned long long gen = *xgen + 1;
    __asm__ volatile("" : "+s"(gen));  // loaded with the kernel's first loads, not at its end
    if (G.n_wave > 0) {
        k6_body<false>(G, Pr, Wk, blockIdx.x, threadIdx.x, sh, shp, shs, nullptr, gen, nullptr, k6part);
        const LmState s = *Wk.st;
        if (s.done || !s.solve_ok) return;  // (k6_body's own early exit: no partials, no decision pending)
        // this wave's partial stores complete before its ticket (vmcnt(0): a store at device scope
        // is acknowledged once it is visible at that scope), and the ticket is an agent-scope
        // acquire-release: the fence releases every lane's partials with it, and the last ticket's
        // acquire fence orders k6_last_push's loads after every other wave's release (the HIP memory
        // model's guarantee, not only the store counter's)
        __builtin_amdgcn_s_waitcnt(kWaitStores);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        unsigned t = 0;
        if (threadIdx.x == 0) t = __hip_atomic_fetch_add(k6cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        t = __builtin_amdgcn_readfirstlane(t);
        if (t != (unsigned)G.n_wave - 1) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (threadIdx.x == 0) __hip_atomic_store(k6cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        k6_last_push(G, Pr, Wk, P, xgen, gen, k6part, s);
    } else {
        const LmState s = *Wk.st;
        if (s.done || !s.solve_ok) return;
        k6_last_push(G, Pr, Wk, P, xgen, gen, k6part, s);
    }
}

// K6r (sharded): this rank's trial scalars (|x|^2 of the poses on the owner rank) -> trial4,
// ready for the all-reduce
__global__ __launch_bounds__(64) void ba_reduce_trial(Geometry G, Prob Pr, Work Wk, int include_poses) {
    const LmState s = *Wk.st;
    if (s.done) return;
    double v[4];
    trial_scalars_wave(G, Pr, Wk, s, include_poses, v);
    if (threadIdx.x == 0)
        for (int k = 0; k < 4; ++k) Wk.trial4[k] = v[k];
}

// ---------------------------------------------------------------------------------------
// K7: the pending decision at the end of a chunk of iterations.  Like K4c it reads the state
// copy the last iteration left (st_prev, its trial pending) and writes the decided state to the
// other copy (st): the next chunk's first K4c decides the same pending trial again from st_prev
// (identical bits), so no block ever reads a copy another block of the launch writes.
// host: the pinned LmState copy; htick (pinned, fine-grained): [1] solve start, [2] this
// decision's wall clock, then [0] = the decision's ticket, a system-scope release the host polls
// (rsvio_ba_wait returns on it, before the kernel's end-of-kernel signal) -- all by block 0.
// hout (pinned, fine-grained, or null; then the grid is one block): when the decision ends the
// solve, the kK7Blocks blocks (each deciding redundantly) copy one slice each of the optimised
// state -- poses then points of the current buffers -- into it, and each publishes the solve's
// start stamp in its own slot htick[4 + block] (release): rsvio_ba_get_state waits for the slots
// and copies from host memory.  A slice per CU keeps each CU's PCIe writes within one round of
// outstanding requests (one block writing all 48.6 KB took ~10 us).
constexpr int kK7Threads = 256;
#ifndef RSVIO_K7_BLOCKS  // build-time A/B: 48 blocks measured no faster and less stable
#define RSVIO_K7_BLOCKS 16  // (profiles/r03w_k7_blocks_ab.txt)
#endif
constexpr int kK7Blocks = RSVIO_K7_BLOCKS;
__device__ __forceinline__ void lm_decide_body(const Geometry& G, const Prob& Pr, const Work& Wk, int pre_reduced,
                                               const LmArgs& la, LmState* host, unsigned long long* htick,
                                               double* hout, const P2P* PP = nullptr,
                                               const unsigned long long* xgen = nullptr, int* err = nullptr) {
    STAMP(8);
    __shared__ LmState sd;
    if (threadIdx.x < 64) {  // the decision by wave 0 of every block
        const LmState d = lm_decide(G, Pr, Wk, Wk.st_prev, pre_reduced, la, PP, xgen, err);
        if (threadIdx.x == 0) {
            sd = d;
            if (blockIdx.x == 0) {
                LmState h = d;
                h.p2p_err = Wk.p2p_err ? *Wk.p2p_err : 0;  // the exchanges before this decision
                *Wk.st = d;
                *host = h;
            }
        }
    }
    __syncthreads();
    const LmState s = sd;
    if (hout && s.done) {
        const double* pose = Wk.pose[s.cur];
        const double* pw = Wk.pw[s.cur];
        const int np = 7 * G.n_kf, n = np + 3 * G.n_lm;
        // even slices, written 16 B per store (half the PCIe write requests of 8-B stores)
        const int per = (((n + (int)gridDim.x - 1) / (int)gridDim.x) + 1) & ~1;
        const int i0 = (int)blockIdx.x * per, i1 = min(n, i0 + per);
        for (int i = i0 + 2 * (int)threadIdx.x; i < i1; i += 2 * kK7Threads) {
            const double a = i < np ? pose[i] : pw[i - np];
            if (i + 1 < i1) {
                const double b = i + 1 < np ? pose[i + 1] : pw[i + 1 - np];
                *reinterpret_cast<double2*>(hout + i) = make_double2(a, b);
            } else {
                hout[i] = a;
            }
        }
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(htick + 4 + blockIdx.x, Wk.tick[1], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long t = Wk.tick[0] + 1;
        Wk.tick[0] = t;
        htick[1] = Wk.tick[1];
        htick[2] = wall_clock64();
        __threadfence_system();
        __hip_atomic_store(htick, t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    STAMP(10);
}

__global__ __launch_bounds__(kK7Threads) void ba_lm_decide(Geometry G, Prob Pr, Work Wk, int pre_reduced, LmArgs la,
                                                           LmState* host, unsigned long long* htick, double* hout) {
    lm_decide_body(G, Pr, Wk, pre_reduced, la, host, htick, hout);
}

// K7 of the P2P-sharded solve with the folded trial exchange (RSVIO_P2P_FOLD=2; mode 4: fold 4)
__global__ __launch_bounds__(kK7Threads) void ba_lm_decide_p2p(Geometry G, Prob Pr, Work Wk, LmArgs la, LmState* host,
                                                               unsigned long long* htick, double* hout, P2P P,
                                                               const unsigned long long* xgen, int* err, int mode) {
    lm_decide_body(G, Pr, Wk, mode, la, host, htick, hout, &P, xgen, err);
}

// ---------------------------------------------------------------------------------------
// Batched mode (SURVEY 8d "expected regime"): B independent windows solved by ONE launch chain --
// the window is the grid's y dimension of every LM kernel (K4, then per iteration K4c, K5, K6, and
// K7 per chunk), each block reads its window's descriptor (geometry, problem and the four state
// views) from a device table.  Grids are as wide as the widest window; a block past its window's
// waves / chunks, or of a window that is skipped or has terminated, returns at once.  Every window
// takes exactly the single-window operations, so its result equals its own solve bit for bit.
// ---------------------------------------------------------------------------------------
struct WinDesc {
    Geometry G;
    Prob Pr;
    Work W[4];  // work(0), work(1) (iteration parity), work_at(0), work_at(1)
    int skip;
};

// The descriptor's fields a block needs before its first data load -- the skip flag, its grid
// bound and the problem pointers -- are read at entry, unconditionally, so their scalar loads
// go out together (one round trip to the descriptor); an early exit tested first (a
// short-circuit `skip || n_wave` test) chained two more dependent round trips before any data
// load could issue.  (The state views stay references into the descriptor: a local copy of Work
// is indexed by the state's cur at run time, which puts it in scratch memory.)
// Forces pointer fields of the descriptor into SGPRs at this point (their scalar loads are
// issued with the ones before, one wait for all); the body's later reads of the same fields are
// the same loads (no store in between), so its first data loads issue right after the exit test.
__device__ __forceinline__ void desc_touch1(const void* p) { __asm__ volatile("" ::"s"(p)); }
template <class... T>
__device__ __forceinline__ void desc_touch(const T*... p) {
    (desc_touch1(p), ...);
}


__global__ __launch_bounds__(64) void bab_linearize(const WinDesc* __restrict__ D, double lambda0) {
    const WinDesc& d = D[blockIdx.y];
    const int skip = d.skip, bound = d.G.n_wave;
    const Prob Pr = d.Pr;
    const Work& Wk = d.W[2];
    desc_touch(Pr.slot_hdr, Pr.slot_uv, Wk.pose_init, Wk.pw_init, Wk.st);
    if (skip | ((int)blockIdx.x >= bound)) return;
    linearize_body(d.G, Pr, Wk, blockIdx.x, 1, lambda0);
}

__global__ __launch_bounds__(kSchurThreads) void bab_schur_chunks(const WinDesc* __restrict__ D, int wi, LmArgs la) {
    const WinDesc& d = D[blockIdx.y];
    const int skip = d.skip, bound = d.G.n_chunk;
    const Prob Pr = d.Pr;
    const Work& Wk = d.W[wi];
    desc_touch(Pr.pairs, Wk.partD, Wk.pose[0], Wk.pose[1], Wk.st_prev, Wk.st);
    if (skip | ((int)blockIdx.x >= bound)) return;
    schur_chunks_body(d.G, Pr, Wk, la, 0, blockIdx.x);
}

template <int NF>
__global__ __launch_bounds__(kK5Threads) void bab_camera_solve(const WinDesc* __restrict__ D, int wi) {
    const WinDesc& d = D[blockIdx.x];
    const int skip = d.skip, nkf = d.G.n_kf, nf = d.G.n_free, npb = d.G.n_pb, nw = d.G.n_wave;
    const Prob Pr = d.Pr;
    const Work& Wk = d.W[wi];
    // the descriptor fields of the combine's first loads in one scalar round trip with the skip
    // flag (the body read them on demand: a second round trip before the partial systems)
    desc_touch(Pr.free_idx, Pr.dmap, Wk.pose[0], Wk.pose[1], Wk.cpart, Wk.partA, Wk.singular, Wk.st);
    __asm__ volatile("" ::"s"(nkf), "s"(nf), "s"(npb), "s"(nw));
    if (skip) return;
    camera_solve_mfma_body<NF>(d.G, Pr, Wk, 1);
}

// the batched mode's K5 past 10 free keyframes: the 6x6-block solver of the window in row
// blockIdx.x of the descriptor table
template <int NF>
__global__ __launch_bounds__(64 * kBkWaves) void bab_camera_solve_blk(const WinDesc* __restrict__ D, int wi) {
    const WinDesc& d = D[blockIdx.x];
    const int skip = d.skip;
    const Prob Pr = d.Pr;
    const Work& Wk = d.W[wi];
    desc_touch(Pr.free_idx, Pr.dmap, Wk.pose[0], Wk.pose[1], Wk.cpart, Wk.partA, Wk.singular, Wk.st);
    if (skip) return;
    camera_solve_blk_body<NF>(d.G, Pr, Wk, 1);
}

__global__ __launch_bounds__(64) void bab_backsub_relinearize(const WinDesc* __restrict__ D, int wi) {
    const WinDesc& d = D[blockIdx.y];
    const int skip = d.skip, bound = d.G.n_wave;
    const Prob Pr = d.Pr;
    const Work& Wk = d.W[wi];
    desc_touch(Pr.slot_hdr, Pr.slot_uv, Wk.st, Wk.raws[0], Wk.raws[1], Wk.rawl[0], Wk.rawl[1], Wk.pw[0], Wk.pw[1],
               Wk.pose[0], Wk.pose[1], Wk.dc);
    if (skip | ((int)blockIdx.x >= bound)) return;
    __shared__ double sh[10][64];
    __shared__ double shp[3][64];
    __shared__ double shs[4][64];
    k6_body<false>(d.G, Pr, Wk, blockIdx.x, threadIdx.x, sh, shp, shs);
}

// Single-window front end of K7 (the handle's graph in descriptor mode, BundleAdjuster::start_graph):
// the window's geometry, problem and state views from its device descriptor D[0], so the captured
// launch sequence does not change with the window -- a new keyframe window only rewrites D[0]
__global__ __launch_bounds__(kK7Threads) void bad_lm_decide(const WinDesc* __restrict__ D, int wi, LmArgs la,
                                                            LmState* host, unsigned long long* htick, double* hout) {
    const WinDesc& d = D[0];
    const Prob Pr = d.Pr;
    const Work& Wk = d.W[wi];
    lm_decide_body(d.G, Pr, Wk, 0, la, host, htick, hout);
}

// K7 per window: the pending decision in place and into the pinned host copy host[window]
__global__ __launch_bounds__(64) void bab_lm_decide(const WinDesc* __restrict__ D, int wi, LmArgs la, LmState* host) {
    const WinDesc& d = D[blockIdx.x];
    if (d.skip) return;
    const LmState s = lm_decide(d.G, d.Pr, d.W[wi], d.W[wi].st, 0, la);
    if (threadIdx.x == 0) {
        *d.W[wi].st = s;
        host[blockIdx.x] = s;
    }
}

// ---------------------------------------------------------------------------------------
// One-shot peer-to-peer all-reduce over xGMI for the sharded BA's small per-iteration
// messages (the reduced system, ~14 KB at W=10; 4 trial scalars).  Every rank exports an
// uncached exchange buffer (IPC); a call pushes the message into slot [parity][rank] of every
// peer's buffer, raises its flag there (system-scope release), waits for every peer's flag in
// its own buffer (bounded), then sums the slots in rank order -- one kernel, one xGMI
// round trip, identical bits on every rank.  Generations alternate two parities, so a rank
// that runs ahead can never overwrite a slot its slower peer is still reading.
// ---------------------------------------------------------------------------------------

// One exchange by a whole 256-thread block: this rank's message msg[0..n) (LDS or global) is
// pushed into slot [parity][rank] of every peer's buffer, the flags are raised (system-scope
// release), the block waits for every peer's flag in its own buffer (bounded: an error flag the
// host checks), and out[i] = the slots summed in rank order -- identical bits on every rank.
// The generation lives in device memory (xgen, advanced by each exchange): every rank runs the
// same exchange sequence, so the counters agree, and a captured graph replays correctly.
// gen_pre: this exchange's generation when the caller loaded the counter at its start (its
// round trip then overlaps the caller's own loads); 0: loaded here.
__device__ void p2p_exchange(const double* msg, int n, const P2P& P, unsigned long long* xgen, int* err, double* out,
                             unsigned long long gen_pre = 0) {
    __shared__ unsigned long long sgen;
    const int tid = threadIdx.x, nr = P.nranks, me = P.rank;
    if (!gen_pre) {
        if (tid == 0) sgen = *xgen + 1;
        __syncthreads();
    }
    const unsigned long long gen = gen_pre ? gen_pre : sgen;
    const int par = (int)(gen & 1);
    if (n <= kP2PLLMax) {  // flag-in-word: thread (r, i) of the first nr * n pushes / polls one double
        const unsigned g32 = (unsigned)gen;
        const int r = tid / kP2PLLMax, i = tid % kP2PLLMax;
        if (r < nr && i < n) ll_put(p2p_ll(P.peer[r], par, me) + 2 * i, msg[i], g32);
        __shared__ double got[kP2PMax][kP2PLLMax];
        if (r < nr && i < n) {
            const unsigned long long* w = p2p_ll(P.peer[me], par, r) + 2 * i;
            long long spins = 0;
            for (;;) {
                const unsigned long long a = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const unsigned long long b = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((unsigned)(a >> 32) == g32 && (unsigned)(b >> 32) == g32) {
                    got[r][i] = __longlong_as_double((long long)((a & 0xffffffffull) | (b << 32)));
                    break;
                }
                if (++spins > (1ll << 25)) {  // a peer never arrived: report, do not hang
                    atomicExch(err, 1);
                    got[r][i] = 0.0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        if (tid < n) {
            double v = 0.0;
            for (int q = 0; q < nr; ++q) v += got[q][tid];  // rank order: identical bits on every rank
            out[tid] = v;
        }
        if (tid == 0) *xgen = gen;
        return;
    }
    for (int r = 0; r < nr; ++r) {
        double* dst = P.peer[r] + (size_t)(par * kP2PMax + me) * kP2PMsg;
        for (int i = tid; i < n; i += 256) dst[i] = msg[i];
    }
    __threadfence_system();
    __syncthreads();
    if (tid < nr)
        __hip_atomic_store(p2p_flags(P.peer[tid]) + par * kP2PMax + me, gen, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid < nr) {
        const unsigned long long* f = p2p_flags(P.peer[me]) + par * kP2PMax + tid;
        long long spins = 0;
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1ll << 25)) {  // a peer never arrived: report, do not hang
                atomicExch(err, 1);
                break;
            }
        }
        // relaxed polls (no L2 invalidate per poll), one acquire once the flag is seen
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    const double* mine = P.peer[me] + (size_t)(par * kP2PMax) * kP2PMsg;
    for (int i0 = tid; i0 < n; i0 += 4 * 256) {  // 4 values x every rank in flight per round
        double v[4][kP2PMax];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < kP2PMax; ++r)
                v[q][r] = __hip_atomic_load(mine + (size_t)min(r, nr - 1) * kP2PMsg + min(i0 + 256 * q, n - 1),
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double a = 0.0;
#pragma unroll
            for (int r = 0; r < kP2PMax; ++r)
                if (r < nr) a += v[q][r];
            if (i0 + 256 * q < n) out[i0 + 256 * q] = a;
        }
    }
    if (tid == 0) *xgen = gen;
}

// generic exchange of buf[0..n) in place (the attach self-test)
__global__ __launch_bounds__(256) void ba_p2p_allreduce(double* buf, int n, P2P P, unsigned long long* xgen,
                                                        int* err) {
    p2p_exchange(buf, n, P, xgen, err, buf);
}

// X1 (sharded, P2P): K4d folded into the exchange -- this rank's reduced system from its chunk
// partials (+ lambda on rank 0; its initial cost and singular flag) is built in LDS, exchanged,
// and the rank-ordered sum lands in sys.  One launch instead of combine + all-reduce.
__global__ __launch_bounds__(256) void ba_p2p_sys(Geometry G, Prob Pr, Work Wk, P2P P, unsigned long long* xgen,
                                                  int* err) {
    __shared__ double msg[kP2PMsg];
    const LmState* st = Wk.st;
    if (st->done) return;
    combine_system<256>(G, Pr, Wk, msg, st->lambda, P.rank == 0);
    __syncthreads();
    if (threadIdx.x == 0) *Wk.singular = 0;
    p2p_exchange(msg, (int)sys_len(G), P, xgen, err, Wk.sys);
}

// X2 (sharded, P2P): K6r folded into the exchange -- this rank's trial scalars (|x|^2 of the
// poses on rank 0), exchanged and summed into trial4 for the next decision.
__global__ __launch_bounds__(256) void ba_p2p_trial(Geometry G, Prob Pr, Work Wk, P2P P, unsigned long long* xgen,
                                                    int* err) {
    __shared__ double msg[4];
    const unsigned long long gen = *xgen + 1;  // (with the state's load: one round trip for both)
    const LmState s = *Wk.st;
    if (s.done) return;
    if (threadIdx.x < 64) {
        double v[4];
        trial_scalars_wave(G, Pr, Wk, s, P.rank == 0 ? 1 : 0, v);
        if (threadIdx.x == 0)
            for (int k = 0; k < 4; ++k) msg[k] = v[k];
    }
    __syncthreads();
    p2p_exchange(msg, 4, P, xgen, err, Wk.trial4, gen);
}

}  // namespace

RSVIO_DBG_READER(rsvio_dbg_ba_stamps)
RSVIO_RT_READER(rsvio_dbg_ba_rt)

// set_problem's observation pass (keys, masks, (u, v) narrowed) lives in obs_pass.hpp: chunked
// over the calling thread and a few helper threads.
using rsvio_obs::observation_pass;

// slots of a landmark = keyframes with any of its observations (bits 2 kf, 2 kf + 1 of its mask)
__attribute__((target("popcnt"))) static inline int slot_count(unsigned long long m) {
    return __builtin_popcountll((m | (m >> 1)) & kEvenBits);
}

struct BundleAdjuster {
    rsvio_ba_params P{};
    hipStream_t stream = nullptr;
    bool own_stream = true;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    Geometry G{};
    bool has_problem = false;
    int iter_chunk = 2;       // LM iterations enqueued per status read-back after the first chunk
    // Single rank: the start of a solve (K0 + K4 + the first chunk of k LM iterations, ~17
    // kernels) captured once as a HIP graph and replayed by one hipGraphLaunch -- the host
    // enqueue drops from ~80 us to a few us.  Keyed by k and the LM configuration; dropped when
    // set_problem may have moved buffers.  Any capture failure falls back to direct launches.
    // Two execs: gv captures the by-value kernels for the uploaded window (kernel arguments as
    // immediates; keyed by k, the LM configuration, export, free keyframes and the collective, stale
    // after set_problem); gd is the descriptor mode (below), keyed by the window's shape only.  The
    // first solve of a new window runs gd (no capture: a new keyframe window costs one launch); a
    // window solved again (a retry, a resident re-solve) captures gv once and replays it, which
    // saves the descriptor's extra dependent load at the head of every kernel (~0.3 us each).
    struct GraphSlot {
        hipGraphExec_t exec = nullptr;
        int k = -1;
        rsvio_lm_cfg cfg{};
        bool exp = false, stale = false;
        int nf = -1, coll = -1, wcap = 0, chunk = -1;
        const void* dptr = nullptr;
        hipEvent_t ev_launch = nullptr;  // recorded after each launch: update in place once it completed
    };
    GraphSlot gv, gd;
    int solves_of_problem = 0;  // starts since the last set_problem
    bool graphs_ok = true;
    int k5_variant = 2;  // camera solve for n_free <= 10: 2 blocked LDL^T with MFMA trailing updates (default),
                         // 0 pipelined 4-wave LDL^T (RSVIO_K5=pipe4), 1 one-wave Gauss-Jordan (gj1)
    // an exec whose launch may still run is never destroyed (a ticket wait returns before the
    // last decision kernel has exited): unless the stream is idle (known, or queried without
    // waiting) it is retired and destroyed once it is -- set_problem need not wait for the stream
    std::vector<hipGraphExec_t> retired;
    void drop_slot(GraphSlot& sl) {
        if (sl.exec) {
            if (!settled) {
                if (hipStreamQuery(stream) == hipSuccess)
                    settled = true;
                else
                    (void)hipGetLastError();  // hipErrorNotReady is no error here
            }
            if (settled) {
                destroy_retired();
                (void)hipGraphExecDestroy(sl.exec);
            } else {
                retired.push_back(sl.exec);
                if (retired.size() > 4) settle();  // bounded: wait for the stream then
            }
        }
        sl.exec = nullptr;
        sl.k = -1;
        sl.stale = false;
    }
    void drop_graph() {
        drop_slot(gv);
        drop_slot(gd);
    }
    void destroy_retired() {
        for (hipGraphExec_t g : retired) (void)hipGraphExecDestroy(g);
        retired.clear();
    }
    static bool same_cfg(const rsvio_lm_cfg& a, const rsvio_lm_cfg& b) {
        return a.max_iterations == b.max_iterations && a.cost_tolerance == b.cost_tolerance &&
               a.parameter_tolerance == b.parameter_tolerance && a.huber_delta == b.huber_delta &&
               a.lambda_init == b.lambda_init && a.linear_solver == b.linear_solver;
    }
    // (single rank, or sharded over the P2P exchange, whose generation counter lives on the
    // device; RCCL calls stay out of the graph)
    // A new problem keeps gv (stale): its next capture, when the topology is the same (chunk size,
    // LM configuration, export, free keyframes, collective) and the exec's last launch has completed
    // (ev_launch), updates the exec in place (hipGraphExecUpdate) instead of instantiating a new
    // one.  RSVIO_BA_GRAPH_UPDATE=0: always instantiate (A/B switch).
    bool graph_update = true;
    // Descriptor mode (single rank, MFMA camera solve): the graph's kernels (bab_* / bad_lm_decide)
    // read the window's geometry, problem pointers and state views from a device descriptor at the
    // head of the arena (WinDesc, written into the staging image by set_problem and uploaded with
    // it), and K4 / K6 run on a grid of wcap >= n_wave workgroups (the rest return at once).  The
    // launch sequence is then the same for every window of the same shape: a new keyframe window
    // is solved by the exec as it stands -- no capture, no update, one hipGraphLaunch.
    // RSVIO_BA_DESC=0: every window's first solve captures gv too (A/B switch).
    bool desc_on = true;
    WinDesc hdesc{};                      // the descriptor set_problem wrote (host copy)
    double desc_huber = std::nan("");     // the LM configuration the device descriptor holds
    int desc_chol = -1;
    HostBuf<WinDesc> h_desc1;             // staging of a descriptor refresh (another LM configuration)
    hipEvent_t ev_desc = nullptr;
    bool desc_pending = false;
    bool desc_mode() const { return desc_on && coll == 0 && k5_variant == 2 && G.n_free <= 10 && G.n_wave > 0; }
    // the P2P-sharded iteration (RSVIO_P2P_FOLD): 3 (default since round 5) 3 launches -- the
    // reduced system's exchange in K5's prologue, K6 with a reducer workgroup that sums the rank's
    // tagged wave partials and runs the trial exchange (no X2; 0.8 us per iteration below fold 1
    // on the same partition, profiles/r05k_same_basis.txt); 1: 4 launches (the trial scalars by
    // X2); 4: 3 launches, K6's last-arriving wave pushes the rank's scalars and the next decision
    // polls them (measured no faster than 3, profiles/r05l_fold4_same_basis.txt); 2: 3 launches,
    // the next decision summing every wave's partial of every rank (10.6 us slower,
    // profiles/r04k_p2p_fold_kstats.txt); 0: 5 launches (X1 as its own kernel)
    int fold_lvl = 3;
    int fold_req = 3;             // the level asked for (RSVIO_P2P_FOLD); attach_p2p may lower fold_lvl
    bool p2p_shared_gpu = false;  // attach_p2p found two ranks on one device (fold 2 -> 1, 4 -> 3)
    bool p2p_fold() const { return fold_lvl >= 1 && coll == 2 && k5_variant == 2 && G.n_free <= 10; }
    bool p2p_fold2() const { return fold_lvl == 2 && p2p_fold(); }
    bool p2p_fold3() const { return fold_lvl == 3 && p2p_fold() && k6_fits(); }
    // fold 3's reducer waits inside K6's grid for the other workgroups: only while the whole grid
    // (n_wave + 1 one-wave workgroups) fits the stream's resident capacity at once
    int k6_cap = 0;               // resident K6 workgroups on this stream's CUs (refresh_k6_cap)
    bool k6_fits() const { return G.n_wave + 1 <= k6_cap; }
    int p2p_share = 1;            // ranks on this rank's device (attach_p2p)
    bool p2p_fold4() const { return fold_lvl == 4 && p2p_fold(); }
    const WinDesc* dptr() const { return reinterpret_cast<const WinDesc*>(d_arena.p + lay.desc); }
    void fill_desc(WinDesc& d) const {
        d = WinDesc{};
        d.G = G;
        d.G.huber_delta = desc_huber;
        d.G.chol = desc_chol;
        d.Pr = prob();
        d.W[0] = work(0);
        d.W[1] = work(1);
        d.W[2] = work_at(0);
        d.W[3] = work_at(1);
        d.skip = 0;
    }
    // the solve's LM configuration differs from the one the device descriptor holds: rewrite it
    // (stream-ordered before the launch that reads it; the staging copy is guarded by ev_desc)
    void refresh_desc() {
        if (desc_pending && hipEventQuery(ev_desc) != hipSuccess) {
            (void)hipGetLastError();
            RSVIO_HIP(hipEventSynchronize(ev_desc));
        }
        desc_pending = false;
        desc_huber = G.huber_delta;
        desc_chol = G.chol;
        hdesc.G.huber_delta = desc_huber;
        hdesc.G.chol = desc_chol;
        if (!h_desc1.p) h_desc1.alloc(1);
        *h_desc1.p = hdesc;
        settled = false;
        RSVIO_HIP(hipMemcpyAsync(d_arena.p + lay.desc, h_desc1.p, sizeof(WinDesc), hipMemcpyHostToDevice, stream));
        RSVIO_HIP(hipEventRecord(ev_desc, stream));
        desc_pending = true;
    }
    // k: the first chunk wanted (the previous solve's iteration count); on return, the chunk the
    // launched exec enqueues
    bool start_graph(const rsvio_lm_cfg& cfg, int& k) {
        if (coll == 1 || !graphs_ok) return false;
        const bool dm = desc_mode() && solves_of_problem == 0;
        ++solves_of_problem;
        GraphSlot& sl = dm ? gd : gv;
        if (dm && (G.huber_delta != desc_huber || G.chol != desc_chol)) refresh_desc();
        // K4 / K6 grid of a capture: n_wave + 1/4 headroom (the next windows of a similar shape
        // replay it while n_wave > wcap / 2), a multiple of 8 (wave w on XCD w % 8 either way);
        // spare workgroups return at once
        const int wcap = (G.n_wave + G.n_wave / 4 + kGrp - 1) / kGrp * kGrp;
        // descriptor mode: an exec whose first chunk is up to 2 iterations longer than wanted is
        // replayed too (iterations past convergence return at once; cheaper than a re-capture when
        // consecutive windows converge in slightly different counts, as the Estimator's do)
        const bool k_ok = sl.k == k || (dm && sl.k > k && sl.k <= k + 2);
        const bool topo = sl.exec && k_ok && same_cfg(sl.cfg, cfg) && sl.exp == export_on && sl.nf == G.n_free &&
                          sl.coll == coll;
        const bool hit = topo && (dm ? (sl.dptr == dptr() && sl.chunk == G.n_chunk && G.n_wave <= sl.wcap &&
                                        2 * G.n_wave > sl.wcap)
                                     : !sl.stale);
        if (hit) k = sl.k;
        if (!hit) {
            const auto tg0 = std::chrono::steady_clock::now();
            bool try_update = topo && sl.k == k && graph_update;
            if (try_update && hipEventQuery(sl.ev_launch) != hipSuccess) {
                (void)hipGetLastError();  // hipErrorNotReady is no error here
                try_update = false;
            }
            if (!try_update) drop_slot(sl);
            if (hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
                (void)hipGetLastError();
                graphs_ok = false;
                return false;
            }
            bool ok = true;
            try {
                if (dm) {
                    enqueue_start_d(cfg.lambda_init, wcap);
                    for (int i = 0; i < k; ++i) enqueue_iteration_d(cfg, i, wcap);
                    enqueue_decide_d(cfg, k);
                } else {
                    enqueue_start(cfg.lambda_init);
                    for (int i = 0; i < k; ++i) enqueue_iteration(cfg, i);
                    enqueue_decide(cfg, k);
                }
            } catch (...) {
                ok = false;
            }
            hipGraph_t g = nullptr;
            if (hipStreamEndCapture(stream, &g) != hipSuccess) ok = false;
            const auto tg1 = std::chrono::steady_clock::now();
            bool updated = false;
            if (ok && try_update) {
                hipGraphNode_t err_node = nullptr;
                hipGraphExecUpdateResult r = hipGraphExecUpdateError;
                updated = hipGraphExecUpdate(sl.exec, g, &err_node, &r) == hipSuccess && r == hipGraphExecUpdateSuccess;
                if (!updated) {
                    (void)hipGetLastError();
                    drop_slot(sl);  // (its last launch has completed: destroyed at once)
                }
            }
            if (ok && !updated && hipGraphInstantiate(&sl.exec, g, nullptr, nullptr, 0) != hipSuccess) {
                sl.exec = nullptr;
                ok = false;
            }
            const auto tg2 = std::chrono::steady_clock::now();
            if (g) (void)hipGraphDestroy(g);
            if (prof_env)
                fprintf(stderr, "[rsvio] graph us (%s): drop+capture %.1f %s %.1f destroy %.1f\n", dm ? "desc" : "value",
                        std::chrono::duration<double, std::micro>(tg1 - tg0).count(),
                        updated ? "update" : "instantiate",
                        std::chrono::duration<double, std::micro>(tg2 - tg1).count(),
                        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tg2).count());
            if (!ok) {
                (void)hipGetLastError();
                graphs_ok = false;
                return false;
            }
            sl.k = k;
            sl.cfg = cfg;
            sl.exp = export_on;
            sl.nf = G.n_free;
            sl.coll = coll;
            sl.stale = false;
            sl.wcap = wcap;
            sl.chunk = G.n_chunk;
            sl.dptr = dm ? static_cast<const void*>(dptr()) : nullptr;
        }
        settled = false;  // (drop_slot above may have found the stream idle)
        RSVIO_HIP(hipGraphLaunch(sl.exec, stream));
        if (graph_update) RSVIO_HIP(hipEventRecord(sl.ev_launch, stream));
        return true;
    }
    int last_iterations = 3;  // first chunk = previous solve's iteration count
    DevBuf<double> d_pose2, d_pw2;
    // The static problem (initial state, keyframe map, slot headers + observations, Schur pair
    // lists, camera-block table) lives in one device arena, filled in one pinned staging image
    // and uploaded by ONE asynchronous copy (ba_stage_in, or hipMemcpyAsync under
    // RSVIO_BA_STAGE=sdma).  The staging image may be refilled once the copy has read it: a solve
    // waited for since (its ticket comes after the copy in stream order) or a settled stream
    // proves that; otherwise the next set_problem synchronises the stream (up_pending) -- no event
    // per upload on the step's critical path.  Offsets in bytes, 256-B aligned.
    DevBuf<uint8_t> d_arena;
    HostBuf<uint8_t> h_arena;
    bool up_pending = false;
    struct ArenaLayout {
        size_t desc, pose_init, pw_init, free_idx, pb_fa, pb_fb, dmap, mask, lm_base, wave_fill, wave_lm, key, ouv, upload;
        size_t hdr, uv, pairs, total;  // built on the device
    } lay{};
    bool prof_env = false;      // RSVIO_BA_PROFILE: host phase times of set_problem on stderr
    bool prof_slow = false;     // RSVIO_BA_PROFILE=slow: only the slow calls, with the mappings added since
    std::string prof_maps;      // (the last /proc/self/maps of a slow-call report)
    bool uv_env = true;         // RSVIO_BA_UV32=0: always upload (u, v) as f64 (A/B)
    // RSVIO_BA_EARLY_COPY=1: the observation section's copy issued as soon as the pass fills it
    // (rounds 3-5); default one copy at the end: set_problem 61 -> 56 us of host time alone
    // (profiles/r06g_setprob.txt), the step no slower (profiles/r06h_early_copy_ab.txt)
    bool early_env = false;
    bool stage_kernel = true;   // RSVIO_BA_STAGE=sdma: the staging image by hipMemcpyAsync (A/B)
    bool stage_split = true;    // RSVIO_BA_STAGE_SPLIT=0: one stage-in launch at the end (A/B)
    const void* h_arena_dev = nullptr;  // the staging image's device address
    // the optimised state of the last solve, written by its final decision kernel (K7) before the
    // ticket: [pose7 n_kf x 7 | p_W n_lm x 3]; state_export = it holds the handle's current state
    // export_on: the final decisions export it -- turned on by the first rsvio_ba_get_state, so a
    // caller that never reads the state back (re-solving a resident window) pays nothing for it
    HostBuf<double> h_out;
    bool state_export = false, export_on = false;
    bool state_fresh = false;  // set_problem without a run since: get_state resets the buffers first
    // host scratch of set_problem, kept across problems (no per-problem allocations)
    std::vector<int> hs_free, hs_pb_fa, hs_pb_fb;
    DevBuf<double> d_raws, d_rawl, d_partA, d_partD, d_cpart, d_sys, d_dc, d_trial4;
    DevBuf<int> d_singular;
    size_t n_pad = 0;
    DevBuf<LmState> d_state;  // two copies, alternating by iteration (LmState)
    HostBuf<LmState> h_state;
    // decision tickets (ba_lm_decide): device counter + start stamp, pinned fine-grained host
    // copy; n_tick = decisions enqueued (graph launches included); settled = stream known idle
    DevBuf<unsigned long long> d_tick;
    unsigned long long* h_tick = nullptr;
    unsigned long long n_tick = 0;
    bool settled = true, tick_wait = true;
    double wclk_khz = 1.0e5;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // collective of the sharded path: 0 none (single rank), 1 RCCL, 2 peer-to-peer one-shot
    int coll = 0;
    bool sharded() const { return coll != 0; }
    double* xbuf = nullptr;               // P2P exchange buffer (uncached, IPC-exported)
    P2P p2p{};
    bool p2p_opened[kP2PMax] = {};
    DevBuf<int> d_p2p_err;
    DevBuf<unsigned long long> d_xgen;  // P2P exchange generation (advanced on the device)
    DevBuf<int> d_xnw;                  // every rank's wave count (K5's exchange carries it)
    DevBuf<unsigned long long> d_k6tag; // fold 3: K6 wave partials, flag-in-word (2 kPartD words per wave);
                                        // fold 4: the plain partials (kPartD words per wave)
    DevBuf<unsigned> d_k6cnt;           // fold 4: K6's ticket counter (back to 0 by the last wave)

    void init(const rsvio_ba_params& p) {
        P = p;
        if (P.max_keyframes < 2 || P.max_keyframes > kMaxFree + 1 || P.max_landmarks < 1 ||
            P.max_landmarks > (1 << 26) || P.max_observations < 1)
            throw std::invalid_argument("invalid BA capacities (max_keyframes in [2, 21], max_landmarks <= 2^26)");
        RSVIO_HIP(hipSetDevice(P.device));
        RSVIO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        RSVIO_HIP(hipEventCreate(&ev0));
        RSVIO_HIP(hipEventCreate(&ev1));
        RSVIO_HIP(hipEventCreateWithFlags(&gv.ev_launch, hipEventDisableTiming));
        RSVIO_HIP(hipEventCreateWithFlags(&gd.ev_launch, hipEventDisableTiming));
        RSVIO_HIP(hipEventCreateWithFlags(&ev_desc, hipEventDisableTiming));
        const char* fv = std::getenv("RSVIO_P2P_FOLD");  // "0" .. "4" (A/B switch)
        if (fv && fv[0] >= '0' && fv[0] <= '4') fold_lvl = fold_req = fv[0] - '0';
        const char* dv = std::getenv("RSVIO_BA_DESC");  // "0": by-value kernels captured per window
        desc_on = !(dv && dv[0] == '0');
        const char* gu = std::getenv("RSVIO_BA_GRAPH_UPDATE");  // "0": instantiate every new problem
        graph_update = !(gu && gu[0] == '0');
        h_state.alloc(1, hipHostMallocCoherent);  // read on the decision's ticket (wait_tick)
        // (coarse-grained host memory, the stores gathered in L2 and written back whole by K7's
        // system-scope release, measured the same: profiles/r04k_ab_multi.txt)
        h_out.alloc((size_t)7 * P.max_keyframes + (size_t)3 * P.max_landmarks, hipHostMallocCoherent);
        d_tick.alloc(2);
        RSVIO_HIP(hipMemset(d_tick.p, 0, 2 * sizeof(unsigned long long)));
        RSVIO_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_tick), (4 + kK7Blocks) * sizeof(unsigned long long),
                                hipHostMallocCoherent));
        std::memset(h_tick, 0, (4 + kK7Blocks) * sizeof(unsigned long long));
        {
            int khz = 0;
            if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, P.device) == hipSuccess && khz > 0)
                wclk_khz = khz;
        }
        const char* wv = std::getenv("RSVIO_BA_WAIT");  // "sync": hipStreamSynchronize (A/B switch)
        tick_wait = !(wv && std::strcmp(wv, "sync") == 0);
        const char* ge = std::getenv("RSVIO_BA_GRAPHS");  // "0": direct launches (A/B switch)
        graphs_ok = !(ge && ge[0] == '0');
        const char* pv = std::getenv("RSVIO_BA_PROFILE");
        prof_env = pv != nullptr;
        prof_slow = pv && std::strcmp(pv, "slow") == 0;
        const char* u32v = std::getenv("RSVIO_BA_UV32");
        uv_env = !(u32v && u32v[0] == '0');
        const char* ecv = std::getenv("RSVIO_BA_EARLY_COPY");
        early_env = ecv && ecv[0] == '1';
        const char* stv = std::getenv("RSVIO_BA_STAGE");
        stage_kernel = !(stv && std::strcmp(stv, "sdma") == 0);
        if (stage_kernel) early_env = false;
        const char* ssv = std::getenv("RSVIO_BA_STAGE_SPLIT");
        stage_split = stage_kernel && !(ssv && ssv[0] == '0');
        const char* kv = std::getenv("RSVIO_K5");  // A/B switch: "gj1" one-wave Gauss-Jordan
        if (kv && std::strcmp(kv, "gj1") == 0) k5_variant = 1;
        if (kv && std::strcmp(kv, "pipe4") == 0) k5_variant = 0;
        if (kv && std::strcmp(kv, "mfma") == 0) k5_variant = 2;
    }
    ~BundleAdjuster() {
        if (stream) (void)hipStreamSynchronize(stream);
        settled = true;
        if (h_tick) (void)hipHostFree(h_tick);
        drop_graph();
        destroy_retired();
        if (comm) ncclCommDestroy(comm);
        for (int r = 0; r < kP2PMax; ++r)
            if (p2p_opened[r]) (void)hipIpcCloseMemHandle(p2p.peer[r]);
        if (xbuf) (void)hipFree(xbuf);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (gv.ev_launch) (void)hipEventDestroy(gv.ev_launch);
        if (gd.ev_launch) (void)hipEventDestroy(gd.ev_launch);
        if (ev_desc) (void)hipEventDestroy(ev_desc);
        if (stream && own_stream) (void)hipStreamDestroy(stream);
    }

    template <class T>
    static void grow(DevBuf<T>& b, size_t n) {
        if (b.n < n) b.alloc(std::max<size_t>(n, 1));
    }
    Prob prob() const {
        Prob p;
        p.free_idx = reinterpret_cast<const int*>(d_arena.p + lay.free_idx);
        p.slot_hdr = reinterpret_cast<const int4*>(d_arena.p + lay.hdr);
        p.slot_uv = reinterpret_cast<const double2*>(d_arena.p + lay.uv);
        p.pairs = reinterpret_cast<const int4*>(d_arena.p + lay.pairs);
        p.pb_fa = reinterpret_cast<const int*>(d_arena.p + lay.pb_fa);
        p.pb_fb = reinterpret_cast<const int*>(d_arena.p + lay.pb_fb);
        p.dmap = reinterpret_cast<const int*>(d_arena.p + lay.dmap);
        return p;
    }
    // the kernels of LM iteration `it` read state copy it & 1 and work on copy (it + 1) & 1
    Work work(int it) const {
        Work w = work_at((it + 1) & 1);
        w.st_prev = d_state.p + (it & 1);
        return w;
    }
    // every kernel on one state copy (reset, K4, K7, build_system's combine)
    Work work_at(int si) const {
        Work w;
        w.pose[0] = d_pose2.p; w.pose[1] = d_pose2.p + 7 * (size_t)G.n_kf;
        w.pw[0] = d_pw2.p; w.pw[1] = d_pw2.p + 3 * (size_t)std::max(G.n_lm, 1);
        w.pose_init = reinterpret_cast<const double*>(d_arena.p + lay.pose_init);
        w.pw_init = reinterpret_cast<const double*>(d_arena.p + lay.pw_init);
        w.raws[0] = d_raws.p; w.raws[1] = d_raws.p + (size_t)kRawF * std::max<size_t>(n_pad, 1);
        w.rawl[0] = d_rawl.p; w.rawl[1] = d_rawl.p + (size_t)kLmF * std::max(G.n_lm, 1);
        w.singular = d_singular.p;
        w.p2p_err = coll == 2 ? d_p2p_err.p : nullptr;
        w.partA = d_partA.p; w.partD = d_partD.p;
        w.cpart = d_cpart.p;
        w.sys = d_sys.p; w.dc = d_dc.p; w.trial4 = d_trial4.p;
        w.st = d_state.p + si;
        w.st_prev = w.st;
        w.tick = d_tick.p;
        return w;
    }

    // sliding_window.rs:159-299 problem assembly, restated for the device layout (see Prob).  No
    // sort: one pass over the observations validates them, sets a bit per (keyframe, camera) in a
    // 64-bit mask per landmark (n_kf <= 21) and packs each observation's key, all straight into
    // the pinned staging image; one pass over the landmarks packs whole landmarks into waves
    // (greedy, <= 64 slots).  The mask fixes the landmark's slots (its keyframes, ascending), each
    // slot's observations and camera bits, and every observation's place in its slot, so the slot
    // headers, the (u, v) layout and the Schur pair lists are written on the device in one launch
    // (ba_build_layout) after one H2D copy.  No stream synchronisation: the initial state is
    // set by the solve's first kernel (K4 with K0 folded in).
    // the per-problem work buffers, grown to the uploaded window (G set)
    void grow_buffers() {
        const int n_kf = G.n_kf, n_lm = G.n_lm, n_pb = G.n_pb, n_free = G.n_free, n_wave = G.n_wave;
        grow(d_pose2, 14 * (size_t)n_kf);
        grow(d_pw2, 6 * (size_t)std::max(n_lm, 1));
        {  // partial systems: every entry of every slot is written by K4c each iteration; zeroed
           // once when (re)allocated
            const size_t nc = (size_t)kGrp * ((size_t)36 * n_pb + 12 * n_free + 2);
            if (d_cpart.n < nc) {
                grow(d_cpart, nc);
                RSVIO_HIP(hipMemsetAsync(d_cpart.p, 0, sizeof(double) * d_cpart.n, stream));
            }
        }
        grow(d_raws, (size_t)2 * kRawF * std::max<size_t>(n_pad, 1));
        grow(d_rawl, (size_t)2 * kLmF * std::max(n_lm, 1));
        grow(d_singular, 1);
        grow(d_partA, (size_t)kPartA * std::max(n_wave, 1));
        grow(d_partD, (size_t)kPartD * std::max(n_wave, 1));
        grow(d_sys, (size_t)36 * n_pb + 12 * n_free + 2);
        grow(d_dc, (size_t)6 * n_free);
        grow(d_trial4, 4);
        grow(d_state, 2);
        if (d_k6tag.n < (size_t)2 * kPartD * std::max(n_wave, 1)) {  // fold 3's tagged K6 partials
            grow(d_k6tag, (size_t)2 * kPartD * std::max(n_wave, 1));
            RSVIO_HIP(hipMemsetAsync(d_k6tag.p, 0, sizeof(unsigned long long) * d_k6tag.n, stream));
        }
        if (d_k6cnt.n < 1) {
            grow(d_k6cnt, 1);
            RSVIO_HIP(hipMemsetAsync(d_k6cnt.p, 0, sizeof(unsigned), stream));
        }
    }

    void set_problem(int n_kf, const double* pose7, const uint8_t* kf_fixed, int n_lm, const double* pW, int n_obs,
                     const int32_t* obs_lm, const int32_t* obs_kf, const uint8_t* obs_cam, const double* obs_uv,
                     const double* TCB2) {
        const bool prof = prof_env;
        auto tp0 = std::chrono::steady_clock::now();
        double tms[12];
        long flt[12];
        int ntm = 0;
        auto faults = [] {
            struct rusage ru;
            getrusage(RUSAGE_THREAD, &ru);
            return (long)ru.ru_minflt;
        };
        long f0 = prof ? faults() : 0;
        auto mark = [&] {
            if (!prof) return;
            const auto t = std::chrono::steady_clock::now();
            const long f = faults();
            tms[ntm] = std::chrono::duration<double, std::micro>(t - tp0).count();
            flt[ntm++] = f - f0;
            tp0 = t;
            f0 = f;
        };
        // no stream synchronisation: the staging image is guarded by up_pending, the device buffers by
        // stream order (a buffer that grows is freed by hipFree, which waits for the device), and
        // the previous solve's graph is retired until the stream is next settled
        if (pend.active) throw CallOrderError("set_problem: a solve is in flight (call rsvio_ba_wait first)");
        // kernel arguments (sizes, buffers) change with the problem: the exec is updated or
        // replaced by the next start
        if (graph_update && gv.exec)
            gv.stale = true;
        else
            drop_slot(gv);
        solves_of_problem = 0;
        state_export = false;
        if (n_kf < 1 || n_kf > P.max_keyframes || n_lm < 0 || n_lm > P.max_landmarks || n_obs < 0 ||
            n_obs > P.max_observations)
            throw std::invalid_argument("problem exceeds the handle's capacities");
        auto& free_idx = hs_free;
        free_idx.assign(n_kf, -1);
        int n_free = 0;
        for (int k = 0; k < n_kf; ++k)
            if (!kf_fixed[k]) free_idx[k] = n_free++;
        if (n_free > kMaxFree) throw std::invalid_argument("too many free keyframes");
        if (n_free < 1) throw std::invalid_argument("no free keyframe");
        // camera blocks (fa <= fb)
        auto &pb_fa = hs_pb_fa, &pb_fb = hs_pb_fb;
        pb_fa.clear();
        pb_fb.clear();
        for (int a = 0; a < n_free; ++a)
            for (int b = a; b < n_free; ++b) {
                pb_fa.push_back(a);
                pb_fb.push_back(b);
            }
        const int n_pb = (int)pb_fa.size();
        const int n_chunk = kGrp * n_pb;
        // the uploaded part of the arena (sizes known before the passes)
        auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
        const size_t nl1 = (size_t)std::max(n_lm, 1);
        ArenaLayout L{};
        size_t off = 0;
        L.desc = off;      off += al(sizeof(WinDesc));  // descriptor mode's WinDesc (start_graph)
        L.pose_init = off; off += al(sizeof(double) * 7 * (size_t)n_kf);
        L.pw_init = off;   off += al(sizeof(double) * 3 * nl1);
        L.free_idx = off;  off += al(sizeof(int) * (size_t)n_kf);
        L.pb_fa = off;     off += al(sizeof(int) * (size_t)n_pb);
        L.pb_fb = off;     off += al(sizeof(int) * (size_t)n_pb);
        L.dmap = off;      off += al(sizeof(int) * ((size_t)36 * n_pb + 12 * n_free));
        L.lm_base = off;   off += al(sizeof(int) * nl1);
        L.wave_fill = off; off += al(sizeof(int) * nl1);  // n_wave <= n_lm
        L.wave_lm = off;   off += al(sizeof(int) * (nl1 + 1));
        // [mask, key, ouv] last: complete after the observation pass, so their copy (the bulk of
        // the upload) starts while the host still packs waves and tables
        L.mask = off;      off += al(sizeof(unsigned long long) * nl1);
        L.key = off;       off += al(sizeof(unsigned) * std::max(n_obs, 1));
        L.ouv = off;       off += al(sizeof(double2) * std::max(n_obs, 1));
        L.upload = off;
        mark();
        if (up_pending) settle();  // the previous upload may still read the staging image
        if (h_arena.n < L.upload) {
            h_arena.alloc(L.upload + L.upload / 4, hipHostMallocCoherent);
            void* dp = nullptr;
            RSVIO_HIP(hipHostGetDevicePointer(&dp, h_arena.p, 0));
            h_arena_dev = dp;
        }
        uint8_t* hb = h_arena.p;
        mark();
        // observations: validated, a (keyframe, camera) bit per landmark, packed keys
        auto* m2 = reinterpret_cast<unsigned long long*>(hb + L.mask);
        auto* key = reinterpret_cast<unsigned*>(hb + L.key);
        // fast path: vectorised keys + validation, masks by run-aligned chains and the (u, v) as f32
        // when exact (half the bytes to copy and to upload), in landmark-run-aligned chunks over the
        // helper threads (obs_pass.hpp); anything else (an index out of range, a duplicate, a
        // landmark in two runs) takes the exact pass below, which reports the error or builds the
        // masks of any order
        bool uv32 = false;
        if (!observation_pass(n_obs, obs_lm, obs_kf, obs_cam, obs_uv, n_lm, n_kf, key, m2,
                              uv_env ? reinterpret_cast<float*>(hb + L.ouv) : nullptr, &uv32)) {
            std::memset(m2, 0, sizeof(unsigned long long) * (size_t)n_lm);
            // the mask of the current run of one landmark's observations stays in a register (a
            // landmark-major list would otherwise chain every read-modify-write of m2[l] through
            // store-to-load forwarding)
            int cl = -1;
            unsigned long long cm = 0;
            for (int i = 0; i < n_obs; ++i) {
                const int l = obs_lm[i], k = obs_kf[i], c = obs_cam[i];
                if (l < 0 || l >= n_lm || k < 0 || k >= n_kf || c > 1)
                    throw std::invalid_argument("observation index out of range");
                if (l != cl) {
                    if (cl >= 0) m2[cl] = cm;
                    cl = l;
                    cm = m2[l];
                }
                const unsigned long long b = 1ull << (2 * k + c);
                if (cm & b)
                    throw std::invalid_argument("more than one observation of a landmark per camera and keyframe");
                cm |= b;
                key[i] = (unsigned)l << 6 | (unsigned)k << 1 | (unsigned)c;
            }
            if (cl >= 0) m2[cl] = cm;
            uv32 = uv_env && rsvio_obs::uv_narrow(2 * (size_t)n_obs, obs_uv, reinterpret_cast<float*>(hb + L.ouv));
        }
        if (!uv32) std::memcpy(hb + L.ouv, obs_uv, sizeof(double2) * (size_t)n_obs);
        L.upload = L.ouv + al((uv32 ? sizeof(float2) : sizeof(double2)) * std::max(n_obs, 1));
        if (d_arena.n < L.upload) {  // (grown for the whole arena below once its size is known)
            d_arena.alloc(2 * L.upload);
        }
        settled = false;  // (the upload, grow_buffers' memset and ba_build_layout go on the stream)
        // the staging image's [off0, off1) into the arena by ba_stage_in (both 256-B aligned)
        auto stage = [&](size_t off0, size_t off1) {
            const int nw = (int)((off1 - off0) / 16);
            if (nw <= 0) return;
            hipLaunchKernelGGL(ba_stage_in, dim3((nw + 511) / 512), dim3(256), 0, stream,
                               reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(h_arena_dev) + off0),
                               reinterpret_cast<uint4*>(d_arena.p + off0), nw);
            RSVIO_HIP(hipGetLastError());
        };
        // split: the observation section (masks, keys, (u, v): ~300 KB of the ~390) goes up now,
        // while the host packs the waves and fills the tables; the rest at the end
        if (stage_split) stage(L.mask, L.upload);
        if (early_env)
            RSVIO_HIP(hipMemcpyAsync(d_arena.p + L.mask, hb + L.mask, L.upload - L.mask, hipMemcpyHostToDevice, stream));
        mark();
        // waves: whole landmarks, <= 64 slots each (greedy, in landmark order); the Schur pair
        // stride is the largest XCD group's landmark count (at most one pair per landmark and
        // chunk).  Wave w (K4 / K6 workgroup w, whole landmarks) is dispatched to XCD w % 8, so
        // the landmarks of group x are those of the waves w % 8 == x; their Schur chunks run on
        // XCD x too (chunk c on XCD c % 8) and re-read what K6 wrote there.
        auto* lm_base = reinterpret_cast<int*>(hb + L.lm_base);
        auto* wave_fill = reinterpret_cast<int*>(hb + L.wave_fill);
        auto* wave_lm = reinterpret_cast<int*>(hb + L.wave_lm);
        int n_wave = 0, fill = 0;
        int gl[kGrp] = {0, 0, 0, 0, 0, 0, 0, 0};
        // the camera system's symbolic envelope (the 6x6-block solver past 10 free keyframes
        // skips the tiles outside it): a landmark couples every free keyframe between its first
        // and last one (a superset of its pairs); cand[a] = the last keyframe of the landmarks
        // starting at a, env[k] = the prefix maximum (the rows of L's column block k that may be
        // nonzero: LDL^T keeps the envelope)
        const bool want_env = n_free > 10;
        unsigned long long freebits = 0;
        for (int k = 0; k < n_kf; ++k)
            if (free_idx[k] >= 0) freebits |= 1ull << (2 * k);
        int cand[kMaxFree];
        for (int k = 0; k < kMaxFree; ++k) cand[k] = -1;
        for (int l = 0; l < n_lm; ++l) {
            const int ns = slot_count(m2[l]);
            if (!ns) {
                lm_base[l] = -1;
                continue;
            }
            if (want_env) {
                const unsigned long long kb = (m2[l] | (m2[l] >> 1)) & freebits;
                if (kb) {
                    const int a = free_idx[__builtin_ctzll(kb) >> 1], b = free_idx[(63 - __builtin_clzll(kb)) >> 1];
                    cand[a] = std::max(cand[a], b);
                }
            }
            if (n_wave == 0 || fill + ns > 64) {
                if (n_wave) wave_fill[n_wave - 1] = fill;
                wave_lm[n_wave] = l;
                ++n_wave;
                fill = 0;
            }
            lm_base[l] = 64 * (n_wave - 1) + fill;
            gl[(n_wave - 1) % kGrp] += 1;
            fill += ns;
        }
        if (n_wave) wave_fill[n_wave - 1] = fill;
        wave_lm[n_wave] = n_lm;
        int stride = 1;
        for (int x = 0; x < kGrp; ++x) stride = std::max(stride, gl[x]);
        n_pad = (size_t)64 * n_wave;
        if (coll == 2 && fold_lvl == 2 && n_wave > kP2PWaves)  // (every rank must take the same path)
            throw std::invalid_argument("shard exceeds the folded P2P trial exchange (16384 waves): RSVIO_P2P_FOLD=1");
        mark();
        // device-built part of the arena
        L.hdr = off;   off += al(sizeof(int4) * 2 * std::max<size_t>(n_pad, 1));
        L.uv = off;    off += al(sizeof(double2) * 2 * std::max<size_t>(n_pad, 1));
        L.pairs = off; off += al(sizeof(int4) * (size_t)n_chunk * stride);
        L.total = off;
        if (d_arena.n < L.total) {  // the observation copy above went to the old arena: redo it
            d_arena.alloc(L.total + L.total / 4);
            if (stage_split) stage(L.mask, L.upload);
            if (early_env)
                RSVIO_HIP(hipMemcpyAsync(d_arena.p + L.mask, hb + L.mask, L.upload - L.mask, hipMemcpyHostToDevice,
                                         stream));
        }
        lay = L;
        std::memcpy(hb + L.pose_init, pose7, sizeof(double) * 7 * (size_t)n_kf);
        if (n_lm) std::memcpy(hb + L.pw_init, pW, sizeof(double) * 3 * (size_t)n_lm);
        std::memcpy(hb + L.free_idx, free_idx.data(), sizeof(int) * (size_t)n_kf);
        std::memcpy(hb + L.pb_fa, pb_fa.data(), sizeof(int) * (size_t)n_pb);
        std::memcpy(hb + L.pb_fb, pb_fb.data(), sizeof(int) * (size_t)n_pb);
        if (n_free <= 10)
            mf_dense_map(n_free, n_pb, pb_fa.data(), pb_fb.data(), reinterpret_cast<int*>(hb + L.dmap));
        else  // the 6x6-block solver's padded template (13 / 16 / 20 free keyframes), leading dimension 129
            mf_dense_map(n_free, n_pb, pb_fa.data(), pb_fb.data(), reinterpret_cast<int*>(hb + L.dmap),
                         6 * bk_template_nf(n_free), kBkLd);
        G.n_kf = n_kf; G.n_free = n_free; G.n_lm = n_lm; G.n_obs = n_obs; G.n_slot = (int)n_pad;
        G.n_pb = n_pb; G.n_wave = n_wave; G.n_chunk = n_chunk; G.pair_stride = stride;
        for (int k = 0, run = -1; k < kMaxFree; ++k) {
            run = std::max(run, cand[k]);
            G.env[k] = (unsigned char)(k >= n_free ? k : want_env ? std::max(k, run) : n_free - 1);
        }
        G.env_on = want_env ? 1 : 0;
        for (int c = 0; c < 2; ++c)
            for (int i = 0; i < 16; ++i) G.TCB[c].m[i] = TCB2[16 * c + i];
        grow_buffers();  // (before the descriptor: it holds their addresses)
        fill_desc(hdesc);
        std::memcpy(hb + L.desc, &hdesc, sizeof(WinDesc));
        mark();
        if (stage_kernel) {
            stage(0, stage_split ? L.mask : L.upload);  // (L.mask and L.upload are multiples of 256)
        } else {
            RSVIO_HIP(hipMemcpyAsync(d_arena.p, hb, early_env ? L.mask : L.upload, hipMemcpyHostToDevice, stream));
        }
        up_pending = true;
        {
            SlotSrc S;
            S.mask = reinterpret_cast<const unsigned long long*>(d_arena.p + L.mask);
            S.lm_base = reinterpret_cast<const int*>(d_arena.p + L.lm_base);
            S.wave_fill = reinterpret_cast<const int*>(d_arena.p + L.wave_fill);
            S.key = reinterpret_cast<const unsigned*>(d_arena.p + L.key);
            S.uv = reinterpret_cast<const double2*>(d_arena.p + L.ouv);
            S.uv32 = uv32 ? 1 : 0;
            S.wave_lm = reinterpret_cast<const int*>(d_arena.p + L.wave_lm);
            S.nb_lm = (n_lm + 255) / 256;
            S.nb_pad = (int)((n_pad + 255) / 256);
            const int nb = S.nb_lm + S.nb_pad + (n_obs + 255) / 256;
            hipLaunchKernelGGL(ba_build_layout, dim3(nb + n_chunk), dim3(256), 0, stream, G, prob(), S, nb,
                               reinterpret_cast<int4*>(d_arena.p + L.hdr), reinterpret_cast<double2*>(d_arena.p + L.uv),
                               reinterpret_cast<int4*>(d_arena.p + L.pairs));
            RSVIO_HIP(hipGetLastError());
        }
        mark();
        *h_state.p = LmState{};  // cur = 0: buffer 0 holds the initial state once it is set
        state_fresh = true;
        has_problem = true;
        mark();
        if (prof) {
            double tot = 0.0;
            long ftot = 0;
            for (int i = 0; i < ntm; ++i) tot += tms[i], ftot += flt[i];
            if (!prof_slow || tot > 1000.0 || ftot > 100)
                fprintf(stderr, "[rsvio] set_problem us: checks+layout %.1f upload wait %.1f observations %.1f waves %.1f "
                        "tables %.1f enqueue %.1f grow %.1f (upload %zu B, arena %zu B); minor faults %ld %ld %ld %ld "
                        "%ld %ld %ld\n",
                        tms[0], tms[1], tms[2], tms[3], tms[4], tms[5], tms[6], L.upload, L.total, flt[0], flt[1],
                        flt[2], flt[3], flt[4], flt[5], flt[6]);
            if (prof_slow && (tot > 1000.0 || ftot > 100)) {  // what the process mapped since the last report
                std::string maps;
                if (FILE* fm = std::fopen("/proc/self/maps", "r")) {
                    char buf[4096];
                    size_t n;
                    while ((n = std::fread(buf, 1, sizeof buf, fm)) > 0) maps.append(buf, n);
                    std::fclose(fm);
                }
                std::vector<std::string> now, was;
                auto split = [](const std::string& t, std::vector<std::string>& out) {
                    size_t a = 0;
                    while (a < t.size()) {
                        size_t b = t.find('\n', a);
                        if (b == std::string::npos) b = t.size();
                        out.emplace_back(t, a, b - a);
                        a = b + 1;
                    }
                };
                split(maps, now);
                split(prof_maps, was);
                std::sort(was.begin(), was.end());
                for (const auto& l : now)
                    if (!std::binary_search(was.begin(), was.end(), l)) fprintf(stderr, "[rsvio]   new map: %s\n", l.c_str());
                prof_maps.swap(maps);
            }
        }
    }

    void allreduce(double* buf, size_t n) {
        if (!sharded() || n == 0) return;
        if (coll == 2) {
            if (n > kP2PMsg) throw std::runtime_error("message exceeds the P2P slot");
            hipLaunchKernelGGL(ba_p2p_allreduce, dim3(1), dim3(256), 0, stream, buf, (int)n, p2p, d_xgen.p,
                               d_p2p_err.p);
            RSVIO_HIP(hipGetLastError());
            return;
        }
        if (ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, comm, stream) != ncclSuccess)
            throw std::runtime_error("RCCL all-reduce failed");
    }

    void enqueue_reset(double lambda0) {
        settled = false;
        const int n = std::max(std::max(7 * G.n_kf, 3 * G.n_lm), 1);
        hipLaunchKernelGGL(ba_reset, dim3((n + 255) / 256), dim3(256), 0, stream, G, work_at(0), lambda0);
        RSVIO_HIP(hipGetLastError());
    }

    // K0 + K4: initial state and its linearisation (buffer 0); the LM state in copy 0
    void enqueue_start(double lambda0) {
        settled = false;
        if (G.n_wave)  // K0 folded into K4
            hipLaunchKernelGGL(ba_linearize, dim3(G.n_wave), dim3(64), 0, stream, G, prob(), work_at(0), lambda0);
        else
            enqueue_reset(lambda0);
        RSVIO_HIP(hipGetLastError());
    }

    // K4c of iteration `it` (the pending decision, then this rank's chunk partials); sharded (or
    // materialise): K4d sums them into d_sys (+ lambda on rank 0), all-reduced over the ranks
    void enqueue_linear_system(int it, const LmArgs& la, bool materialise) {
        const Prob pr = prob();
        const Work wk = work(it);
        hipLaunchKernelGGL(ba_schur_chunks, dim3(G.n_chunk), dim3(kSchurThreads), 0, stream, G, pr, wk, la,
                           sharded() ? 1 : 0);
        RSVIO_HIP(hipGetLastError());
        if (!sharded() && !materialise) {  // single rank: K5 sums the partials itself
            if (wide_combine()) {  // ... or, past 10 free keyframes, pulls one pre-summed system
                hipLaunchKernelGGL(ba_schur_combine_wide, dim3((36 * G.n_pb + 12 * G.n_free + 255) / 256), dim3(256),
                                   0, stream, G, pr, wk);
                RSVIO_HIP(hipGetLastError());
            }
            return;
        }
        if (coll == 2) {  // P2P: combine + exchange in one launch (X1)
            hipLaunchKernelGGL(ba_p2p_sys, dim3(1), dim3(256), 0, stream, G, pr, wk, p2p, d_xgen.p, d_p2p_err.p);
            RSVIO_HIP(hipGetLastError());
            return;
        }
        hipLaunchKernelGGL(ba_schur_combine, dim3(1), dim3(256), 0, stream, G, pr, wk, rank == 0 ? 1 : 0);
        RSVIO_HIP(hipGetLastError());
        allreduce(d_sys.p, (size_t)36 * G.n_pb + 12 * G.n_free + 2);
    }

    // register-resident factorisation for n_free <= 10, two rows per lane otherwise; combine:
    // the reduced system is summed from the chunk partials in K5's prologue (single rank)
    // single rank past 10 free keyframes (the 6x6-block solver): the partial systems summed by
    // ba_schur_combine_wide, so K5's one workgroup pulls one system instead of eight
    bool wide_combine() const { return !sharded() && k5_variant == 2 && G.n_free > 10; }
    void launch_camera_solve(const Prob& pr, const Work& wk, int combine) {
        if (combine && wide_combine()) combine = 0;
        const dim3 g(1), b(kK5Threads);
        if (k5_variant == 2 && G.n_free <= 10) {
            switch (G.n_free) {
#define RSVIO_CAMM(NF) \
    case NF: hipLaunchKernelGGL(ba_camera_solve_mfma<NF>, g, b, 0, stream, G, pr, wk, combine); break;
                RSVIO_CAMM(1) RSVIO_CAMM(2) RSVIO_CAMM(3) RSVIO_CAMM(4) RSVIO_CAMM(5)
                RSVIO_CAMM(6) RSVIO_CAMM(7) RSVIO_CAMM(8) RSVIO_CAMM(9) RSVIO_CAMM(10)
#undef RSVIO_CAMM
                default: break;
            }
            RSVIO_HIP(hipGetLastError());
            return;
        }
        switch (G.n_free <= 10 ? G.n_free : 0) {
#define RSVIO_CAM(NF) \
    case NF: hipLaunchKernelGGL(ba_camera_solve<NF>, g, b, 0, stream, G, pr, wk, combine, k5_variant); break;
            RSVIO_CAM(1) RSVIO_CAM(2) RSVIO_CAM(3) RSVIO_CAM(4) RSVIO_CAM(5)
            RSVIO_CAM(6) RSVIO_CAM(7) RSVIO_CAM(8) RSVIO_CAM(9) RSVIO_CAM(10)
#undef RSVIO_CAM
            default: {
                if (k5_variant == 2) {  // the 6x6-block solver with MFMA updates (the default)
                    const dim3 b3(64 * kBkWaves);
                    switch (bk_template_nf(G.n_free)) {
                        case 13: hipLaunchKernelGGL(ba_camera_solve_blk<13>, g, b3, 0, stream, G, pr, wk, combine); break;
                        case 16: hipLaunchKernelGGL(ba_camera_solve_blk<16>, g, b3, 0, stream, G, pr, wk, combine); break;
                        default: hipLaunchKernelGGL(ba_camera_solve_blk<20>, g, b3, 0, stream, G, pr, wk, combine); break;
                    }
                    break;
                }
                const dim3 b2(64 * kX2Waves);
                if (G.n_free <= 13) hipLaunchKernelGGL(ba_camera_solve_x2<13>, g, b2, 0, stream, G, pr, wk, combine);
                else if (G.n_free <= 16) hipLaunchKernelGGL(ba_camera_solve_x2<16>, g, b2, 0, stream, G, pr, wk, combine);
                else hipLaunchKernelGGL(ba_camera_solve_x2<20>, g, b2, 0, stream, G, pr, wk, combine);
                break;
            }
        }
        RSVIO_HIP(hipGetLastError());
    }

    static LmArgs lm_args(const rsvio_lm_cfg& cfg) {
        return LmArgs{cfg.max_iterations, cfg.cost_tolerance, cfg.parameter_tolerance};
    }

    // LM iteration `it`: K4c (decision of it - 1 + Schur partials), [K4d + all-reduce], K5, K6,
    // [K6r + all-reduce of the trial scalars].  Its own decision is taken by iteration it + 1's
    // K4c or by enqueue_decide at the end of the chunk.
    void enqueue_iteration(const rsvio_lm_cfg& cfg, int it) {
        const Prob pr = prob();
        const Work wk = work(it);
        if (p2p_fold()) {  // sharded over P2P: K4c, K5 with X1 folded in, K6[, X2]
            if (p2p_fold2() || p2p_fold4())
                hipLaunchKernelGGL(ba_schur_chunks_p2p, dim3(G.n_chunk), dim3(kSchurThreads), 0, stream, G, pr, wk,
                                   lm_args(cfg), p2p, d_xgen.p, d_p2p_err.p, p2p_fold4() ? 4 : 2);
            else
                hipLaunchKernelGGL(ba_schur_chunks, dim3(G.n_chunk), dim3(kSchurThreads), 0, stream, G, pr, wk,
                                   lm_args(cfg), 1);
            RSVIO_HIP(hipGetLastError());
            switch (G.n_free) {
#define RSVIO_CAMP(NF) \
    case NF:                                                                                                            \
        if (p2p.ll)                                                                                                     \
            hipLaunchKernelGGL((ba_camera_solve_mfma_p2p<NF, true>), dim3(1), dim3(kK5Threads), 0, stream, G, pr, wk,  \
                               p2p, d_xgen.p, d_p2p_err.p);                                                            \
        else                                                                                                            \
            hipLaunchKernelGGL((ba_camera_solve_mfma_p2p<NF, false>), dim3(1), dim3(kK5Threads), 0, stream, G, pr, wk, \
                               p2p, d_xgen.p, d_p2p_err.p);                                                            \
        break;
                RSVIO_CAMP(1) RSVIO_CAMP(2) RSVIO_CAMP(3) RSVIO_CAMP(4) RSVIO_CAMP(5)
                RSVIO_CAMP(6) RSVIO_CAMP(7) RSVIO_CAMP(8) RSVIO_CAMP(9) RSVIO_CAMP(10)
#undef RSVIO_CAMP
                default: throw std::logic_error("p2p_fold: more than 10 free keyframes");
            }
            RSVIO_HIP(hipGetLastError());
        } else {
            enqueue_linear_system(it, lm_args(cfg), false);
            launch_camera_solve(pr, wk, sharded() ? 0 : 1);
        }
        if (p2p_fold2()) {  // K6 pushes its wave partials; the next decision sums them (no X2)
            if (G.n_wave)
                hipLaunchKernelGGL(ba_backsub_relinearize_p2p, dim3(G.n_wave), dim3(64), 0, stream, G, pr, wk, p2p,
                                   d_xgen.p);
            RSVIO_HIP(hipGetLastError());
            return;
        }
        if (p2p_fold4()) {  // K6, its last wave pushing this rank's trial scalars (no X2, no wait)
            hipLaunchKernelGGL(ba_backsub_relinearize_p2p4, dim3(std::max(G.n_wave, 1)), dim3(64), 0, stream, G, pr,
                               wk, p2p, d_xgen.p, d_k6cnt.p, d_k6tag.p);
            RSVIO_HIP(hipGetLastError());
            return;
        }
        if (p2p_fold3()) {  // K6 + its reducer workgroup: the trial exchange without X2
            hipLaunchKernelGGL(ba_backsub_relinearize_p2p3, dim3(G.n_wave + 1), dim3(64), 0, stream, G, pr, wk, p2p,
                               d_xgen.p, d_p2p_err.p, d_k6tag.p);
            RSVIO_HIP(hipGetLastError());
            return;
        }
        if (G.n_wave) hipLaunchKernelGGL(ba_backsub_relinearize, dim3(G.n_wave), dim3(64), 0, stream, G, pr, wk);
        RSVIO_HIP(hipGetLastError());
        if (coll == 2) {  // P2P: trial scalars + exchange in one launch (X2)
            hipLaunchKernelGGL(ba_p2p_trial, dim3(1), dim3(256), 0, stream, G, pr, wk, p2p, d_xgen.p, d_p2p_err.p);
            RSVIO_HIP(hipGetLastError());
        } else if (sharded()) {
            hipLaunchKernelGGL(ba_reduce_trial, dim3(1), dim3(64), 0, stream, G, pr, wk, rank == 0 ? 1 : 0);
            RSVIO_HIP(hipGetLastError());
            allreduce(d_trial4.p, 4);
        }
    }

    // K7: the decision pending after `it` iterations, in place in state copy it & 1
    void enqueue_decide(const rsvio_lm_cfg& cfg, int it) {
        // reads state copy it & 1 (the last iteration's pending trial), writes copy (it + 1) & 1
        if (p2p_fold2() || p2p_fold4()) {
            hipLaunchKernelGGL(ba_lm_decide_p2p, dim3(export_on ? kK7Blocks : 1), dim3(kK7Threads), 0, stream, G,
                               prob(), work(it), lm_args(cfg), h_state.p, h_tick, export_on ? h_out.p : nullptr, p2p,
                               d_xgen.p, d_p2p_err.p, p2p_fold4() ? 4 : 2);
            RSVIO_HIP(hipGetLastError());
            return;
        }
        hipLaunchKernelGGL(ba_lm_decide, dim3(export_on ? kK7Blocks : 1), dim3(kK7Threads), 0, stream, G, prob(),
                           work(it), sharded() ? 1 : 0, lm_args(cfg), h_state.p, h_tick, export_on ? h_out.p : nullptr);
        RSVIO_HIP(hipGetLastError());
    }

    // descriptor mode (start_graph): K4, the LM iterations and K7 from the device descriptor, K4 / K6 on
    // wcap >= n_wave workgroups -- the same kernels' bodies as enqueue_start / _iteration / _decide
    void enqueue_start_d(double lambda0, int wcap) {
        hipLaunchKernelGGL(bab_linearize, dim3(wcap, 1), dim3(64), 0, stream, dptr(), lambda0);
        RSVIO_HIP(hipGetLastError());
    }
    void enqueue_iteration_d(const rsvio_lm_cfg& cfg, int it, int wcap) {
        const int wi = it & 1;  // work(it) depends on the parity of it only
        hipLaunchKernelGGL(bab_schur_chunks, dim3(G.n_chunk, 1), dim3(kSchurThreads), 0, stream, dptr(), wi, lm_args(cfg));
        RSVIO_HIP(hipGetLastError());
        switch (G.n_free) {
#define RSVIO_CAMD(NF) \
    case NF: hipLaunchKernelGGL(bab_camera_solve<NF>, dim3(1), dim3(kK5Threads), 0, stream, dptr(), wi); break;
            RSVIO_CAMD(1) RSVIO_CAMD(2) RSVIO_CAMD(3) RSVIO_CAMD(4) RSVIO_CAMD(5)
            RSVIO_CAMD(6) RSVIO_CAMD(7) RSVIO_CAMD(8) RSVIO_CAMD(9) RSVIO_CAMD(10)
#undef RSVIO_CAMD
            default: throw std::logic_error("descriptor mode: more than 10 free keyframes");
        }
        RSVIO_HIP(hipGetLastError());
        hipLaunchKernelGGL(bab_backsub_relinearize, dim3(wcap, 1), dim3(64), 0, stream, dptr(), wi);
        RSVIO_HIP(hipGetLastError());
    }
    void enqueue_decide_d(const rsvio_lm_cfg& cfg, int it) {
        hipLaunchKernelGGL(bad_lm_decide, dim3(export_on ? kK7Blocks : 1), dim3(kK7Threads), 0, stream, dptr(), it & 1,
                           lm_args(cfg), h_state.p, h_tick, export_on ? h_out.p : nullptr);
        RSVIO_HIP(hipGetLastError());
    }

    // Pipelined solve: start() enqueues the reset and the first chunk of LM iterations and
    // returns; finish() waits, enqueues further chunks while the LM has not terminated, and
    // fills the result.  run() = start() + finish().  The host reads the LM state once per
    // chunk; the first chunk is the previous solve's iteration count (consecutive windows
    // converge alike), so the common case costs one read-back and no iteration enqueued after
    // convergence.
    struct Pending {
        bool active = false, skipped = false;
        bool by_tick = false;  // the wait mode fixed at start(): finish() never switches it mid-solve
        rsvio_lm_cfg cfg{};
        int enq = 0, max_it = 0;
    } pend;

    void enqueue_chunk(int k) {
        settled = false;
        for (int i = 0; i < k; ++i) enqueue_iteration(pend.cfg, pend.enq + i);
        pend.enq += k;
        enqueue_decide(pend.cfg, pend.enq);  // K7 also writes the state into h_state
        ++n_tick;
        if (!pend.by_tick) RSVIO_HIP(hipEventRecord(ev1, stream));
    }

    // After a failed enqueue or a lost ticket the host's ticket count may be off by the decisions
    // that did (not) reach the queue: settle the stream and take the device's count.
    void resync_ticks() noexcept {
        (void)hipStreamSynchronize(stream);
        (void)hipGetLastError();
        settled = true;
        unsigned long long t = 0;
        if (hipMemcpy(&t, d_tick.p, sizeof t, hipMemcpyDeviceToHost) == hipSuccess) n_tick = t;
        pend.active = false;
    }

    void start(const rsvio_lm_cfg& cfg) {
        // refusals first: they leave an in-flight solve untouched
        if (!has_problem) throw std::invalid_argument("no problem uploaded");
        if (pend.active) throw CallOrderError("a solve is already in flight (call finish first)");
        try {
            start_impl(cfg);
        } catch (...) {
            resync_ticks();
            throw;
        }
    }

    void start_impl(const rsvio_lm_cfg& cfg) {
        G.huber_delta = cfg.huber_delta;
        G.chol = cfg.linear_solver == RSVIO_SOLVER_CHOLESKY ? 1 : 0;
        pend = Pending{};
        pend.active = true;
        pend.cfg = cfg;
        pend.by_tick = by_tick();
        state_export = false;
        // sliding_window.rs:303-319: too few residuals / underconstrained -> skipped (Ok(false))
        if (!sharded() && (G.n_obs < 6 || G.n_obs < G.n_kf + G.n_lm)) {
            pend.skipped = true;
            return;
        }
        pend.max_it = std::max(cfg.max_iterations, 1);
        settled = false;
        state_fresh = false;  // K4 (K0 folded in) sets both state buffers
        if (!pend.by_tick) RSVIO_HIP(hipEventRecord(ev0, stream));  // the ticket carries device stamps
        int k = std::min(std::max(last_iterations, 1), pend.max_it);
        // a new problem (every keyframe in the Estimator) is re-captured: capture + instantiate +
        // one launch measured cheaper in host time than its ~25 direct launches (config-4 BA stage
        // 0.100 vs 0.115 ms per frame, round 2), so graphs stay on for fresh problems too
        if (start_graph(cfg, k)) {
            ++n_tick;
            pend.enq += k;
            if (!pend.by_tick) RSVIO_HIP(hipEventRecord(ev1, stream));
        } else {
            enqueue_start(cfg.lambda_init);
            enqueue_chunk(k);
        }
    }

    void finish(rsvio_ba_result* res) {
        if (!pend.active) throw CallOrderError("no solve in flight");
        try {
            finish_impl(res);
        } catch (...) {
            resync_ticks();
            throw;
        }
    }

    void finish_impl(rsvio_ba_result* res) {
        pend.active = false;
        res->iterations = 0;
        if (pend.skipped) {
            res->status = RSVIO_LM_SKIPPED;
            res->initial_cost = res->final_cost = 0.0;
            res->solve_ms = 0.0;
            return;
        }
        // return as soon as the last decision's ticket lands in pinned host memory (its state was
        // written before it); the stream settles before anything else touches the handle's
        // buffers (require_idle).  RSVIO_BA_WAIT=sync: stream sync.
        const bool by_tick = pend.by_tick;
        while (true) {
            if (by_tick)
                wait_tick();
            else
                RSVIO_HIP(hipStreamSynchronize(stream));
            if (h_state.p->done || pend.enq >= pend.max_it) break;
            enqueue_chunk(std::min(iter_chunk, pend.max_it - pend.enq));
        }
        up_pending = false;  // (the ticket comes after the window's upload in stream order)
        last_iterations = h_state.p->iter;
        if (coll == 2) {  // the exchange error flag came with the ticket (K7); the sync path reads it
            if (by_tick) {
                if (h_state.p->p2p_err) {
                    settle();
                    throw std::runtime_error("P2P all-reduce: a peer did not arrive");
                }
            } else {
                p2p_check();
            }
        }
        state_export = export_on && h_state.p->done != 0;  // the final K7 exported it with its ticket
        float ms = 0.0f;
        if (by_tick) {
            ms = (float)((double)(h_tick[2] - h_tick[1]) / wclk_khz);
        } else {
            settled = true;
            RSVIO_HIP(hipEventElapsedTime(&ms, ev0, ev1));
        }
        const LmState& s = *h_state.p;
        res->status = s.status;
        res->iterations = s.iter;
        res->initial_cost = s.initial_cost;
        res->final_cost = s.cost;
        res->solve_ms = ms;
    }

    // ---- peer-to-peer collective (sharded path) ----
    void p2p_export(int nr, hipIpcMemHandle_t* h) {
        if (nr < 1 || nr > kP2PMax) throw std::invalid_argument("P2P: 1..8 ranks");
        if (!xbuf) {
            const size_t bytes = kP2PBytes;
            RSVIO_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&xbuf), bytes, hipDeviceMallocUncached));
            RSVIO_HIP(hipMemset(xbuf, 0, bytes));
            d_p2p_err.alloc(1);
            RSVIO_HIP(hipMemset(d_p2p_err.p, 0, sizeof(int)));
            d_xgen.alloc(1);
            RSVIO_HIP(hipMemset(d_xgen.p, 0, sizeof(unsigned long long)));
            d_xnw.alloc(kP2PMax);
            RSVIO_HIP(hipMemset(d_xnw.p, 0, sizeof(int) * kP2PMax));
        }
        RSVIO_HIP(hipIpcGetMemHandle(h, xbuf));
    }

    void p2p_check() {
        int err = 0;
        RSVIO_HIP(hipMemcpy(&err, d_p2p_err.p, sizeof(int), hipMemcpyDeviceToHost));
        if (err) throw std::runtime_error("P2P all-reduce: a peer did not arrive");
    }

    // open the peers' exchange buffers and self-test one all-reduce; on any failure the
    // handle keeps its previous collective
    void p2p_attach(int nr, int rk, const hipIpcMemHandle_t* hs) {
        require_idle("rsvio_ba_attach_p2p");
        if (nr < 1 || nr > kP2PMax || rk < 0 || rk >= nr) throw std::invalid_argument("P2P: bad rank layout");
        if (!xbuf) throw CallOrderError("P2P: export the buffer first");
        P2P P{};
        P.nranks = nr;
        P.rank = rk;
        P.xnw = d_xnw.p;
        const char* llv = std::getenv("RSVIO_P2P_LL");  // "1": K5's system exchange flag-in-word (A/B)
        P.ll = llv && llv[0] == '1';
        for (int r = 0; r < nr; ++r) {
            if (r == rk) {
                P.peer[r] = xbuf;
                continue;
            }
            void* ptr = nullptr;
            RSVIO_HIP(hipIpcOpenMemHandle(&ptr, hs[r], hipIpcMemLazyEnablePeerAccess));
            P.peer[r] = static_cast<double*>(ptr);
            p2p_opened[r] = true;
        }
        // self-test, which also makes the ranks agree on the exchange protocol: rank r contributes
        // r + 1 and 1 (every rank must read nr (nr + 1) / 2 and nr), its fold level and flag-in-word
        // switch with their squares (all ranks hold the same value iff sum = nr v and sum of squares
        // = nr v^2 on every rank: a mismatch fails on EVERY rank, so all keep their previous
        // collective together), and its device's PCI location in entry 6 + r (so every rank sees
        // which ranks share a GPU)
        int pci_dom = 0, pci_bus = 0, pci_dev = 0;
        RSVIO_HIP(hipDeviceGetAttribute(&pci_dom, hipDeviceAttributePciDomainID, this->P.device));
        RSVIO_HIP(hipDeviceGetAttribute(&pci_bus, hipDeviceAttributePciBusId, this->P.device));
        RSVIO_HIP(hipDeviceGetAttribute(&pci_dev, hipDeviceAttributePciDeviceId, this->P.device));
        constexpr int kSelf = 6 + kP2PMax;
        static_assert(kSelf <= kP2PLLMax, "the self-test is one flag-in-word message");
        double tv[kSelf] = {};
        const double fl = (double)fold_req, lv = P.ll ? 1.0 : 0.0;
        tv[0] = rk + 1; tv[1] = 1.0; tv[2] = fl; tv[3] = fl * fl; tv[4] = lv; tv[5] = lv * lv;
        tv[6 + rk] = 1.0 + (double)(((long long)pci_dom << 16) | (pci_bus << 8) | pci_dev);
        const int n_self = 6 + nr;
        DevBuf<double> t(kSelf);
        RSVIO_HIP(hipMemcpy(t.p, tv, sizeof(double) * n_self, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(ba_p2p_allreduce, dim3(1), dim3(256), 0, stream, t.p, n_self, P, d_xgen.p, d_p2p_err.p);
        RSVIO_HIP(hipGetLastError());
        double out[kSelf] = {};
        RSVIO_HIP(hipMemcpyAsync(out, t.p, sizeof(double) * n_self, hipMemcpyDeviceToHost, stream));
        RSVIO_HIP(hipStreamSynchronize(stream));
        p2p_check();
        if (out[0] != nr * (nr + 1) / 2.0 || out[1] != (double)nr)
            throw std::runtime_error("P2P all-reduce self-test returned wrong sums");
        if (out[2] != nr * fl || out[3] != nr * fl * fl || out[4] != nr * lv || out[5] != nr * lv)
            throw std::runtime_error("P2P: the ranks disagree on RSVIO_P2P_FOLD / RSVIO_P2P_LL");
        bool shared_gpu = false;
        for (int a = 0; a < nr; ++a)
            for (int b = a + 1; b < nr; ++b) shared_gpu |= out[6 + a] == out[6 + b];
        // fold 2's K4c blocks poll every rank's K6 partials while they hold CUs: on a shared GPU
        // they can starve a peer's K6 until the spin bound, so co-resident ranks take fold 1 (all
        // ranks see the same codes and decide alike)
        // (RSVIO_P2P_FOLD_SHARED=1 keeps fold 2 anyway: the A/B test of its sums on one GPU)
        const char* fsv = std::getenv("RSVIO_P2P_FOLD_SHARED");
        const bool keep2 = fsv && fsv[0] == '1';
        // (ranks sharing one GPU: a decision that waits in K4c -- folds 2 and 4 -- can starve a
        // peer's K6 of CUs; they take the nearest level that waits inside K6 or K5 instead)
        fold_lvl = shared_gpu && !keep2 && (fold_req == 2 || fold_req == 4) ? fold_req - 1 : fold_req;
        p2p_shared_gpu = shared_gpu;
        p2p_share = 0;
        for (int a = 0; a < nr; ++a) p2p_share += out[6 + a] == out[6 + rk];
        refresh_k6_cap();
        p2p = P;
        nranks = nr;
        rank = rk;
        coll = 2;
        drop_graph();  // the iteration's launch sequence changes with the collective
    }

    // fold 3's resident capacity: K6 workgroups per CU (occupancy of the reducer kernel, one wave
    // each) x the CUs the stream may use (its CU mask), shared among the ranks on this device
    void refresh_k6_cap() {
        int per_cu = 0;
        RSVIO_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(ba_backsub_relinearize_p2p3), 64, 0));
        int n_cu = 0;
        RSVIO_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, P.device));
        uint32_t mask[32] = {};
        if (hipExtStreamGetCUMask(stream, 32, mask) == hipSuccess) {
            int c = 0;
            for (uint32_t w : mask) c += __builtin_popcount(w);
            if (c > 0) n_cu = std::min(n_cu, c);
        } else {
            (void)hipGetLastError();
        }
        const char* ov = std::getenv("RSVIO_K6_CAP");  // test hook: pretend a smaller capacity
        k6_cap = per_cu * n_cu / std::max(p2p_share, 1);
        if (ov && ov[0]) k6_cap = std::min(k6_cap, std::atoi(ov));
    }
    // the exchange level the current problem's iterations take: -1 not P2P-sharded, 0 X1 + X2
    // launches, 1 K5 exchange + X2, 2 / 3 / 4 the folded trial exchanges
    int p2p_level() const {
        if (coll != 2) return -1;
        if (!p2p_fold()) return 0;
        return p2p_fold2() ? 2 : p2p_fold3() ? 3 : p2p_fold4() ? 4 : 1;
    }

    // measured exchange latency: one warm-up exchange (absorbs the ranks' start skew), then reps
    // back-to-back exchanges of n doubles timed with events on this handle's stream; every rank
    // must make the same call.  Average device microseconds per exchange.
    double p2p_latency(int reps, int n) {
        require_idle("rsvio_ba_p2p_latency");
        if (coll != 2) throw CallOrderError("P2P latency: the P2P exchange is not attached");
        if (reps < 1 || n < 1 || n > kP2PMsg) throw std::invalid_argument("P2P latency: bad reps or size");
        DevBuf<double> t(n);
        RSVIO_HIP(hipMemsetAsync(t.p, 0, (size_t)n * sizeof(double), stream));
        hipEvent_t a, b;
        RSVIO_HIP(hipEventCreate(&a));
        RSVIO_HIP(hipEventCreate(&b));
        for (int k = 0; k <= reps; ++k) {
            if (k == 1) RSVIO_HIP(hipEventRecord(a, stream));
            hipLaunchKernelGGL(ba_p2p_allreduce, dim3(1), dim3(256), 0, stream, t.p, n, p2p, d_xgen.p, d_p2p_err.p);
        }
        RSVIO_HIP(hipGetLastError());
        RSVIO_HIP(hipEventRecord(b, stream));
        RSVIO_HIP(hipEventSynchronize(b));
        float ms = 0.f;
        RSVIO_HIP(hipEventElapsedTime(&ms, a, b));
        RSVIO_HIP(hipEventDestroy(a));
        RSVIO_HIP(hipEventDestroy(b));
        p2p_check();
        return 1e3 * (double)ms / reps;
    }

    void p2p_detach() {
        require_idle("rsvio_ba_detach_p2p");
        if (coll == 2) coll = comm ? 1 : 0;
        drop_graph();
    }

    // run on a caller-owned stream (e.g. one restricted to a CU subset); nullptr = own stream
    void set_stream(hipStream_t s) {
        if (pend.active) throw CallOrderError("a solve is in flight");
        RSVIO_HIP(hipStreamSynchronize(stream));
        if (s) {
            if (own_stream) RSVIO_HIP(hipStreamDestroy(stream));
            stream = s;
            own_stream = false;
        } else if (!own_stream) {
            RSVIO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
            own_stream = true;
        }
        if (coll == 2) {
            refresh_k6_cap();
            drop_graph();  // (fold 3 may come or go with the stream's CUs)
        }
    }

    void run(const rsvio_lm_cfg& cfg, rsvio_ba_result* res) {
        start(cfg);
        finish(res);
    }

    // entry points that read or replace what an in-flight solve uses (rsvio_ba_run_async before
    // rsvio_ba_wait) are refused, as set_stream is
    // every collective waits on the decision ticket (RSVIO_BA_WAIT=sync: on the stream + events):
    // K7 is enqueued after the chunk's last exchange on the same stream, so its ticket lands only
    // after the exchanges completed -- ours (P2P: K7 also publishes their error flag with it) or
    // RCCL's all-reduces.  A failed RCCL collective never lets K7 run: the bounded spin (1 s) then
    // synchronises the stream, which reports the error (a slow peer merely ends the spin late).
    bool by_tick() const { return tick_wait; }

    void require_idle(const char* what) {
        if (pend.active) throw CallOrderError(std::string(what) + ": a solve is in flight (call rsvio_ba_wait first)");
        settle();
    }

    // the stream's tail after a ticket (the decision kernel's exit, its cache write-back) is
    // drained before host-side copies touch the buffers
    void settle() {
        if (!settled) {
            RSVIO_HIP(hipStreamSynchronize(stream));
            settled = true;
        }
        up_pending = false;
        destroy_retired();
    }

    // spin on the ticket of the last enqueued decision; a bounded spin (1 s) falls back to a
    // stream sync, which reports a device error if there was one
    void wait_tick() {
        const unsigned long long want = n_tick;
        auto t0 = std::chrono::steady_clock::now();
        for (unsigned it = 1;; ++it) {
            if (__atomic_load_n(h_tick, __ATOMIC_ACQUIRE) >= want) return;
            if ((it & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
                RSVIO_HIP(hipStreamSynchronize(stream));
                settled = true;
                if (__atomic_load_n(h_tick, __ATOMIC_ACQUIRE) >= want) return;
                throw std::runtime_error("BA: the decision ticket never arrived");
            }
            __builtin_ia32_pause();
        }
    }

    // every export slot carries this solve's start stamp (h_tick[1], published with the ticket);
    // false after a bounded spin (the caller then settles and copies from the device)
    bool wait_export() {
        const unsigned long long want = h_tick[1];
        auto t0 = std::chrono::steady_clock::now();
        for (int b = 0; b < kK7Blocks; ++b)
            for (unsigned it = 1; __atomic_load_n(h_tick + 4 + b, __ATOMIC_ACQUIRE) != want; ++it) {
                if ((it & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) {
                    state_export = false;
                    return false;
                }
                __builtin_ia32_pause();
            }
        return true;
    }

    void get_state(double* pose7, double* pW) {
        if (pend.active) throw CallOrderError("get_state: a solve is in flight (call rsvio_ba_wait first)");
        if (state_export && wait_export()) {  // the final decision's slices: no stream sync needed
            std::memcpy(pose7, h_out.p, sizeof(double) * 7 * G.n_kf);
            if (G.n_lm) std::memcpy(pW, h_out.p + 7 * G.n_kf, sizeof(double) * 3 * G.n_lm);
            return;
        }
        export_on = true;  // from the next solve on, its final decision exports the state
        require_idle("get_state");
        if (state_fresh) {  // no solve since set_problem: the initial state into both buffers
            enqueue_reset(1e-4);
            state_fresh = false;
        }
        const int cur = h_state.p->cur;
        const Work wk = work_at(0);
        RSVIO_HIP(hipMemcpyAsync(pose7, wk.pose[cur], sizeof(double) * 7 * G.n_kf, hipMemcpyDeviceToHost, stream));
        if (G.n_lm)
            RSVIO_HIP(hipMemcpyAsync(pW, wk.pw[cur], sizeof(double) * 3 * G.n_lm, hipMemcpyDeviceToHost, stream));
        RSVIO_HIP(hipStreamSynchronize(stream));
    }

    void build_system(double lambda, double huber_delta, double* S, double* b, double* cost) {
        require_idle("build_system");
        state_export = false;  // K4 below resets the state buffers
        if (!has_problem) throw std::invalid_argument("no problem uploaded");
        G.huber_delta = huber_delta;
        G.chol = 0;
        enqueue_start(lambda);
        enqueue_linear_system(0, LmArgs{1, 0.0, 0.0}, true);
        std::vector<double> sys((size_t)36 * G.n_pb + 12 * G.n_free + 2);
        RSVIO_HIP(hipMemcpyAsync(sys.data(), d_sys.p, sizeof(double) * sys.size(), hipMemcpyDeviceToHost, stream));
        RSVIO_HIP(hipMemcpyAsync(h_state.p, d_state.p + 1, sizeof(LmState), hipMemcpyDeviceToHost, stream));
        RSVIO_HIP(hipStreamSynchronize(stream));
        const int n = 6 * G.n_free;
        std::vector<int> fa, fb;
        for (int a = 0; a < G.n_free; ++a)
            for (int c = a; c < G.n_free; ++c) {
                fa.push_back(a);
                fb.push_back(c);
            }
        for (int pb = 0; pb < G.n_pb; ++pb)
            for (int e = 0; e < 36; ++e) {
                const int a = e / 6, c = e % 6;
                S[(size_t)(6 * fa[pb] + a) * n + 6 * fb[pb] + c] = sys[pb * 36 + e];
                if (fa[pb] != fb[pb]) S[(size_t)(6 * fb[pb] + c) * n + 6 * fa[pb] + a] = sys[pb * 36 + e];
            }
        for (int i = 0; i < n; ++i) b[i] = sys[36 * G.n_pb + i];
        *cost = sys[36 * G.n_pb + 12 * G.n_free];
    }

    // diagnostic: one reduced system at lambda and its camera solve (K4c + K5) -> dc
    void camera_step(double lambda, double huber_delta, double* dc) {
        require_idle("camera_step");
        state_export = false;
        if (!has_problem) throw std::invalid_argument("no problem uploaded");
        G.huber_delta = huber_delta;
        G.chol = 0;
        enqueue_start(lambda);
        enqueue_linear_system(0, LmArgs{1, 0.0, 0.0}, false);
        launch_camera_solve(prob(), work(0), sharded() ? 0 : 1);
        RSVIO_HIP(hipMemcpyAsync(dc, d_dc.p, sizeof(double) * 6 * G.n_free, hipMemcpyDeviceToHost, stream));
        RSVIO_HIP(hipStreamSynchronize(stream));
    }
};

// Batched mode over B window handles (their problems uploaded by rsvio_ba_set_problem): one
// launch chain on the batch's stream, the host reading the B LM states once per chunk.
struct BundleBatch {
    std::vector<BundleAdjuster*> win;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    DevBuf<WinDesc> d_desc;
    HostBuf<WinDesc> h_desc;
    HostBuf<LmState> h_states;
    DevBuf<int> d_dmap;
    HostBuf<int> h_dmap;
    std::vector<hipEvent_t> ev_win;  // per window: its stream's pending work (an upload) before the batch
    int last_iterations = 3;

    void init(BundleAdjuster* const* w, int n) {
        if (n < 1) throw std::invalid_argument("a batch needs at least one window");
        for (int i = 0; i < n; ++i) {
            if (!w[i]) throw std::invalid_argument("null window handle");
            if (i && w[i]->P.device != w[0]->P.device) throw std::invalid_argument("windows on different devices");
            if (w[i]->sharded()) throw std::invalid_argument("a sharded window cannot join a batch");
            for (int j = 0; j < i; ++j)  // two grid rows on one set of state buffers would race
                if (w[j] == w[i]) throw std::invalid_argument("a window handle appears twice in the batch");
            win.push_back(w[i]);
        }
        device = w[0]->P.device;
        RSVIO_HIP(hipSetDevice(device));
        RSVIO_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        RSVIO_HIP(hipEventCreate(&ev0));
        RSVIO_HIP(hipEventCreate(&ev1));
        ev_win.assign(n, nullptr);
        for (int i = 0; i < n; ++i) RSVIO_HIP(hipEventCreateWithFlags(&ev_win[i], hipEventDisableTiming));
        d_desc.alloc(n);
        h_desc.alloc(n);
        h_states.alloc(n, hipHostMallocCoherent);
    }
    ~BundleBatch() {
        if (stream) (void)hipStreamSynchronize(stream);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        for (hipEvent_t e : ev_win)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }

    void launch_k5(int nf, int wi) {
        const int B = (int)win.size();
        switch (nf) {
#define RSVIO_BAB(NF) \
    case NF: hipLaunchKernelGGL(bab_camera_solve<NF>, dim3(B), dim3(kK5Threads), 0, stream, d_desc.p, wi); break;
            RSVIO_BAB(1) RSVIO_BAB(2) RSVIO_BAB(3) RSVIO_BAB(4) RSVIO_BAB(5)
            RSVIO_BAB(6) RSVIO_BAB(7) RSVIO_BAB(8) RSVIO_BAB(9) RSVIO_BAB(10)
#undef RSVIO_BAB
            case 13: hipLaunchKernelGGL(bab_camera_solve_blk<13>, dim3(B), dim3(64 * kBkWaves), 0, stream, d_desc.p, wi); break;
            case 16: hipLaunchKernelGGL(bab_camera_solve_blk<16>, dim3(B), dim3(64 * kBkWaves), 0, stream, d_desc.p, wi); break;
            case 20: hipLaunchKernelGGL(bab_camera_solve_blk<20>, dim3(B), dim3(64 * kBkWaves), 0, stream, d_desc.p, wi); break;
            default: throw std::logic_error("batched mode: no camera-solve template for this window size");
        }
        RSVIO_HIP(hipGetLastError());
    }

    void run(const rsvio_lm_cfg& cfg, rsvio_ba_result* res) {
        const int B = (int)win.size();
        int nf = 1, max_wave = 1, max_chunk = 1, active = 0;
        std::vector<int> skip(B, 0);
        size_t ne_total = 0;
        for (int i = 0; i < B; ++i) {
            BundleAdjuster& w = *win[i];
            if (w.pend.active) throw CallOrderError("rsvio_ba_batch_run: a solve is in flight (call rsvio_ba_wait first)");
            w.state_export = false;  // the batch's decisions leave the state in device memory
            if (!w.has_problem) throw std::invalid_argument("batch window without a problem");
            const Geometry& G = w.G;
            // sliding_window.rs:303-319 guards, as the single-window start()
            skip[i] = (G.n_obs < 6 || G.n_obs < G.n_kf + G.n_lm || G.n_wave == 0) ? 1 : 0;
            if (skip[i]) continue;
            ++active;
            nf = std::max(nf, G.n_free);
            max_wave = std::max(max_wave, G.n_wave);
            max_chunk = std::max(max_chunk, G.n_chunk);
            ne_total += (size_t)36 * G.n_pb + 12 * G.n_free;
        }
        // past 10 free keyframes every window runs the 6x6-block solver's padded template
        if (nf > 10) nf = bk_template_nf(nf);
        max_wave = (max_wave + kGrp - 1) / kGrp * kGrp;  // wave w on XCD w % 8 in every window
        // descriptors and the camera-solve maps for the batch's template (b row at 6 nf)
        if (h_dmap.n < std::max<size_t>(ne_total, 1)) {
            h_dmap.alloc(ne_total + 1);
            d_dmap.alloc(ne_total + 1);
        }
        size_t off = 0;
        for (int i = 0; i < B; ++i) {
            BundleAdjuster& w = *win[i];
            WinDesc& d = h_desc.p[i];
            d.skip = skip[i];
            d.G = w.G;
            d.G.huber_delta = cfg.huber_delta;
            d.G.chol = cfg.linear_solver == RSVIO_SOLVER_CHOLESKY ? 1 : 0;
            d.Pr = w.prob();
            d.W[0] = w.work(0);
            d.W[1] = w.work(1);
            d.W[2] = w.work_at(0);
            d.W[3] = w.work_at(1);
            if (skip[i]) continue;
            const size_t ne = (size_t)36 * w.G.n_pb + 12 * w.G.n_free;
            mf_dense_map(w.G.n_free, w.G.n_pb, w.hs_pb_fa.data(), w.hs_pb_fb.data(), h_dmap.p + off, 6 * nf,
                         nf > 10 ? kBkLd : kMfLd);
            d.Pr.dmap = d_dmap.p + off;
            off += ne;
        }
        for (int i = 0; i < B; ++i) {
            if (skip[i]) {
                res[i] = rsvio_ba_result{};
                res[i].status = RSVIO_LM_SKIPPED;
            }
        }
        if (!active) return;
        // the batch's kernels read what each window's stream may still be writing (set_problem's
        // upload and ba_build_layout are asynchronous): the batch stream waits on an event of each
        // window's stream instead of synchronising the host
        for (int i = 0; i < B; ++i) {
            BundleAdjuster& w = *win[i];
            if (w.settled) continue;
            RSVIO_HIP(hipEventRecord(ev_win[i], w.stream));
            RSVIO_HIP(hipStreamWaitEvent(stream, ev_win[i], 0));
        }
        RSVIO_HIP(hipMemcpyAsync(d_dmap.p, h_dmap.p, sizeof(int) * std::max<size_t>(off, 1), hipMemcpyHostToDevice, stream));
        RSVIO_HIP(hipMemcpyAsync(d_desc.p, h_desc.p, sizeof(WinDesc) * B, hipMemcpyHostToDevice, stream));
        RSVIO_HIP(hipEventRecord(ev0, stream));
        hipLaunchKernelGGL(bab_linearize, dim3(max_wave, B), dim3(64), 0, stream, d_desc.p, cfg.lambda_init);
        RSVIO_HIP(hipGetLastError());
        const LmArgs la{cfg.max_iterations, cfg.cost_tolerance, cfg.parameter_tolerance};
        const int max_it = std::max(cfg.max_iterations, 1);
        int enq = 0;
        int k = std::min(std::max(last_iterations, 1), max_it);
        int max_iter_seen = 0;
        while (true) {
            for (int i = 0; i < k; ++i, ++enq) {
                const int wi = enq & 1;
                hipLaunchKernelGGL(bab_schur_chunks, dim3(max_chunk, B), dim3(kSchurThreads), 0, stream, d_desc.p, wi, la);
                RSVIO_HIP(hipGetLastError());
                launch_k5(nf, wi);
                hipLaunchKernelGGL(bab_backsub_relinearize, dim3(max_wave, B), dim3(64), 0, stream, d_desc.p, wi);
                RSVIO_HIP(hipGetLastError());
            }
            hipLaunchKernelGGL(bab_lm_decide, dim3(B), dim3(64), 0, stream, d_desc.p, 2 + (enq & 1), la, h_states.p);
            RSVIO_HIP(hipGetLastError());
            RSVIO_HIP(hipEventRecord(ev1, stream));
            RSVIO_HIP(hipStreamSynchronize(stream));
            bool all_done = true;
            for (int i = 0; i < B; ++i)
                if (!skip[i]) {
                    all_done = all_done && h_states.p[i].done;
                    max_iter_seen = std::max(max_iter_seen, h_states.p[i].iter);
                }
            if (all_done || enq >= max_it) break;
            k = std::min(2, max_it - enq);
        }
        float ms = 0.0f;
        RSVIO_HIP(hipEventElapsedTime(&ms, ev0, ev1));
        last_iterations = std::max(max_iter_seen, 1);
        for (int i = 0; i < B; ++i) {
            if (skip[i]) continue;
            BundleAdjuster& w = *win[i];
            const LmState& st = h_states.p[i];
            *w.h_state.p = st;
            w.state_fresh = false;
            // the window's stream ran nothing after the event the batch waited on, and the batch
            // stream is synchronised: both are idle
            w.settled = true;
            w.destroy_retired();
            w.last_iterations = st.iter;
            res[i].status = st.status;
            res[i].iterations = st.iter;
            res[i].initial_cost = st.initial_cost;
            res[i].final_cost = st.cost;
            res[i].solve_ms = ms;
        }
    }
};

}  // namespace rsvio

struct rsvio_ba {
    rsvio::BundleAdjuster b;
};

struct rsvio_ba_batch {
    rsvio::BundleBatch b;
};

using rsvio::guarded;

extern "C" {

int rsvio_ba_create(const rsvio_ba_params* params, rsvio_ba** out) {
    if (!params || !out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto* h = new rsvio_ba();
        try {
            h->b.init(*params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
        return (int)RSVIO_OK;
    });
}

void rsvio_ba_destroy(rsvio_ba* ba) { delete ba; }

static bool problem_args_ok(int32_t n_kf, const double* pose7, const uint8_t* kf_fixed, int32_t n_lm, const double* p_W,
                            int32_t n_obs, const int32_t* obs_lm, const int32_t* obs_kf, const uint8_t* obs_cam,
                            const double* obs_uv, const double* T_C_B2) {
    if (n_kf < 1 || n_lm < 0 || n_obs < 0 || !pose7 || !kf_fixed || !T_C_B2) return false;
    if (n_lm > 0 && !p_W) return false;
    if (n_obs > 0 && (!obs_lm || !obs_kf || !obs_cam || !obs_uv)) return false;
    return true;
}

int rsvio_ba_set_problem(rsvio_ba* ba, int32_t n_kf, const double* pose7, const uint8_t* kf_fixed, int32_t n_lm,
                         const double* p_W, int32_t n_obs, const int32_t* obs_lm, const int32_t* obs_kf,
                         const uint8_t* obs_cam, const double* obs_uv, const double* T_C_B2) {
    if (!ba || !problem_args_ok(n_kf, pose7, kf_fixed, n_lm, p_W, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2))
        return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.set_problem(n_kf, pose7, kf_fixed, n_lm, p_W, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_run(rsvio_ba* ba, const rsvio_lm_cfg* cfg, rsvio_ba_result* res) {
    if (!ba || !cfg || !res) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.run(*cfg, res);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_set_stream(rsvio_ba* ba, void* stream) {
    if (!ba) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.set_stream(static_cast<hipStream_t>(stream));
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_run_async(rsvio_ba* ba, const rsvio_lm_cfg* cfg) {
    if (!ba || !cfg) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.start(*cfg);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_wait(rsvio_ba* ba, rsvio_ba_result* res) {
    if (!ba || !res) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.finish(res);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_get_state(rsvio_ba* ba, double* pose7, double* p_W) {
    if (!ba || !pose7 || (!p_W && ba->b.G.n_lm)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.get_state(pose7, p_W);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_solve(rsvio_ba* ba, int32_t n_kf, double* pose7, const uint8_t* kf_fixed, int32_t n_lm, double* p_W,
                   int32_t n_obs, const int32_t* obs_lm, const int32_t* obs_kf, const uint8_t* obs_cam,
                   const double* obs_uv, const double* T_C_B2, const rsvio_lm_cfg* cfg, rsvio_ba_result* res) {
    if (!ba || !cfg || !res ||
        !problem_args_ok(n_kf, pose7, kf_fixed, n_lm, p_W, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2))
        return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& B = ba->b;
        B.set_problem(n_kf, pose7, kf_fixed, n_lm, p_W, n_obs, obs_lm, obs_kf, obs_cam, obs_uv, T_C_B2);
        B.run(*cfg, res);
        if (res->status > 0) B.get_state(pose7, p_W);  // success: hand back the optimised state (:364-374)
        return (int)RSVIO_OK;
    });
}

int rsvio_dbg_ba_camera_step(rsvio_ba* ba, double lambda, double huber_delta, double* dc) {
    if (!ba || !dc) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.camera_step(lambda, huber_delta, dc);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_build_system(rsvio_ba* ba, double lambda, double huber_delta, double* S, double* b, double* cost) {
    if (!ba || !S || !b || !cost) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.build_system(lambda, huber_delta, S, b, cost);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_batch_create(rsvio_ba* const* windows, int32_t n, rsvio_ba_batch** out) {
    if (!windows || n < 1 || !out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        std::vector<rsvio::BundleAdjuster*> w(n);
        for (int i = 0; i < n; ++i) w[i] = windows[i] ? &windows[i]->b : nullptr;
        auto* h = new rsvio_ba_batch();
        try {
            h->b.init(w.data(), n);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_batch_run(rsvio_ba_batch* batch, const rsvio_lm_cfg* cfg, rsvio_ba_result* results) {
    if (!batch || !cfg || !results) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        batch->b.run(*cfg, results);
        return (int)RSVIO_OK;
    });
}

void rsvio_ba_batch_destroy(rsvio_ba_batch* batch) { delete batch; }

int rsvio_rccl_unique_id(uint8_t* out, size_t cap) {
    if (!out || cap < sizeof(ncclUniqueId)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ncclUniqueId id;
        if (ncclGetUniqueId(&id) != ncclSuccess) {
            rsvio::set_last_error("ncclGetUniqueId failed");
            return (int)RSVIO_ERR_RCCL;
        }
        __builtin_memcpy(out, &id, sizeof(id));
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_attach_comm(rsvio_ba* ba, int32_t nranks, int32_t rank, const uint8_t* unique_id) {
    if (!ba || !unique_id || nranks < 1 || rank < 0 || rank >= nranks) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        auto& B = ba->b;
        ncclUniqueId id;  // a 1-rank communicator is legal: it runs the sharded code path on one GPU
        __builtin_memcpy(&id, unique_id, sizeof(id));
        RSVIO_HIP(hipSetDevice(B.P.device));
        B.require_idle("rsvio_ba_attach_comm");
        if (ncclCommInitRank(&B.comm, nranks, id, rank) != ncclSuccess) {
            rsvio::set_last_error("ncclCommInitRank failed");
            return (int)RSVIO_ERR_RCCL;
        }
        B.nranks = nranks;
        B.rank = rank;
        B.coll = 1;
        B.drop_graph();
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_p2p_export(rsvio_ba* ba, int32_t nranks, uint8_t* handle_out, size_t cap) {
    if (!ba || !handle_out || cap < sizeof(hipIpcMemHandle_t)) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        hipIpcMemHandle_t h;
        ba->b.p2p_export(nranks, &h);
        __builtin_memcpy(handle_out, &h, sizeof h);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_attach_p2p(rsvio_ba* ba, int32_t nranks, int32_t rank, const uint8_t* handles) {
    if (!ba || !handles) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        std::vector<hipIpcMemHandle_t> hs(nranks > 0 ? nranks : 1);
        for (int r = 0; r < nranks; ++r) __builtin_memcpy(&hs[r], handles + (size_t)r * sizeof(hipIpcMemHandle_t), sizeof(hipIpcMemHandle_t));
        try {
            ba->b.p2p_attach(nranks, rank, hs.data());
        } catch (const rsvio::CallOrderError&) {
            throw;  // refused while a solve is in flight: a caller error, not a P2P failure
        } catch (const std::exception& e) {
            rsvio::set_last_error(std::string("P2P attach failed: ") + e.what());
            return (int)RSVIO_ERR_RCCL;
        }
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_p2p_latency(rsvio_ba* ba, int32_t reps, int32_t n, double* us_out) {
    if (!ba || !us_out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        *us_out = ba->b.p2p_latency(reps, n);
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_p2p_level(rsvio_ba* ba, int32_t* level_out) {
    if (!ba || !level_out) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        *level_out = ba->b.p2p_level();
        return (int)RSVIO_OK;
    });
}

int rsvio_ba_detach_p2p(rsvio_ba* ba) {
    if (!ba) return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        ba->b.p2p_detach();
        return (int)RSVIO_OK;
    });
}

}  // extern "C"
