// window.hip -- host code only (no device work): the Estimator's per-keyframe host logic around
// the BA solve, in C++ instead of the Python mirror's numpy calls (~0.5 ms per keyframe there, the
// largest host cost of the config-4 frame loop):
//   * rsvio_window_problem: SlidingWindow::optimize's problem assembly
//     (src/estimator/sliding_window.rs:174-300) -- landmark selection, indexing, initial values;
//   * rsvio_window_apply: process_optimization_result (:418-486) -- map points as f32 by ascending
//     id, keyframe T_W_B = inverse(SE3(pose7)).
// Both are shared by the device and the oracle Estimators (rsvio.ba.SlidingWindow), so they carry
// no parity question between the two; against the reference they are restatements of its loops.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "rotation.hpp"

namespace rsvio {
namespace {

struct CapacityError {};

// Matrix4::try_inverse (nalgebra do_inverse4: the cofactor closed form, each entry / det), row-major
// in and out; false when det == 0.  (nalgebra's exact term order is unpinned offline: the crate is
// absent; this is the standard cofactor expansion.)
bool inverse4(const double* a, double* out) {
    auto m = [&](int r, int c) { return a[4 * r + c]; };
    double inv[16];
    inv[0] = m(1, 1) * m(2, 2) * m(3, 3) - m(1, 1) * m(2, 3) * m(3, 2) - m(2, 1) * m(1, 2) * m(3, 3) +
             m(2, 1) * m(1, 3) * m(3, 2) + m(3, 1) * m(1, 2) * m(2, 3) - m(3, 1) * m(1, 3) * m(2, 2);
    inv[4] = -m(1, 0) * m(2, 2) * m(3, 3) + m(1, 0) * m(2, 3) * m(3, 2) + m(2, 0) * m(1, 2) * m(3, 3) -
             m(2, 0) * m(1, 3) * m(3, 2) - m(3, 0) * m(1, 2) * m(2, 3) + m(3, 0) * m(1, 3) * m(2, 2);
    inv[8] = m(1, 0) * m(2, 1) * m(3, 3) - m(1, 0) * m(2, 3) * m(3, 1) - m(2, 0) * m(1, 1) * m(3, 3) +
             m(2, 0) * m(1, 3) * m(3, 1) + m(3, 0) * m(1, 1) * m(2, 3) - m(3, 0) * m(1, 3) * m(2, 1);
    inv[12] = -m(1, 0) * m(2, 1) * m(3, 2) + m(1, 0) * m(2, 2) * m(3, 1) + m(2, 0) * m(1, 1) * m(3, 2) -
              m(2, 0) * m(1, 2) * m(3, 1) - m(3, 0) * m(1, 1) * m(2, 2) + m(3, 0) * m(1, 2) * m(2, 1);
    inv[1] = -m(0, 1) * m(2, 2) * m(3, 3) + m(0, 1) * m(2, 3) * m(3, 2) + m(2, 1) * m(0, 2) * m(3, 3) -
             m(2, 1) * m(0, 3) * m(3, 2) - m(3, 1) * m(0, 2) * m(2, 3) + m(3, 1) * m(0, 3) * m(2, 2);
    inv[5] = m(0, 0) * m(2, 2) * m(3, 3) - m(0, 0) * m(2, 3) * m(3, 2) - m(2, 0) * m(0, 2) * m(3, 3) +
             m(2, 0) * m(0, 3) * m(3, 2) + m(3, 0) * m(0, 2) * m(2, 3) - m(3, 0) * m(0, 3) * m(2, 2);
    inv[9] = -m(0, 0) * m(2, 1) * m(3, 3) + m(0, 0) * m(2, 3) * m(3, 1) + m(2, 0) * m(0, 1) * m(3, 3) -
             m(2, 0) * m(0, 3) * m(3, 1) - m(3, 0) * m(0, 1) * m(2, 3) + m(3, 0) * m(0, 3) * m(2, 1);
    inv[13] = m(0, 0) * m(2, 1) * m(3, 2) - m(0, 0) * m(2, 2) * m(3, 1) - m(2, 0) * m(0, 1) * m(3, 2) +
              m(2, 0) * m(0, 2) * m(3, 1) + m(3, 0) * m(0, 1) * m(2, 2) - m(3, 0) * m(0, 2) * m(2, 1);
    inv[2] = m(0, 1) * m(1, 2) * m(3, 3) - m(0, 1) * m(1, 3) * m(3, 2) - m(1, 1) * m(0, 2) * m(3, 3) +
             m(1, 1) * m(0, 3) * m(3, 2) + m(3, 1) * m(0, 2) * m(1, 3) - m(3, 1) * m(0, 3) * m(1, 2);
    inv[6] = -m(0, 0) * m(1, 2) * m(3, 3) + m(0, 0) * m(1, 3) * m(3, 2) + m(1, 0) * m(0, 2) * m(3, 3) -
             m(1, 0) * m(0, 3) * m(3, 2) - m(3, 0) * m(0, 2) * m(1, 3) + m(3, 0) * m(0, 3) * m(1, 2);
    inv[10] = m(0, 0) * m(1, 1) * m(3, 3) - m(0, 0) * m(1, 3) * m(3, 1) - m(1, 0) * m(0, 1) * m(3, 3) +
              m(1, 0) * m(0, 3) * m(3, 1) + m(3, 0) * m(0, 1) * m(1, 3) - m(3, 0) * m(0, 3) * m(1, 1);
    inv[14] = -m(0, 0) * m(1, 1) * m(3, 2) + m(0, 0) * m(1, 2) * m(3, 1) + m(1, 0) * m(0, 1) * m(3, 2) -
              m(1, 0) * m(0, 2) * m(3, 1) - m(3, 0) * m(0, 1) * m(1, 2) + m(3, 0) * m(0, 2) * m(1, 1);
    inv[3] = -m(0, 1) * m(1, 2) * m(2, 3) + m(0, 1) * m(1, 3) * m(2, 2) + m(1, 1) * m(0, 2) * m(2, 3) -
             m(1, 1) * m(0, 3) * m(2, 2) - m(2, 1) * m(0, 2) * m(1, 3) + m(2, 1) * m(0, 3) * m(1, 2);
    inv[7] = m(0, 0) * m(1, 2) * m(2, 3) - m(0, 0) * m(1, 3) * m(2, 2) - m(1, 0) * m(0, 2) * m(2, 3) +
             m(1, 0) * m(0, 3) * m(2, 2) + m(2, 0) * m(0, 2) * m(1, 3) - m(2, 0) * m(0, 3) * m(1, 2);
    inv[11] = -m(0, 0) * m(1, 1) * m(2, 3) + m(0, 0) * m(1, 3) * m(2, 1) + m(1, 0) * m(0, 1) * m(2, 3) -
              m(1, 0) * m(0, 3) * m(2, 1) - m(2, 0) * m(0, 1) * m(1, 3) + m(2, 0) * m(0, 3) * m(1, 1);
    inv[15] = m(0, 0) * m(1, 1) * m(2, 2) - m(0, 0) * m(1, 2) * m(2, 1) - m(1, 0) * m(0, 1) * m(2, 2) +
              m(1, 0) * m(0, 2) * m(2, 1) + m(2, 0) * m(0, 1) * m(1, 2) - m(2, 0) * m(0, 2) * m(1, 1);
    // inv[] above is the adjugate stored row-major (inv[4 r + c] = cofactor(c, r))
    const double det = m(0, 0) * inv[0] + m(0, 1) * inv[4] + m(0, 2) * inv[8] + m(0, 3) * inv[12];
    if (det == 0.0 || !std::isfinite(det)) return false;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] / det;
    return true;
}

// 3x3 block of a row-major 4x4 times v, plus the translation column (nalgebra gemv: per row
// ((a0 v0 + a1 v1) + a2 v2), then + t)
inline void affine3(const double* T, const double* v, double* out) {
    for (int i = 0; i < 3; ++i)
        out[i] = ((T[4 * i] * v[0] + T[4 * i + 1] * v[1]) + T[4 * i + 2] * v[2]) + T[4 * i + 3];
}

}  // namespace
}  // namespace rsvio

using rsvio::guarded;

extern "C" {

int rsvio_window_problem(int32_t n_kf, const double* T_W_B, const double* T_B_C2, const uint64_t* ids_all,
                         const float* uv_all, const int32_t* n_feat, const uint64_t* map_ids, const float* map_pw,
                         int32_t n_map, double* pose7, uint8_t* kf_fixed, double* T_C_B2, int32_t cap_lm,
                         uint64_t* lm_ids, double* p_init, int32_t* n_lm, int32_t cap_obs, int32_t* obs_lm,
                         int32_t* obs_kf, uint8_t* obs_cam, double* obs_uv, int32_t* n_obs) {
    if (n_kf < 1 || !T_W_B || !T_B_C2 || !n_feat || (n_map && (!map_ids || !map_pw)) || !pose7 ||
        !kf_fixed || !T_C_B2 || !lm_ids || !p_init || !n_lm || !obs_lm || !obs_kf || !obs_cam || !obs_uv || !n_obs)
        return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
      try {
        using namespace rsvio;
        // T_Cl_B, T_Cr_B of the front keyframe (:180-181) and their inverses T_B_C (the ray
        // initialisation inverts T_C_B again, :254-258)
        double T_B_C[2][16];
        for (int c = 0; c < 2; ++c) {
            if (!inverse4(T_B_C2 + 16 * c, T_C_B2 + 16 * c) || !inverse4(T_C_B2 + 16 * c, T_B_C[c]))
                throw std::invalid_argument("rsvio_window_problem: T_B_C is not invertible");
        }
        // the lists back to back: list 2k + c = keyframe k, camera c
        std::vector<const uint64_t*> ids(2 * (size_t)n_kf);
        std::vector<const float*> uv(2 * (size_t)n_kf);
        size_t total = 0;
        for (int i = 0; i < 2 * n_kf; ++i) {
            if (n_feat[i] < 0) throw std::invalid_argument("bad feature list");
            ids[i] = ids_all + total;
            uv[i] = uv_all + 2 * total;
            total += (size_t)n_feat[i];
        }
        if (total && (!ids_all || !uv_all)) throw std::invalid_argument("bad feature list");
        // landmark observation counts per camera (:183-209): bit 0 left, bit 1 right, then the
        // landmark index + 1 << 2.  Feature ids are consecutive detection counters, so a window's
        // ids span a short range: a flat table over [min, max] when it is at most 8x the list
        // size, a hash map otherwise.
        uint64_t lo = ~0ull, hi = 0;
        for (size_t j = 0; j < total; ++j) {
            lo = std::min(lo, ids_all[j]);
            hi = std::max(hi, ids_all[j]);
        }
        const bool flat = total && hi - lo < 8 * total + 64;
        std::vector<int> table(flat ? (size_t)(hi - lo + 1) : 0, 0);
        std::unordered_map<uint64_t, int> hmap;
        if (!flat) hmap.reserve(2 * total + 16);
        auto slot = [&](uint64_t id) -> int& { return flat ? table[(size_t)(id - lo)] : hmap[id]; };
        for (int i = 0; i < 2 * n_kf; ++i) {
            const int bit = 1 << (i & 1);
            for (int j = 0; j < n_feat[i]; ++j) slot(ids[i][j]) |= bit;
        }
        // factors in window order (:212-300): keyframe, left then right, feature order; a
        // landmark's index is its first stereo-kept appearance
        int nl = 0, no = 0;
        for (int k = 0; k < n_kf; ++k) {
            const double* Twb = T_W_B + 16 * k;
            for (int c = 0; c < 2; ++c) {
                const int li = 2 * k + c;
                for (int j = 0; j < n_feat[li]; ++j) {
                    const uint64_t id = ids[li][j];
                    int& e = slot(id);
                    if ((e & 3) != 3) continue;  // not seen in both cameras
                    if (no >= cap_obs) throw CapacityError{};
                    const double u = (double)uv[li][2 * j], v = (double)uv[li][2 * j + 1];
                    int lm = (e >> 2) - 1;
                    if (lm < 0) {  // the landmark's initial value (:231-262)
                        if (nl >= cap_lm) throw CapacityError{};
                        lm = nl++;
                        e |= (lm + 1) << 2;
                        lm_ids[lm] = id;
                        double* p = p_init + 3 * (size_t)lm;
                        const uint64_t* it = n_map ? std::lower_bound(map_ids, map_ids + n_map, id) : nullptr;
                        if (it && it != map_ids + n_map && *it == id) {  // map_points.get (as f64)
                            const size_t m = (size_t)(it - map_ids);
                            for (int a = 0; a < 3; ++a) p[a] = (double)map_pw[3 * m + a];
                        } else {  // depth 2 along the first observation's ray
                            const double pc[3] = {u, v, 2.0};
                            double pb[3];
                            affine3(T_B_C[c], pc, pb);
                            affine3(Twb, pb, p);
                        }
                    }
                    obs_lm[no] = lm;
                    obs_kf[no] = k;
                    obs_cam[no] = (uint8_t)c;
                    obs_uv[2 * (size_t)no] = u;
                    obs_uv[2 * (size_t)no + 1] = v;
                    ++no;
                }
            }
            // KF_k's pose: T_B_W = try_inverse(T_W_B), [t; UnitQuaternion::from_matrix(R)] (:214-226)
            double Tbw[16];
            if (!inverse4(Twb, Tbw)) throw std::invalid_argument("rsvio_window_problem: T_W_B is not invertible");
            double* x = pose7 + 7 * (size_t)k;
            x[0] = Tbw[3]; x[1] = Tbw[7]; x[2] = Tbw[11];
            const double R[9] = {Tbw[0], Tbw[1], Tbw[2], Tbw[4], Tbw[5], Tbw[6], Tbw[8], Tbw[9], Tbw[10]};
            rot::quat_from_matrix(R, x + 3);
            kf_fixed[k] = k == 0 ? 1 : 0;  // KF_0 fixed (:281-285)
        }
        *n_lm = nl;
        *n_obs = no;
        return (int)RSVIO_OK;
      } catch (const rsvio::CapacityError&) {
        rsvio::set_last_error("rsvio_window_problem: landmarks or observations exceed cap_lm / cap_obs");
        return (int)RSVIO_ERR_CAPACITY;
      }
    });
}

int rsvio_window_apply(int32_t n_kf, const double* pose7, int32_t n_lm, const uint64_t* lm_ids, const double* p_W,
                       double* T_W_B, uint64_t* map_ids, float* map_pw) {
    if (n_kf < 0 || n_lm < 0 || (n_kf && (!pose7 || !T_W_B)) || (n_lm && (!lm_ids || !p_W || !map_ids || !map_pw)))
        return RSVIO_ERR_INVALID_ARG;
    return guarded([&] {
        using namespace rsvio;
        // T_W_B = inverse(SE3::from(pose7)) (:427-450): the quaternion normalised, then its rotation
        for (int k = 0; k < n_kf; ++k) {
            const double* x = pose7 + 7 * (size_t)k;
            const double nq = 1.0 / std::sqrt(x[3] * x[3] + x[4] * x[4] + x[5] * x[5] + x[6] * x[6]);
            const double q[4] = {x[3] * nq, x[4] * nq, x[5] * nq, x[6] * nq};
            double R[9];
            rot::rotation_of_quat(q, R);
            const double T[16] = {R[0], R[1], R[2], x[0], R[3], R[4], R[5], x[1],
                                  R[6], R[7], R[8], x[2], 0.0,  0.0,  0.0,  1.0};
            if (!inverse4(T, T_W_B + 16 * (size_t)k)) throw std::invalid_argument("rsvio_window_apply: singular pose");
        }
        // map_points <- optimised landmarks as [f32; 3] (:466-475), kept by ascending id
        std::vector<int> ord((size_t)n_lm);
        std::iota(ord.begin(), ord.end(), 0);
        std::sort(ord.begin(), ord.end(), [&](int a, int b) { return lm_ids[a] < lm_ids[b]; });
        for (int i = 0; i < n_lm; ++i) {
            const int l = ord[i];
            if (i && lm_ids[l] == map_ids[i - 1]) throw std::invalid_argument("rsvio_window_apply: duplicate id");
            map_ids[i] = lm_ids[l];
            for (int a = 0; a < 3; ++a) map_pw[3 * (size_t)i + a] = (float)p_W[3 * (size_t)l + a];
        }
        return (int)RSVIO_OK;
    });
}

}  // extern "C"
