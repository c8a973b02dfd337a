// lk_track.hpp -- K2 launch descriptor (see lk_track.hip).
#pragma once
#include "common.hpp"

namespace rsvio {

constexpr int kMaxTrackBatches = 4;

// Up to 4 independent track_points batches (e.g. cam0 and cam1 temporal tracking) per launch;
// one 64-lane workgroup per feature.
struct TrackLaunch {
    uint32_t w, h;
    int levels;
    int max_iter;
    float thresh;
    int nb;
    int start[kMaxTrackBatches + 1];           // prefix of batch sizes (launch capacity)
    const uint8_t* pyr0[kMaxTrackBatches];
    const uint8_t* pyr1[kMaxTrackBatches];
    const float* ain[kMaxTrackBatches];        // n x 6 {m11, m12, m21, m22, m13, m23}
    float* aout[kMaxTrackBatches];
    uint8_t* valid[kMaxTrackBatches];
    const int* dcount[kMaxTrackBatches];       // optional device-side count (early exit)
    const int4* mask[kMaxTrackBatches];        // optional: job i runs only when mask[i].w != 0 (else valid = 0)
    // batched serving mode (rsvio_track_points_table_d): when set, batch descriptors and the
    // prefix of their sizes come from device memory and nb may exceed kMaxTrackBatches
    const rsvio_track_batch* table;
    const int32_t* tstart;
    int njobs;  // set by enqueue_track: jobs in this launch
};

void enqueue_track(const TrackLaunch& L, hipStream_t s);

}  // namespace rsvio
