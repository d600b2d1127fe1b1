// SPDX-License-Identifier: MIT
//
// sfmx ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's scene bookkeeping,
// as literal loops (the reference's own complexity), for parity tests:
//   orc_find_3d2d_matches      Scene::find3d2dMatches   src/photogrammetrie/common/Scene.cpp:369-424
//     for every point origin (shot o, point q) with o != shot: the first pair
//     in list order joining {shot, o} (:389-394), then the first DMatch whose
//     keypoint on o's side satisfies cv::Point2d(kp.pt) == q (:396-405), and
//     the keypoint on shot's side (:407-411).
//   orc_ba_observations        BundleAdjustment.cpp:50-91: residual blocks in
//     point order then origin order, a camera-pose block per shot on its first
//     appearance (linear find_if over the created blocks, :64-79), the
//     observation as cv::Point2f (ICamera.h:161).
// Inputs are the flattened origin records of PointcloudElement::getOriginPoints
// (Scene.cpp:162-185); see include/sfmx_scene.h.
#include <cmath>
#include <cstdint>
#include <vector>
#include <omp.h>

namespace {
struct DM { int32_t q, t, img; float dist; };
}

extern "C" {

int orc_find_3d2d_matches(const float* const* kp, const int32_t* pairs, int npairs, const void* matches_v,
                          const int64_t* off, const int64_t* oo, int npoints, const int32_t* oshot,
                          const double* oxy, int shot, int32_t* out_kp, int32_t* out_pair, int nthreads) {
    const DM* m = (const DM*)matches_v;
    const int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
    #pragma omp parallel for schedule(dynamic, 64) num_threads(nt)   // Scene.cpp:375, omp over the point cloud
    for (int p = 0; p < npoints; ++p)
        for (int64_t r = oo[p]; r < oo[p + 1]; ++r) {
            out_kp[r] = -1;
            out_pair[r] = -1;
            const int o = oshot[r];
            if (o == shot) continue;                                           // :385-387
            int sm = -1;
            for (int q = 0; q < npairs && sm < 0; ++q)                         // :389-394 find_if
                if ((pairs[2 * q] == shot && pairs[2 * q + 1] == o) || (pairs[2 * q + 1] == shot && pairs[2 * q] == o))
                    sm = q;
            if (sm < 0) continue;
            const bool o_left = pairs[2 * sm] == o;
            for (int64_t i = off[sm]; i < off[sm + 1]; ++i) {                  // :396-405 find_if
                const int ki = o_left ? m[i].q : m[i].t;
                const float* k = kp[o] + 2 * ki;
                if ((double)k[0] == oxy[2 * r] && (double)k[1] == oxy[2 * r + 1]) {
                    out_kp[r] = pairs[2 * sm] == shot ? m[i].q : m[i].t;       // :407-409
                    out_pair[r] = sm;
                    break;
                }
            }
        }
    return 0;
}

int orc_ba_observations(const int64_t* oo, int npoints, const int32_t* oshot, const double* oxy, int nshots,
                        int32_t* obs_point, int32_t* obs_cam, double* obs_xy, int32_t* shot_of_pose) {
    int np = 0;
    for (int p = 0; p < npoints; ++p)
        for (int64_t r = oo[p]; r < oo[p + 1]; ++r) {
            int pose = -1;
            for (int c = 0; c < np; ++c)                                        // find_if over ceresShots
                if (shot_of_pose[c] == oshot[r]) { pose = c; break; }
            if (pose < 0) { pose = np; shot_of_pose[np++] = oshot[r]; }
            obs_point[r] = p;
            obs_cam[r] = pose;
            obs_xy[2 * r] = (double)(float)oxy[2 * r];
            obs_xy[2 * r + 1] = (double)(float)oxy[2 * r + 1];
        }
    (void)nshots;
    return np;
}

}  // extern "C"
