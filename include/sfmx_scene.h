/* SPDX-License-Identifier: MIT
 *
 * sfmx — scene bookkeeping around bundle adjustment:
 * the 3D-2D correspondence search for a new shot and the construction of the
 * Ceres problem's observation arrays from the point cloud.
 *
 * Point-cloud origins are passed flattened, one record per distinct (shot,
 * 2-D point) of PointcloudElement::getOriginPoints (common/Scene.cpp:162-185,
 * first-appearance order, left point before right point of every origin),
 * as a CSR over points:
 *     origin_offsets[n_points + 1], origin_shot[n_origins], origin_xy[2 * n_origins] (double, cv::Point2d)
 * Shot matches are the packed lists of sfmx.h (pairs[2 * n_pairs] = (left,
 * right) shot indices in Scene::getShotMatches() order, matches, pair_offsets).
 *
 * Status codes and threading as in sfmx.h.
 */
#ifndef SFMX_SCENE_H
#define SFMX_SCENE_H

#include <stdint.h>
#include "sfmx.h"
#include "sfmx_homography.h"   /* sfmx_point2f */

#ifdef __cplusplus
extern "C" {
#endif

/* Scene::find3d2dMatches(ShotMatches3d2d&) (common/Scene.cpp:369-424) for the
 * new shot `shot`: for every origin record (point p, origin shot o, 2-D point q)
 * with o != shot, the FIRST shot-match pair in list order joining {shot, o}
 * (:389-394), then the FIRST DMatch in that pair's list whose keypoint on o's
 * side has cv::Point2d(kp.pt) == q (:396-405); the 3D-2D match is the keypoint
 * on `shot`'s side (:407-411).
 *   out_keypoint[i]  keypoint index in `shot` matched through origin record i, -1 if none
 *   out_pair[i]      index of the shot-match pair used, -1 if none
 *   out_xy[2i]       that keypoint's position (cv::KeyPoint::pt), NaN if none (may be NULL)
 * The reference appends matches under `omp critical` in a nondeterministic
 * order; here they are reported per origin record (point-major), which keys
 * parity by (point, origin).
 * inputs_on_device = 1: keypoints[i], matches, pair_offsets, origin_* and the
 * out_* arrays are device pointers on `device`; 0: host memory. */
int sfmx_find_3d2d_matches(const sfmx_point2f* const* keypoints, const int32_t* n_keypoints, int32_t n_shots,
                           const int32_t* pairs, int32_t n_pairs, const sfmx_dmatch* matches,
                           const int64_t* pair_offsets, const int64_t* origin_offsets, int32_t n_points,
                           const int32_t* origin_shot, const double* origin_xy, int32_t shot,
                           int32_t inputs_on_device, int32_t device, void* stream, int32_t* out_keypoint,
                           int32_t* out_pair, float* out_xy);

/* Device time (ms) of the last sfmx_find_3d2d_matches call on this thread
 * (table build + lookup kernels, HIP events on its stream); -1 before any call. */
float sfmx_find_3d2d_last_kernel_ms(void);

/* BundleAdjustment::doBundleAdjustment(const Scene&, ...)'s problem assembly
 * (common/BundleAdjustment.cpp:50-91) as flat sfmx_ba_problem arrays: one
 * observation per origin record, in point order then origin order (the
 * AddResidualBlock order); the camera-pose block of a shot is created on its
 * first appearance (the OpenMpUtils::find_if over ceresShots, :64-79, made
 * O(1) by a shot -> pose table).  The observation is the cv::Point2f the
 * cost function receives (ICamera::ceresCostFunction(const cv::Point2f&),
 * ICamera.h:161), stored as double.
 *   obs_point[n_origins], obs_cam[n_origins], obs_xy[2 * n_origins]
 *   pose_of_shot[n_shots]  pose index of each shot (-1: not observed)
 *   shot_of_pose[n_shots]  inverse (first *n_poses entries valid)
 * Host memory only (O(n_origins) host work). */
int sfmx_ba_observations_from_origins(const int64_t* origin_offsets, int32_t n_points, const int32_t* origin_shot,
                                      const double* origin_xy, int32_t n_shots, int32_t* obs_point, int32_t* obs_cam,
                                      double* obs_xy, int32_t* pose_of_shot, int32_t* shot_of_pose, int32_t* n_poses);

#ifdef __cplusplus
}
#endif

#endif /* SFMX_SCENE_H */
