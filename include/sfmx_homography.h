/* SPDX-License-Identifier: MIT
 *
 * sfmx — per-pair homography RANSAC over the match graph.
 *
 * Replaces SfM::calculateHomography(Scene&)      src/photogrammetrie/sfm/SfM.cpp:599-637
 *   for every ShotMatches of the scene (OpenMP over pairs, :603):
 *     < 4 matches            -> skipped, homographyInlierRatio stays -1   (:606-609, Scene.h:56)
 *     aligned keypoints      left[queryIdx], right[trainIdx]              (:612-613, Scene.cpp:58-71)
 *     threshold              t < 0 ? -t : max(wL, hL, hR, hR) * t         (:615-619; the reference
 *                            reads rightSize.height twice, kept)
 *     cv::findHomography(left, right, cv::RANSAC, threshold, mask)         (:621-624)
 *     ratio                  countNonZero(mask) / matches.size(); 0 if H is empty (:625-628)
 *   -> ShotMatches::setHomographyInlierRatio (Scene.h:102-108), consumed by the
 *      initial-pair choice in SfM::triangulate (SfM.cpp:176-188).
 * The RANSAC is OpenCV 4.5.1's (deterministic cv::RNG((uint64)-1) subset
 * sequence, maxIters 2000, confidence 0.995); see oracle/homography_oracle.cpp
 * for the restated algorithm and DESIGN.md for the deviations.
 *
 * Status codes and threading as in sfmx.h.
 */
#ifndef SFMX_HOMOGRAPHY_H
#define SFMX_HOMOGRAPHY_H

#include <stdint.h>
#include "sfmx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* == cv::Point2f (cv::KeyPoint::pt). */
typedef struct sfmx_point2f {
    float x, y;
} sfmx_point2f;

/* Defaults of cv::findHomography and of the reference's -Pransac flag
 * (SfM.h:50: ransacReprojectionMatchingThreshold = -3.0 -> 3 px). */
#define SFMX_RANSAC_MAX_ITERS 2000
#define SFMX_RANSAC_CONFIDENCE 0.995
#define SFMX_RANSAC_MATCHING_THRESHOLD (-3.0)

/* Inlier ratio of every pair of a match graph.
 *   keypoints     n_imgs pointers; image i has n_keypoints[i] points
 *   image_size    2 * n_imgs ints: width, height (CameraShot::getImageSize)
 *   pairs         2 * n_pairs (left, right)
 *   matches       packed DMatch lists, pair p at [pair_offsets[p], pair_offsets[p+1])
 *                 (the layout sfmx_matcher_fetch returns)
 *   threshold     the reference's ransacReprojectionMatchingThreshold
 *   out_ratio     n_pairs doubles; -1 for pairs with fewer than 4 matches
 * inputs_on_device = 0: every pointer above is host memory (copied in);
 * 1: keypoints[i], matches and pair_offsets are device pointers already
 * resident on `device` (e.g. sfmx_matcher_device_results), the small arrays
 * (n_keypoints, image_size, pairs) stay host.  out_ratio is always host memory.
 * A queryIdx / trainIdx outside its image's keypoints returns SFMX_EINVAL
 * (host inputs) or yields ratio NaN for that pair (device inputs, checked in
 * the kernel).  Device inputs are not read back: a pair list of more than 2048
 * matches must lie inside [0, sum over pairs of n_keypoints[left]) of the
 * offsets (at most one match per query keypoint, as the matcher writes them),
 * else its ratio is NaN.
 * Replaces: SfM::calculateHomography, SfM.cpp:599-637. */
int sfmx_homography_ratios(const sfmx_point2f* const* keypoints, const int32_t* n_keypoints, int32_t n_imgs,
                           const int32_t* image_size, const int32_t* pairs, int32_t n_pairs,
                           const sfmx_dmatch* matches, const int64_t* pair_offsets, double threshold,
                           int32_t max_iters, double confidence, int32_t inputs_on_device, int32_t device,
                           void* stream, double* out_ratio);

/* Device time (ms) of the RANSAC kernel of the last sfmx_homography_ratios
 * call on this thread (HIP events on its stream); -1 before any call. */
float sfmx_homography_last_kernel_ms(void);

#ifdef __cplusplus
}
#endif

#endif /* SFMX_HOMOGRAPHY_H */
