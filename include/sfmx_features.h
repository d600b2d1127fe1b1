/* SPDX-License-Identifier: MIT
 *
 * sfmx — feature extraction: the per-shot
 *     featureDetector->detect(image, keypoints);
 *     descriptorExtractor->compute(image, keypoints, descriptors);
 * of SfM::extractFeatures (sfm/SfM.cpp:577-597) for the reference's SIFT
 * setting cv::SIFT::create(featureLimit, 3, 0.09) (cli/PhotogrammetrieCli.cpp:354),
 * i.e. OpenCV 4.5.1's SIFT::detectAndCompute on an 8-bit grayscale image
 * (CameraShot::loadImage defaults to IMREAD_GRAYSCALE, CameraShot.h:149).
 *
 * The output feeds sfmx_matcher_set_images directly: descriptors are n x 128
 * float rows with integer values 0..255 (OpenCV's saturate_cast<uchar>).
 * Status codes and threading as in sfmx.h.
 */
#ifndef SFMX_FEATURES_H
#define SFMX_FEATURES_H

#include <stdint.h>
#include "sfmx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* cv::KeyPoint, same layout (pt.x, pt.y, size, angle, response, octave, class_id). */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} sfmx_keypoint;

/* cv::SIFT::create(nfeatures, nOctaveLayers, contrastThreshold, edgeThreshold, sigma). */
typedef struct {
    int32_t nfeatures;            /* featureLimit; 0 = keep all                      */
    int32_t n_octave_layers;      /* 3                                               */
    double contrast_threshold;    /* 0.09 in the reference (OpenCV default 0.04)     */
    double edge_threshold;        /* 10                                              */
    double sigma;                 /* 1.6                                             */
} sfmx_sift_params;

/* Fills OpenCV's defaults, with the reference's contrast threshold 0.09 and
 * nfeatures = 0. */
void sfmx_sift_default_params(sfmx_sift_params* p);

/* SIFT detect + compute on one width x height 8-bit grayscale image (rows
 * `pitch` bytes apart).  Writes min(n, capacity) keypoints and descriptor rows
 * (128 floats each) and sets *n_keypoints = n; SFMX_ECAPACITY if n > capacity.
 * inputs_on_device = 1: image, keypoints and descriptors are device pointers
 * on `device` (the descriptors can go straight to the matcher); 0: host. */
int sfmx_sift_detect_compute(const uint8_t* image, int32_t width, int32_t height, int64_t pitch,
                             const sfmx_sift_params* params, int32_t inputs_on_device, int32_t device, void* stream,
                             sfmx_keypoint* keypoints, float* descriptors, int32_t capacity, int32_t* n_keypoints);

/* One 8-bit grayscale image (rows `pitch` bytes apart). */
typedef struct {
    const uint8_t* data;
    int32_t width, height;
    int64_t pitch;
} sfmx_gray_image;

/* SfM::extractFeatures over all shots (sfm/SfM.cpp:577-597, an OpenMP loop
 * over shots in the reference): sfmx_sift_detect_compute on each image, with
 * n_streams host workers (1..16), each on its own non-blocking HIP stream with
 * its own scratch, so that the images' small-octave launches and host steps
 * overlap on the GPU.  Per image i: keypoints[i], descriptors[i] (may be NULL
 * as a whole: detect only), capacities[i], n_keypoints[i], status[i] (may be
 * NULL) as for the single-image call.  Results are identical to calling
 * sfmx_sift_detect_compute image by image.  Returns SFMX_OK or the code of the
 * first failing image (sfmx_last_error names it).  One batch call at a time
 * per process. */
int sfmx_sift_detect_compute_batch(const sfmx_gray_image* images, int32_t n_images, const sfmx_sift_params* params,
                                   int32_t inputs_on_device, int32_t device, int32_t n_streams,
                                   sfmx_keypoint* const* keypoints, float* const* descriptors,
                                   const int32_t* capacities, int32_t* n_keypoints, int32_t* status);

/* Device time (ms) of the last sfmx_sift_detect_compute call on this thread
 * (after a batch call: the mean per image of the workers' device times)
 * (HIP events on its stream around all kernels; includes the host keypoint
 * filter between the detection and descriptor kernels);
 * -1 before any call. */
float sfmx_sift_last_kernel_ms(void);

/* ---- ORB ---------------------------------------------------------------------
 * cv::ORB::create(nfeatures, scaleFactor, nlevels, edgeThreshold, firstLevel, WTA_K,
 * scoreType, patchSize, fastThreshold); the reference passes only nfeatures =
 * featureLimit (cli/PhotogrammetrieCli.cpp:347-348) and keeps OpenCV's defaults. */
typedef struct {
    int32_t nfeatures;            /* featureLimit (OpenCV default 500)               */
    float scale_factor;           /* 1.2                                             */
    int32_t n_levels;             /* 8 (1..16)                                       */
    int32_t edge_threshold;       /* 31 (0..256; reads outside a level: OpenCV's bordered pyramid) */
    int32_t first_level;          /* 0 (only 0)                                      */
    int32_t wta_k;                /* 2 (only 2)                                      */
    int32_t score_type;           /* 0 = HARRIS_SCORE (only)                         */
    int32_t patch_size;           /* 31 (only)                                       */
    int32_t fast_threshold;       /* 20                                              */
} sfmx_orb_params;

/* OpenCV's defaults (nfeatures = 500). */
void sfmx_orb_default_params(sfmx_orb_params* p);

/* ORB detect() then compute() on one width x height 8-bit grayscale image, as
 * SfM::extractFeatures calls them (sfm/SfM.cpp:586-587).  Writes min(n, capacity)
 * keypoints and n x 32 descriptor bytes (cv::Mat CV_8U rows, ready for the Hamming
 * matcher) and sets *n_keypoints = n; SFMX_ECAPACITY if n > capacity.
 * inputs_on_device as for sfmx_sift_detect_compute. */
int sfmx_orb_detect_compute(const uint8_t* image, int32_t width, int32_t height, int64_t pitch,
                            const sfmx_orb_params* params, int32_t inputs_on_device, int32_t device, void* stream,
                            sfmx_keypoint* keypoints, uint8_t* descriptors, int32_t capacity, int32_t* n_keypoints);

/* The batch form over all shots, as sfmx_sift_detect_compute_batch. */
int sfmx_orb_detect_compute_batch(const sfmx_gray_image* images, int32_t n_images, const sfmx_orb_params* params,
                                  int32_t inputs_on_device, int32_t device, int32_t n_streams,
                                  sfmx_keypoint* const* keypoints, uint8_t* const* descriptors,
                                  const int32_t* capacities, int32_t* n_keypoints, int32_t* status);

/* Device time of the last call (batch: mean per image), HIP events on its stream. */
float sfmx_orb_last_kernel_ms(void);

#ifdef __cplusplus
}
#endif

#endif /* SFMX_FEATURES_H */
