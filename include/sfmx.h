/* SPDX-License-Identifier: MIT
 *
 * sfmx — MI355X-native SfM matching + bundle-adjustment hot path.
 * C ABI (the drop-in boundary).  Plain pointers and sizes only; no exceptions
 * cross it; every entry point returns SFMX_OK (0) or a negative SFMX_E* code.
 *
 * Reference interfaces replaced (paths relative to brunothg/sfm-mvs-pipeline):
 *   - IFeatureMatchingStrategy::calculateShotMatches(const Scene&, cv::Ptr<DescriptorMatcher>&,
 *         vector<ShotMatches>&)                         src/photogrammetrie/sfm/IFeatureMatchingStrategy.h:45-46
 *     with the BF matcher it is handed                  src/cli/PhotogrammetrieCli.cpp:359-392
 *   - the pair enumeration of the three strategies      sfm/UnorderedFeatureMatchingStrategy.cpp:32-37,
 *                                                       sfm/VideoFeatureMatchingStrategy.cpp:43-48,
 *                                                       sfm/GridFeatureMatchingStrategy.cpp:48-85
 *   - SfM::calculateShotMatches' filters                sfm/SfM.cpp:547-570
 *   - BundleAdjustment::doBundleAdjustment(Scene&) →
 *         CeresUtils::solve(problem, summary)           common/BundleAdjustment.h:85-97, util/CeresUtils.h:69
 *
 * Threading: thread-compatible (one call per context at a time).  Device
 * work runs on the HIP stream passed in (`stream` = hipStream_t as void*,
 * NULL = the legacy default stream).
 */
#ifndef SFMX_H
#define SFMX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
enum {
    SFMX_OK = 0,
    SFMX_EINVAL = -1,        /* bad argument (reference: std::invalid_argument)          */
    SFMX_ENOMEM = -2,        /* device or host allocation failed                          */
    SFMX_EDEVICE = -3,       /* HIP runtime error / no usable gfx950 device               */
    SFMX_ECAPACITY = -4,     /* caller's output buffer too small; required size returned  */
    SFMX_ESTATE = -5,        /* call out of order (e.g. run before set_images)            */
    SFMX_EINTERNAL = -6      /* a device-side self check failed (a bug: please report)     */
};

/* Norm types: numerically equal to cv::NORM_L2 / cv::NORM_HAMMING so a caller
 * can forward cv::BFMatcher::create(normType) unchanged. */
enum { SFMX_NORM_L2 = 4, SFMX_NORM_HAMMING = 6 };

/* Descriptor element types: equal to cv::Mat depth codes CV_8U / CV_32F. */
enum { SFMX_8U = 0, SFMX_32F = 5 };

/* == cv::DMatch {int queryIdx; int trainIdx; int imgIdx; float distance;}, 16 B.
 * queryIdx = left-image feature, trainIdx = right-image feature (Scene.h:47-51). */
typedef struct sfmx_dmatch {
    int32_t queryIdx;
    int32_t trainIdx;
    int32_t imgIdx;
    float distance;
} sfmx_dmatch;

/* One image's descriptor matrix, row-major and contiguous (cv::Mat
 * CameraShot::Features::descriptors, CameraShot.h:39-42).
 * SIFT: type SFMX_32F, cols = 128 (<= 128 accepted); ORB: SFMX_8U, cols = 32 (<= 32). */
typedef struct sfmx_desc {
    const void* data;
    int32_t rows;
    int32_t cols;
    int32_t type;
    int32_t _pad;
} sfmx_desc;

/* ---- a1: pair enumeration ----------------------------------------------
 * Write (left,right) int32 pairs in the reference's loop order into `out`
 * (2*cap int32) and return the pair count (>= 0), or SFMX_EINVAL.  With
 * out == NULL only the count is returned.  If the count exceeds cap, nothing
 * beyond cap is written and the full count is still returned.            */
int64_t sfmx_pairs_unordered(int32_t n_images, int32_t* out, int64_t cap);
int64_t sfmx_pairs_video(int32_t n_images, int32_t sequence_length, int32_t* out, int64_t cap);
/* grid_mode 0 = reference-observable (rowCount = n / rowLength, :48),
 *           1 = intended (rowCount = ceil, empty cells skipped); equal when n % rowLength == 0. */
int64_t sfmx_pairs_grid(int32_t n_images, int32_t sequence_length, int32_t row_length,
                        int32_t grid_mode, int32_t* out, int64_t cap);

/* ---- a2-a5: matching -----------------------------------------------------
 * A matcher context owns one device, the prepared descriptor pool in HBM and
 * the result buffers.  Typical use (what calculateShotMatches becomes):
 *   sfmx_matcher_create(dev, &m);
 *   sfmx_matcher_set_images(m, imgs, n, norm, stream);     // H2D + prepare
 *   sfmx_matcher_run(m, pairs, n_pairs, ratio, distinct, min_count, stream);
 *   sfmx_matcher_fetch(m, out, cap, pair_offsets, keep, stream);       // D2H
 */
typedef struct sfmx_matcher sfmx_matcher;

int sfmx_matcher_create(int32_t device, sfmx_matcher** out);
int sfmx_matcher_destroy(sfmx_matcher* m);

/* Upload + prepare all images (host descriptor buffers).  norm must match the
 * element type (L2 <-> 32F, HAMMING <-> 8U).  Replaces any previous set. */
int sfmx_matcher_set_images(sfmx_matcher* m, const sfmx_desc* imgs, int32_t n_imgs,
                            int32_t norm, void* stream);

/* Same, from descriptor matrices already resident in device memory on this
 * matcher's device (imgs[i].data are device pointers).  The host does not wait
 * for the SIFT integrality check here: the next run assumes integral rows and
 * the check is resolved when its results are first read (fetch, stats,
 * device_results), re-running on the fp32 path if an image is not integral.
 * The device buffers must therefore stay valid and unchanged until the
 * results of the following run have been read. */
int sfmx_matcher_set_images_device(sfmx_matcher* m, const sfmx_desc* imgs, int32_t n_imgs,
                                   int32_t norm, void* stream);

/* Match a pair list (host int32[2*n_pairs], (left,right) image indices).
 * Per pair: knnMatch(left, right, k=2) with exact BF semantics + Lowe ratio
 * test (ratio = 0.7 in the reference, UnorderedFeatureMatchingStrategy.cpp:55),
 * then the SfM filters: distinct != 0 drops non-unique trainIdx (SfM.cpp:547-564),
 * pairs with < min_count matches are marked dropped (SfM.cpp:566-570; pass
 * min_count = 0 to keep all).  Asynchronous on `stream`. */
int sfmx_matcher_run(sfmx_matcher* m, const int32_t* pairs, int32_t n_pairs, double ratio,
                     int32_t distinct, int32_t min_count, void* stream);

/* Synchronise `stream` and copy results to the host.  out receives the
 * matches of all pairs back to back in pair order (each pair's list in query
 * order); pair_offsets[n_pairs+1] delimit them; keep[n_pairs] = 1 if the pair
 * passed min_count (dropped pairs keep their matches in `out` so a caller can
 * still inspect them).  Returns SFMX_ECAPACITY and sets *required if cap is
 * too small.  Any of out / pair_offsets / keep may be NULL to skip it. */
int sfmx_matcher_fetch(sfmx_matcher* m, sfmx_dmatch* out, int64_t cap, int64_t* required,
                       int64_t* pair_offsets, int32_t* keep, void* stream);

/* Device-side views of the last run's results (valid until the next run):
 * packed DMatch array, int64 pair offsets [n_pairs+1], int32 keep flags. */
int sfmx_matcher_device_results(sfmx_matcher* m, const sfmx_dmatch** matches,
                                const int64_t** pair_offsets, const int32_t** keep);

/* Diagnostics of the last run: number of queries routed to the exact
 * float-sqrt slow path, and number of pairs matched by the fp32 fallback
 * (non-integer SIFT descriptors).  Synchronises `stream`. */
int sfmx_matcher_stats(sfmx_matcher* m, int64_t* slow_queries, int64_t* fp32_pairs, void* stream);

/* Device time of the last run, from HIP events recorded on the run's stream:
 * main_kernel_ms = the 2-NN kernel (sift_knn2 / orb_knn2) launch alone,
 * total_ms = first to last kernel of the run.  Synchronises the run's end event. */
int sfmx_matcher_timing(sfmx_matcher* m, float* main_kernel_ms, float* total_ms);

/* The two-pass split of main_kernel_ms (SIFT-L2 and ORB-FP4 paths): screen_ms = pass 1 (the
 * screening kernel), pass2_ms = the rest of the 2-NN launch (work compaction + the exact kernel on
 * the forwarded queries).  Single-pass variants report screen_ms = 0. */
int sfmx_matcher_pass_timing(sfmx_matcher* m, float* screen_ms, float* pass2_ms);

/* The main-kernel and pass-1 times (ms, HIP events on the run's stream) of the last min(n, runs, 32)
 * runs, oldest first, so a loop of runs can be timed per run without a host sync inside it.
 * Synchronises on the last run.  Returns the count written (>= 0) or a negative code. */
int sfmx_matcher_timing_history(sfmx_matcher* m, float* main_kernel_ms, float* screen_ms, int32_t n);

/* One-shot convenience wrapper = the whole strategy call
 * (IFeatureMatchingStrategy::calculateShotMatches, IFeatureMatchingStrategy.h:45-46, as SfM.cpp:545
 * calls it): uses n_gpus devices (pairs split by Σ Nq·Nt, one host thread per device; each device
 * uploads only the images its slice references) and host buffers.  Each query yields at most one
 * match, so cap = Σ over pairs of rows(left) always suffices and ONE call does the whole job; with a
 * smaller cap the call still matches once, sets *required and returns SFMX_ECAPACITY. */
int sfmx_match_pairs(const sfmx_desc* imgs, int32_t n_imgs, const int32_t* pairs, int32_t n_pairs,
                     int32_t norm, double ratio, int32_t distinct, int32_t min_count, int32_t n_gpus,
                     sfmx_dmatch* out, int64_t cap, int64_t* required,
                     int64_t* pair_offsets, int32_t* keep);

/* Library/device probe: returns the number of visible gfx950 devices (>= 0)
 * or SFMX_EDEVICE. */
int sfmx_device_count(void);
const char* sfmx_version(void);
/* Human-readable description of the calling thread's last failure. */
const char* sfmx_last_error(void);

/* Self-test: out_bits[s] = float bits of the device's correctly rounded
 * sqrt of the integer s for s in [0, n) (the distance the L2 kernels report).
 * Used by the tests to compare against the host's sqrtf exhaustively. */
int sfmx_selftest_sqrt(int32_t device, int64_t n, uint32_t* out_bits);

#ifdef __cplusplus
}
#endif
#endif /* SFMX_H */
