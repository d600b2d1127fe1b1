/* SPDX-License-Identifier: MIT
 *
 * sfmx — the openMVS seam: OpenMvsUtils::toOpenMVS
 * (util/OpenMvsUtils.cpp:31-154), which hands the sparse reconstruction to the
 * openMVS densify stage (reader: mvs/MVS.cpp:26-31, openMVS Scene::Load).
 *
 *   sfmx_undistort_images    the per-shot cv::undistort of :142-150
 *                            (ICamera::undistort, common/ICamera.cpp:72-80)
 *   sfmx_openmvs_serialize   the Interface assembly of :44-133 and
 *   sfmx_openmvs_write       openMVS::ARCHIVE::SerializeSave of :152
 *
 * Image encoding (cv::imwrite of the undistorted PNGs) stays with the caller.
 * Status codes and threading as in sfmx.h.
 */
#ifndef SFMX_MVS_H
#define SFMX_MVS_H

#include <stdint.h>
#include "sfmx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- undistort */

/* One 8-bit image, interleaved channels (cv::Mat CV_8UC<channels>). */
typedef struct {
    const uint8_t* src;       /* height rows of src_pitch bytes                              */
    uint8_t* dst;             /* same size/type; must not alias src (cv::undistort asserts it) */
    int32_t width, height;    /* 0 < width, height < 32767 (cv::remap's short maps)          */
    int32_t channels;         /* 1..4                                                          */
    int32_t _pad;
    int64_t src_pitch, dst_pitch;   /* bytes per row, >= width * channels                     */
    double K[9];              /* ICamera::getK, row-major 3x3, K[1] = K[3] = K[6] = K[7] = 0, K[8] = 1 */
    double dist[5];           /* k1 k2 p1 p2 k3 (ICamera::getDistortion is 1x4: pass k3 = 0) */
} sfmx_undistort_image;

/* cv::undistort(in, out, K, distortion) (OpenCV 4.5.1, as called from
 * ICamera::undistort, ICamera.cpp:72-80) for every image: the inverse map of
 * initUndistortRectifyMap in fixed-point CV_16SC2 + CV_16UC1 form (1/32 px),
 * then cv::remap INTER_LINEAR with BORDER_CONSTANT 0, in the same horizontal
 * stripes cv::undistort uses.  All images go in one launch.
 * inputs_on_device = 1: src/dst are device pointers on `device`; 0: host
 * memory (copied in and out). */
int sfmx_undistort_images(const sfmx_undistort_image* images, int32_t n_images, int32_t inputs_on_device,
                          int32_t device, void* stream);

/* Device time (ms) of the last sfmx_undistort_images call on this thread
 * (the remap kernel, HIP events on its stream); -1 before any call. */
float sfmx_undistort_last_kernel_ms(void);

/* ---------------------------------------------------------------- interface */

/* openMVS Interface::Platform::Camera inputs: ICamera::getResolution, getK. */
typedef struct {
    int32_t width, height;
    double K[9];
} sfmx_mvs_camera;

/* One CameraShot of Scene::getShots(). */
typedef struct {
    int32_t camera;           /* index into the camera list (-1: no camera; skipped like :77) */
    int32_t recovered;        /* CameraShot::isRecovered                                     */
    double pose[12];          /* CameraShot::getPose, 3x4 [R | t] row-major                  */
    const char* image_name;   /* Interface::Image::name (the reference: images/<id>.png,
                                 absolute or relative to the interface file, :81-82)          */
} sfmx_mvs_shot;

/* The openMVS Interface built as OpenMvsUtils::toOpenMVS does (:44-133) and
 * serialized as openMVS ARCHIVE::SerializeSave (openMVS v1.1.1, header
 * "MVSI", stream version, reserved 0; vectors and strings as uint64 count +
 * elements; Mat33d / Point3 as raw doubles/floats):
 *   - one platform per camera, holding one camera (K, R = I, C = 0) (:44-70);
 *   - one image + pose per shot that is recovered and has a camera, in shot
 *     order; pose R = [R], C = -R^T t (CameraShot::getCenter) (:72-101);
 *   - one vertex per point with >= 2 distinct origin shots that became
 *     images, X = (float) coordinates, views sorted by image id, confidence 0
 *     (:104-133; PointcloudElement::getOriginShots, Scene.cpp:152-160).
 * Origins: origin_offsets[n_points + 1] CSR over origin_shot (shot indices;
 * duplicates are allowed and collapse, like the reference's std::set).
 * version: the stream version to write, 1..3 (the fields each version adds
 * follow openMVS Interface.h's serialize()).  openMVS loads any version up to
 * its own MVSI_PROJECT_VER; 1 carries everything toOpenMVS sets.
 * Writes at most `capacity` bytes to `out` (may be NULL with capacity 0) and
 * sets *size to the full serialized size; SFMX_ECAPACITY if it did not fit.
 * n_images / n_vertices (may be NULL) receive the counts written. */
int sfmx_openmvs_serialize(uint32_t version, const sfmx_mvs_camera* cameras, int32_t n_cameras,
                           const sfmx_mvs_shot* shots, int32_t n_shots, const double* points, int32_t n_points,
                           const int64_t* origin_offsets, const int32_t* origin_shot, uint8_t* out,
                           int64_t capacity, int64_t* size, int32_t* n_images, int32_t* n_vertices);

/* sfmx_openmvs_serialize straight to the file `path` (OpenMvsUtils.cpp:152). */
int sfmx_openmvs_write(const char* path, uint32_t version, const sfmx_mvs_camera* cameras, int32_t n_cameras,
                       const sfmx_mvs_shot* shots, int32_t n_shots, const double* points, int32_t n_points,
                       const int64_t* origin_offsets, const int32_t* origin_shot, int32_t* n_images,
                       int32_t* n_vertices);

#ifdef __cplusplus
}
#endif

#endif /* SFMX_MVS_H */
