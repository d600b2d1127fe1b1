// SPDX-License-Identifier: MIT
// sfmx openMVS interface export, host side.
//
//   sfmx_openmvs_serialize / sfmx_openmvs_write
//       OpenMvsUtils::toOpenMVS (util/OpenMvsUtils.cpp:31-154): the Interface
//       assembly (:44-133) and openMVS::ARCHIVE::SerializeSave (:152).
//
// The serialized stream is openMVS's own archive format (openMVS v1.1.1,
// libs/MVS/Interface.h, an external dependency not present here):
//   "MVSI" | uint32 version | uint32 reserved (0) | Interface
// with std::vector / std::string as a uint64 element count followed by the
// elements, cv::Matx as its raw values (row-major), cv::Point3_ as x, y, z and
// every struct as its members in serialize() order; the fields a stream
// version adds are gated exactly as serialize() gates them (see put_* below).
// Everything is written little-endian, as on the reference's x86 hosts.
// O(shots + origins) host work; no GPU involved.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sfmx_mvs.h"
#include "match_common.hpp"

namespace sfmx {
namespace mvs {

struct Sink {               // counts every byte; copies while the buffer lasts
    uint8_t* out;
    int64_t cap, n = 0;
    void put(const void* p, size_t k) {
        if (out && n < cap) std::memcpy(out + n, p, (size_t)std::min<int64_t>((int64_t)k, cap - n));
        n += (int64_t)k;
    }
    template <class T> void pod(const T& v) { put(&v, sizeof(T)); }
    void count(uint64_t c) { pod(c); }
    void str(const char* s) {
        const uint64_t k = s ? std::strlen(s) : 0;
        count(k);
        if (k) put(s, k);
    }
};

struct Plan {
    std::vector<int32_t> image_of_shot;   // shotToId (-1: not an image)
    std::vector<int32_t> image_shot;      // shot of each image, in image order
    std::vector<int64_t> vtx_point;       // point of each vertex
    std::vector<int64_t> vtx_off{0};      // CSR into vtx_view
    std::vector<uint32_t> vtx_view;       // sorted image ids
};

// OpenMvsUtils.cpp:72-133 (which shots become images, which points vertices).  A point's image ids
// are kept sorted and unique as they arrive (insertion into a short run; the reference's std::set),
// straight into the CSR, which is rolled back when fewer than two remain.
static int plan(const sfmx_mvs_shot* shots, int32_t n_shots, int32_t n_cameras, int32_t n_points,
                const int64_t* oo, const int32_t* osh, Plan& pl) {
    pl.image_of_shot.assign(n_shots, -1);
    for (int s = 0; s < n_shots; ++s) {
        if (!shots[s].recovered || shots[s].camera < 0 || shots[s].camera >= n_cameras) continue;   // :76-78
        pl.image_of_shot[s] = (int32_t)pl.image_shot.size();
        pl.image_shot.push_back(s);
    }
    if (n_points > 0) {
        pl.vtx_point.reserve(n_points);
        pl.vtx_off.reserve((size_t)n_points + 1);
        pl.vtx_view.reserve((size_t)std::max<int64_t>(oo[n_points] - oo[0], 0));
    }
    for (int p = 0; p < n_points; ++p) {
        if (oo[p + 1] < oo[p]) { set_last_error("origin offsets not ascending"); return SFMX_EINVAL; }
        const size_t b = pl.vtx_view.size();
        for (int64_t k = oo[p]; k < oo[p + 1]; ++k) {
            const int s = osh[k];
            if (s < 0 || s >= n_shots) { set_last_error("origin shot out of range"); return SFMX_EINVAL; }
            const int32_t id = pl.image_of_shot[s];
            if (id < 0) continue;                                                       // :109-112
            size_t e = pl.vtx_view.size(), i = e;                                       // :127-128
            while (i > b && pl.vtx_view[i - 1] > (uint32_t)id) --i;
            if (i > b && pl.vtx_view[i - 1] == (uint32_t)id) continue;                  // getOriginShots: std::set
            pl.vtx_view.push_back(0);
            for (; e > i; --e) pl.vtx_view[e] = pl.vtx_view[e - 1];
            pl.vtx_view[i] = (uint32_t)id;
        }
        if (pl.vtx_view.size() - b < 2) { pl.vtx_view.resize(b); continue; }            // :122-124
        pl.vtx_point.push_back(p);
        pl.vtx_off.push_back((int64_t)pl.vtx_view.size());
    }
    return SFMX_OK;
}

static const double I33[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};

static void emit(Sink& o, uint32_t version, const sfmx_mvs_camera* cameras, int32_t n_cameras,
                 const sfmx_mvs_shot* shots, const double* points, const Plan& pl) {
    o.put("MVSI", 4);
    o.pod(version);
    o.pod((uint32_t)0);
    // platforms: Platform{name, cameras, poses}
    std::vector<std::vector<int32_t>> poses(n_cameras);   // image order per platform (poseID)
    for (int32_t s : pl.image_shot) poses[shots[s].camera].push_back(s);
    o.count((uint64_t)n_cameras);
    for (int c = 0; c < n_cameras; ++c) {
        o.str("");                                   // Platform::name
        o.count(1);                                  // one Camera per platform (:55-56)
        o.str("");                                   // Camera::name
        if (version > 0) {
            o.pod((uint32_t)cameras[c].width);
            o.pod((uint32_t)cameras[c].height);
        }
        o.put(cameras[c].K, sizeof(double) * 9);     // K
        o.put(I33, sizeof(double) * 9);              // R = eye (:51)
        const double C0[3] = {0, 0, 0};
        o.put(C0, sizeof(C0));                       // C = 0 (:52)
        o.count(poses[c].size());
        for (int32_t s : poses[c]) {                 // Pose{R, C}; C = -R^T t (CameraShot::getCenter)
            const double* P = shots[s].pose;
            const double R[9] = {P[0], P[1], P[2], P[4], P[5], P[6], P[8], P[9], P[10]};
            const double t[3] = {P[3], P[7], P[11]};
            double C[3];
            for (int i = 0; i < 3; ++i) {
                double acc = 0;
                for (int k = 0; k < 3; ++k) acc += R[3 * k + i] * t[k];
                C[i] = -acc;
            }
            o.put(R, sizeof(R));
            o.put(C, sizeof(C));
        }
    }
    // images: Image{name, platformID, cameraID, poseID[, ID]}
    std::vector<uint32_t> pose_id(pl.image_shot.size());
    {
        std::vector<uint32_t> next(n_cameras, 0);
        for (size_t i = 0; i < pl.image_shot.size(); ++i) pose_id[i] = next[shots[pl.image_shot[i]].camera]++;
    }
    o.count(pl.image_shot.size());
    for (size_t i = 0; i < pl.image_shot.size(); ++i) {
        const sfmx_mvs_shot& sh = shots[pl.image_shot[i]];
        o.str(sh.image_name);
        o.pod((uint32_t)sh.camera);                  // platformID
        o.pod((uint32_t)0);                          // cameraID (:83)
        o.pod(pose_id[i]);                           // poseID (:84)
        if (version > 2) o.pod((uint32_t)0xFFFFFFFFu);   // ID: never set by toOpenMVS (NO_ID)
    }
    // vertices: Vertex{X (Point3f), views: View{imageID, confidence}}
    o.count(pl.vtx_point.size());
    const int64_t vbytes = 20 * (int64_t)pl.vtx_point.size() + 8 * (int64_t)pl.vtx_view.size();
    if (o.out && o.n + vbytes <= o.cap) {   // the section fits: written in place, element by element
        uint8_t* w = o.out + o.n;
        for (size_t v = 0; v < pl.vtx_point.size(); ++v) {
            const double* X = points + 3 * pl.vtx_point[v];
            const float Xf[3] = {(float)X[0], (float)X[1], (float)X[2]};
            const uint64_t nview = (uint64_t)(pl.vtx_off[v + 1] - pl.vtx_off[v]);
            std::memcpy(w, Xf, 12);
            std::memcpy(w + 12, &nview, 8);
            w += 20;
            for (int64_t k = pl.vtx_off[v]; k < pl.vtx_off[v + 1]; ++k) {
                const uint32_t id = pl.vtx_view[k];
                const float conf = 0.0f;                 // confidence (:115-118)
                std::memcpy(w, &id, 4);
                std::memcpy(w + 4, &conf, 4);
                w += 8;
            }
        }
        o.n += vbytes;
    } else
    for (size_t v = 0; v < pl.vtx_point.size(); ++v) {
        const double* X = points + 3 * pl.vtx_point[v];
        const float Xf[3] = {(float)X[0], (float)X[1], (float)X[2]};
        o.put(Xf, sizeof(Xf));
        o.count((uint64_t)(pl.vtx_off[v + 1] - pl.vtx_off[v]));
        for (int64_t k = pl.vtx_off[v]; k < pl.vtx_off[v + 1]; ++k) {
            o.pod(pl.vtx_view[k]);
            o.pod(0.0f);                             // confidence (:115-118)
        }
    }
    o.count(0);                                      // verticesNormal
    o.count(0);                                      // verticesColor
    if (version > 0) {
        o.count(0);                                  // lines
        o.count(0);                                  // linesNormal
        o.count(0);                                  // linesColor
        if (version > 1) {
            static const double I44[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
            o.put(I44, sizeof(I44));                 // transform (identity: toOpenMVS leaves it unset)
        }
    }
}

static int check(uint32_t version, const sfmx_mvs_camera* cameras, int32_t n_cameras, const sfmx_mvs_shot* shots,
                 int32_t n_shots, const double* points, int32_t n_points, const int64_t* oo, const int32_t* osh) {
    if (version < 1 || version > 3) { set_last_error("stream version must be 1..3"); return SFMX_EINVAL; }
    if (n_cameras < 0 || n_shots < 0 || n_points < 0) { set_last_error("negative count"); return SFMX_EINVAL; }
    if ((n_cameras && !cameras) || (n_shots && !shots) || (n_points && (!points || !oo))) {
        set_last_error("null argument");
        return SFMX_EINVAL;
    }
    if (n_points && oo[n_points] > 0 && !osh) { set_last_error("null origin shots"); return SFMX_EINVAL; }
    for (int c = 0; c < n_cameras; ++c)
        if (cameras[c].width < 0 || cameras[c].height < 0) { set_last_error("negative resolution"); return SFMX_EINVAL; }
    return SFMX_OK;
}

}  // namespace mvs
}  // namespace sfmx

using namespace sfmx;
using namespace sfmx::mvs;

extern "C" {

int sfmx_openmvs_serialize(uint32_t version, const sfmx_mvs_camera* cameras, int32_t n_cameras,
                           const sfmx_mvs_shot* shots, int32_t n_shots, const double* points, int32_t n_points,
                           const int64_t* origin_offsets, const int32_t* origin_shot, uint8_t* out,
                           int64_t capacity, int64_t* size, int32_t* n_images, int32_t* n_vertices) {
    int rc = check(version, cameras, n_cameras, shots, n_shots, points, n_points, origin_offsets, origin_shot);
    if (rc != SFMX_OK) return rc;
    if (!size || capacity < 0 || (capacity && !out)) { set_last_error("bad output buffer"); return SFMX_EINVAL; }
    Plan pl;
    rc = plan(shots, n_shots, n_cameras, n_points, origin_offsets, origin_shot, pl);
    if (rc != SFMX_OK) return rc;
    Sink o{out, capacity};
    emit(o, version, cameras, n_cameras, shots, points, pl);
    *size = o.n;
    if (n_images) *n_images = (int32_t)pl.image_shot.size();
    if (n_vertices) *n_vertices = (int32_t)pl.vtx_point.size();
    if (o.n > capacity) { set_last_error("output buffer too small"); return SFMX_ECAPACITY; }
    return SFMX_OK;
}

int sfmx_openmvs_write(const char* path, uint32_t version, const sfmx_mvs_camera* cameras, int32_t n_cameras,
                       const sfmx_mvs_shot* shots, int32_t n_shots, const double* points, int32_t n_points,
                       const int64_t* origin_offsets, const int32_t* origin_shot, int32_t* n_images,
                       int32_t* n_vertices) {
    if (!path) { set_last_error("null path"); return SFMX_EINVAL; }
    int64_t size = 0;
    int rc = sfmx_openmvs_serialize(version, cameras, n_cameras, shots, n_shots, points, n_points, origin_offsets,
                                    origin_shot, nullptr, 0, &size, n_images, n_vertices);
    if (rc != SFMX_OK && rc != SFMX_ECAPACITY) return rc;
    std::vector<uint8_t> buf((size_t)size);
    rc = sfmx_openmvs_serialize(version, cameras, n_cameras, shots, n_shots, points, n_points, origin_offsets,
                                origin_shot, buf.data(), size, &size, n_images, n_vertices);
    if (rc != SFMX_OK) return rc;
    std::FILE* f = std::fopen(path, "wb");
    if (!f) { set_last_error("cannot open the interface file for writing"); return SFMX_EINVAL; }
    const bool ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
    if (std::fclose(f) != 0 || !ok) { set_last_error("writing the interface file failed"); return SFMX_EDEVICE; }
    return SFMX_OK;
}

}  // extern "C"
