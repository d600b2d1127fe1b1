// Compiled caller of the BA ABI: builds a reference-shaped Scene
// (reference_ba_stub.h) and runs INTEGRATION.md §4's GpuBundleAdjustment::doBundleAdjustment on
// it, as SfM.cpp:235 / :371 call BundleAdjustment::doBundleAdjustment(scene).
// Input file (little-endian):
//   int32 M (cameras), S (shots), P (points)
//   per camera: int32 model (1 / 3 / 7), double f, cx, cy, d[4] (distortion k1, k2, p1, p2)
//   per shot:   int32 camera, double Rt[12] (3x4 row-major pose)
//   per point:  double xyz[3], int32 n, then n x (int32 shot, double x, double y)
// Output file: int32 converged, int32 termination, int32 successful, int32 unsuccessful,
//   double initial_cost, final_cost, then P x 3 coordinates, S x 12 poses, M x (f, cx, cy, d[4]).
#include <cstdio>
#include <cstring>
#include <map>
#include "reference_ba_stub.h"
#include "GpuBundleAdjustment.h"

using namespace photogrammetrie;

static bool rd(FILE* f, void* p, size_t n) { return std::fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
    if (argc != 3) { std::fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 2; }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t hdr[3];
    if (!rd(f, hdr, sizeof hdr)) return 2;
    const int M = hdr[0], S = hdr[1], P = hdr[2];
    Scene scene;
    std::vector<shared_ptr<ICamera>> cams;
    for (int m = 0; m < M; ++m) {
        int32_t model;
        double v[7];
        if (!rd(f, &model, 4) || !rd(f, v, sizeof v)) return 2;
        shared_ptr<CameraBase> c;
        if (model == 1) c = std::make_shared<SimpleCamera>();
        else if (model == 3) c = std::make_shared<SimpleRadialCamera>();
        else c = std::make_shared<DistortionCamera>();
        c->K.at<double>(0, 0) = c->K.at<double>(1, 1) = v[0];
        c->K.at<double>(0, 2) = v[1];
        c->K.at<double>(1, 2) = v[2];
        for (int i = 0; i < 4; ++i) c->distortion.at<double>(0, i) = v[3 + i];
        cams.push_back(c);
    }
    for (int s = 0; s < S; ++s) {
        int32_t cam;
        auto shot = std::make_shared<CameraShot>();
        if (!rd(f, &cam, 4) || !rd(f, shot->pose.v.data(), 12 * sizeof(double))) return 2;
        shot->camera = cams.at(cam);
        scene.shots.push_back(shot);
    }
    for (int p = 0; p < P; ++p) {
        auto e = std::make_shared<PointcloudElement>();
        int32_t n;
        if (!rd(f, &e->coordinates, 3 * sizeof(double)) || !rd(f, &n, 4)) return 2;
        for (int i = 0; i < n; ++i) {
            int32_t s;
            cv::Point2d q;
            if (!rd(f, &s, 4) || !rd(f, &q.x, 8) || !rd(f, &q.y, 8)) return 2;
            e->origins.emplace_back(scene.shots.at(s), q);
        }
        scene.pointcloud.push_back(e);
    }
    std::fclose(f);
    sfmx_ba_summary sum{};
    bool converged = false;
    try {
        converged = GpuBundleAdjustment::doBundleAdjustment(scene, &sum);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "doBundleAdjustment: %s\n", e.what());
        return 1;
    }
    FILE* o = std::fopen(argv[2], "wb");
    if (!o) return 2;
    const int32_t head[4] = {converged ? 1 : 0, sum.termination_type, sum.num_successful_steps, sum.num_unsuccessful_steps};
    std::fwrite(head, 4, 4, o);
    std::fwrite(&sum.initial_cost, 8, 1, o);
    std::fwrite(&sum.final_cost, 8, 1, o);
    for (auto& e : scene.pointcloud) std::fwrite(&e->coordinates, 8, 3, o);
    for (auto& s : scene.shots) std::fwrite(s->pose.v.data(), 8, 12, o);
    for (auto& c : cams) {
        cv::Mat_<double> K, d;
        c->getK(K);
        c->getDistortion(d);
        const double v[7] = {K.at<double>(0, 0), K.at<double>(0, 2), K.at<double>(1, 2), d.at<double>(0, 0),
                             d.at<double>(0, 1), d.at<double>(0, 2), d.at<double>(0, 3)};
        std::fwrite(v, 8, 7, o);
    }
    std::fclose(o);
    std::printf("ok converged=%d cost %.17g -> %.17g\n", (int)converged, sum.initial_cost, sum.final_cost);
    return 0;
}
