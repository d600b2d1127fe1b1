// The INTEGRATION.md §4 adapter, compiled: BundleAdjustment::doBundleAdjustment(Scene&)
// (BundleAdjustment.cpp:29-141) over sfmx_ba_solve.  The text between the markers is the one
// INTEGRATION.md shows (tests/test_abi.py checks that); tests/cpp/ba_adapter_main.cpp drives it
// with a reference-shaped Scene (tests/cpp/reference_ba_stub.h) and tests/test_gpu_adapter.py
// compares its results with the oracle.
#pragma once
#include <sfmx.h>
#include <sfmx_ba.h>
#include <algorithm>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace photogrammetrie {
// --- adapter begin ---
// in BundleAdjustment.cpp, replacing the AddResidualBlock loop + CeresUtils::solve (lines 45-91)
struct GpuBundleAdjustment {
    // the intrinsics block size of the camera class (its CeresRepresentationSize)
    static int32_t sfmxModel(const ICamera& cam) {
        if (dynamic_cast<const DistortionCamera*>(&cam)) return SFMX_CAM_DISTORTION;      // [f,cx,cy,k1,k2,p1,p2]
        if (dynamic_cast<const SimpleRadialCamera*>(&cam)) return SFMX_CAM_SIMPLE_RADIAL;  // [f,k1,k2]
        if (dynamic_cast<const SimpleCamera*>(&cam)) return SFMX_CAM_SIMPLE;              // [f]
        throw std::invalid_argument("GpuBundleAdjustment: unknown ICamera class");
    }

    static bool doBundleAdjustment(Scene& scene, sfmx_ba_summary* summaryOut = nullptr) {
        // :45-48: every camera of the scene gets its parameter block, refreshed from the camera
        vector<shared_ptr<ICamera>> cameras = scene.getCameras();
        std::unordered_map<const ICamera*, int32_t> camIdx;
        std::vector<int32_t> models, poseIntr;
        std::vector<double> intr, centers;
        for (auto& cam : cameras) {
            const double* blk = cam->ceresCameraParameters(true);
            const int32_t k = sfmxModel(*cam);
            camIdx.emplace(cam.get(), (int32_t)models.size());
            models.push_back(k);
            intr.insert(intr.end(), blk, blk + k);
            double cx, cy;
            cam->getCenter(cx, cy);                        // what SimpleRadialCamera.cpp:118-124 captures
            centers.push_back(cx);
            centers.push_back(cy);
        }
        // :50-91: points, shots in first-appearance order, one residual per origin point
        std::vector<shared_ptr<CeresPCE>> pces;
        std::vector<shared_ptr<CeresCameraShot>> shots;
        std::unordered_map<const CameraShot*, int32_t> shotIdx;   // O(1) instead of OpenMpUtils::find_if
        std::vector<double> pts, poses, xy;
        std::vector<int32_t> op, oc;
        for (auto& pce : scene.getPointcloud()) {
            auto cp = std::make_shared<CeresPCE>();
            cp->pce = pce;
            cp->read();
            const int32_t pi = (int32_t)pces.size();
            pces.push_back(cp);
            pts.insert(pts.end(), cp->coordinates, cp->coordinates + 3);
            vector<pair<shared_ptr<CameraShot>, cv::Point2d>> origins;
            pce->getOriginPoints(origins);
            for (auto& origin : origins) {
                const shared_ptr<CameraShot>& shot = origin.first;
                auto it = shotIdx.find(shot.get());
                if (it == shotIdx.end()) {
                    auto cs = std::make_shared<CeresCameraShot>();
                    cs->shot = shot;
                    cs->read();
                    it = shotIdx.emplace(shot.get(), (int32_t)shots.size()).first;
                    shots.push_back(cs);
                    poses.insert(poses.end(), cs->pose, cs->pose + 6);
                    poseIntr.push_back(camIdx.at(shot->getCamera().get()));   // :81 shot->getCamera()
                }
                const cv::Point2f pf(origin.second);       // ceresCostFunction takes a Point2f
                op.push_back(pi);
                oc.push_back(it->second);
                xy.push_back(pf.x);
                xy.push_back(pf.y);
            }
        }
        sfmx_ba_problem prob{};
        prob.n_points = (int32_t)pces.size();
        prob.n_cams = (int32_t)shots.size();
        prob.n_obs = (int32_t)op.size();
        prob.cam_model = models.empty() ? SFMX_CAM_SIMPLE : models[0];
        prob.points = pts.data();
        prob.poses = poses.data();
        prob.intr = intr.data();
        prob.obs_point = op.data();
        prob.obs_cam = oc.data();
        prob.obs_xy = xy.data();
        prob.n_intr = (int32_t)models.size();               // one block per camera (several allowed)
        prob.intr_model = models.data();
        prob.pose_intr = poseIntr.data();
        prob.intr_center = centers.data();
        sfmx_ba_options opt;
        sfmx_ba_default_options(&opt);                       // == CeresUtils::defaultOptions
        sfmx_ba_summary sum{};
        if (sfmx_ba_solve(&prob, &opt, &sum, nullptr, 0) < 0)    // e.g. SFMX_ECAPACITY: too many intrinsics
            throw std::runtime_error(std::string("sfmx_ba_solve: ") + sfmx_last_error());
        // :97-138: write-back of points, shots and every camera
        for (size_t i = 0; i < pces.size(); ++i) {
            std::copy_n(&pts[3 * i], 3, pces[i]->coordinates);
            pces[i]->write();
        }
        for (size_t i = 0; i < shots.size(); ++i) {
            std::copy_n(&poses[6 * i], 6, shots[i]->pose);
            shots[i]->write();
        }
        for (size_t m = 0, off = 0; m < cameras.size(); off += models[m], ++m) {
            std::copy_n(&intr[off], models[m], cameras[m]->ceresCameraParameters(false));
            cameras[m]->ceresApplyParameters();
        }
        if (summaryOut) *summaryOut = sum;
        return sum.termination_type == SFMX_BA_CONVERGENCE;   // :140
    }
};
// --- adapter end ---
}  // namespace photogrammetrie
