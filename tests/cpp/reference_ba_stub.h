// Minimal stand-ins for the reference-side types the bundle-adjustment adapter of
// INTEGRATION.md §4 (GpuBundleAdjustment.h) touches, with the names, members and semantics the
// reference gives them, so that the adapter compiles unchanged against libsfmx.so:
//   cv::Point2d / Point2f / Point3d, cv::Mat_<double> (at, copyTo);
//   ICamera (ICamera.h:34-179: getK / setK, getCenter / setCenter, getFocalLength /
//   setFocalLength as ICamera.cpp:27-66, ceresCostFunction's inputs, ceresCameraParameters(bool),
//   ceresApplyParameters) and its three classes with their ceresRepresentation blocks
//   (SimpleCamera.cpp:114-125 [f], SimpleRadialCamera.cpp:126-141 [f, k1, k2],
//   DistortionCamera.cpp:119-139 [f, cx, cy, k1, k2, p1, p2]);
//   CameraShot::getCamera / getPose / setPose (CameraShot.h:102-181), PointcloudElement
//   getCoordinates / setCoordinates / getOriginPoints (Scene.h:168-204), Scene::getCameras (the
//   shots' distinct cameras in shot order, Scene.cpp:356-367) / getShots / getPointcloud;
//   CeresPCE / CeresCameraShot (BundleAdjustment.h:28-64, read / write as BundleAdjustment.cpp:
//   143-184, the pose conversions of CeresUtils.h:90-148 through sfmx_pose_to_ceres / _from_ceres).
// Test scaffolding for the compiled BA adapter test only; not OpenCV, not Ceres.
#pragma once
#include <algorithm>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include <sfmx_ba.h>

namespace cv {
struct Point2d { double x = 0, y = 0; };
struct Point2f {
    float x = 0, y = 0;
    Point2f() = default;
    explicit Point2f(const Point2d& p) : x((float)p.x), y((float)p.y) {}
};
struct Point3d { double x = 0, y = 0, z = 0; };
template <class T> struct Mat_ {
    int rows = 0, cols = 0;
    std::vector<T> v;
    Mat_() = default;
    Mat_(int r, int c) : rows(r), cols(c), v((size_t)r * c, T(0)) {}
    template <class U> T& at(int i, int j) { return v[(size_t)i * cols + j]; }
    template <class U> const T& at(int i, int j) const { return v[(size_t)i * cols + j]; }
    void copyTo(Mat_& o) const { o = *this; }
};
}  // namespace cv

namespace photogrammetrie {
using std::shared_ptr;
using std::vector;
using std::pair;

class ICamera {
public:
    virtual ~ICamera() = default;
    virtual void getK(cv::Mat_<double>& K) const = 0;
    virtual void setK(const cv::Mat_<double>& K) = 0;
    virtual void setCenter(const double& cx, const double& cy) {
        cv::Mat_<double> K; getK(K); K.at<double>(0, 2) = cx; K.at<double>(1, 2) = cy; setK(K);
    }
    virtual void getCenter(double& cx, double& cy) const {
        cv::Mat_<double> K; getK(K); cx = K.at<double>(0, 2); cy = K.at<double>(1, 2);
    }
    virtual void setFocalLength(const double& fx, const double& fy) {
        cv::Mat_<double> K; getK(K); K.at<double>(0, 0) = fx; K.at<double>(1, 1) = fy; setK(K);
    }
    virtual void setFocalLength(const double& f) { setFocalLength(f, f); }
    virtual void getFocalLength(double& fx, double& fy) const {
        cv::Mat_<double> K; getK(K); fx = K.at<double>(0, 0); fy = K.at<double>(1, 1);
    }
    virtual void getFocalLength(double& f) const {
        double fx, fy; getFocalLength(fx, fy); f = (fx == fy) ? fx : (fx + fy) / 2.0;
    }
    virtual void getDistortion(cv::Mat_<double>& d) const { d = cv::Mat_<double>(1, 4); }
    virtual double* ceresCameraParameters(bool update = true) = 0;
    virtual void ceresApplyParameters() = 0;
};

class CameraBase : public ICamera {   // K handling shared by the three stand-ins (setK averages f)
public:
    CameraBase() : K(3, 3), distortion(1, 4) { K.at<double>(0, 0) = K.at<double>(1, 1) = 2500; K.at<double>(2, 2) = 1; }
    void getK(cv::Mat_<double>& out) const override { K.copyTo(out); }
    void setK(const cv::Mat_<double>& n) override {
        const double fx = n.at<double>(0, 0), fy = n.at<double>(1, 1);
        const double f = (fx == fy) ? fx : (fx + fy) / 2.0;
        K.at<double>(0, 0) = f; K.at<double>(1, 1) = f;
        K.at<double>(0, 2) = n.at<double>(0, 2); K.at<double>(1, 2) = n.at<double>(1, 2);
    }
    void getDistortion(cv::Mat_<double>& d) const override { distortion.copyTo(d); }
    cv::Mat_<double> K, distortion;
};

class SimpleCamera : public CameraBase {
public:
    static const int CeresRepresentationSize = 1;
    double ceresRepresentation[CeresRepresentationSize] = {0};
    double* ceresCameraParameters(bool update = true) override {
        if (update) getFocalLength(ceresRepresentation[0]);
        return ceresRepresentation;
    }
    void ceresApplyParameters() override { setFocalLength(ceresRepresentation[0]); }
};

class SimpleRadialCamera : public CameraBase {
public:
    static const int CeresRepresentationSize = 3;
    double ceresRepresentation[CeresRepresentationSize] = {0};
    double* ceresCameraParameters(bool update = true) override {
        if (update) {
            getFocalLength(ceresRepresentation[0]);
            ceresRepresentation[1] = distortion.at<double>(0, 0);
            ceresRepresentation[2] = distortion.at<double>(0, 1);
        }
        return ceresRepresentation;
    }
    void ceresApplyParameters() override {
        setFocalLength(ceresRepresentation[0]);
        distortion.at<double>(0, 0) = ceresRepresentation[1];
        distortion.at<double>(0, 1) = ceresRepresentation[2];
    }
};

class DistortionCamera : public CameraBase {
public:
    static const int CeresRepresentationSize = 7;
    double ceresRepresentation[CeresRepresentationSize] = {0};
    double* ceresCameraParameters(bool update = true) override {
        if (update) {
            getFocalLength(ceresRepresentation[0]);
            getCenter(ceresRepresentation[1], ceresRepresentation[2]);
            for (int i = 0; i < 4; ++i) ceresRepresentation[3 + i] = distortion.at<double>(0, i);
        }
        return ceresRepresentation;
    }
    void ceresApplyParameters() override {
        setFocalLength(ceresRepresentation[0]);
        setCenter(ceresRepresentation[1], ceresRepresentation[2]);
        for (int i = 0; i < 4; ++i) distortion.at<double>(0, i) = ceresRepresentation[3 + i];
    }
};

class CameraShot {
public:
    shared_ptr<ICamera> camera;
    cv::Mat_<double> pose{3, 4};
    const shared_ptr<ICamera>& getCamera() const { return camera; }
    const cv::Mat_<double>& getPose() const { return pose; }
    void setPose(const cv::Mat_<double>& p) { pose = p; }
};

class PointcloudElement {
public:
    cv::Point3d coordinates;
    vector<pair<shared_ptr<CameraShot>, cv::Point2d>> origins;
    const cv::Point3d& getCoordinates() const { return coordinates; }
    void setCoordinates(const cv::Point3d& c) { coordinates = c; }
    void getOriginPoints(vector<pair<shared_ptr<CameraShot>, cv::Point2d>>& out) const { out = origins; }
};

class Scene {
public:
    vector<shared_ptr<CameraShot>> shots;
    vector<shared_ptr<PointcloudElement>> pointcloud;
    vector<shared_ptr<ICamera>> getCameras() const {
        vector<shared_ptr<ICamera>> cameras;
        for (auto& shot : shots)
            if (std::find(cameras.begin(), cameras.end(), shot->getCamera()) == cameras.end())
                cameras.push_back(shot->getCamera());
        return cameras;
    }
    const vector<shared_ptr<CameraShot>>& getShots() const { return shots; }
    const vector<shared_ptr<PointcloudElement>>& getPointcloud() const { return pointcloud; }
};

struct CeresPCE {
    shared_ptr<PointcloudElement> pce;
    double coordinates[3]{0, 0, 0};
    void read() {
        const cv::Point3d& c = pce->getCoordinates();
        coordinates[0] = c.x; coordinates[1] = c.y; coordinates[2] = c.z;
    }
    void write() { pce->setCoordinates(cv::Point3d{coordinates[0], coordinates[1], coordinates[2]}); }
};

struct CeresCameraShot {
    shared_ptr<CameraShot> shot;
    double pose[6]{0, 0, 0, 0, 0, 0};
    void read() { sfmx_pose_to_ceres(shot->getPose().v.data(), pose); }   // CeresUtils::toCeresPose
    void write() {
        cv::Mat_<double> p(3, 4);
        sfmx_pose_from_ceres(pose, p.v.data());                           // CeresUtils::toOpenCvPose
        shot->setPose(p);
    }
};
}  // namespace photogrammetrie
