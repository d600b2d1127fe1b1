// Minimal stand-ins for the reference-side types the matching adapter touches, with the
// same names, members and layouts as the reference uses them, so that the adapter of
// INTEGRATION.md §2 (GpuFeatureMatchingStrategy.h) compiles unchanged against libsfmx.so:
//   cv::DMatch (16 B: queryIdx, trainIdx, imgIdx, distance), cv::Mat (data/rows/cols/type,
//   isContinuous), cv::Ptr, cv::DescriptorMatcher, CV_Assert;
//   photogrammetrie::Features / CameraShot::getFeatures (CameraShot.h:39-42, :95),
//   ShotMatches(left, right) / setMatches / getMatches (Scene.h:59, :81, :88),
//   Scene::getShots (Scene.h:396), IFeatureMatchingStrategy (IFeatureMatchingStrategy.h:34-48).
// These are test scaffolding for the compiled adapter test only; they are not OpenCV.
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <vector>

namespace cv {
constexpr int CV_8U_ = 0, CV_32F_ = 5;
struct DMatch {
    int queryIdx = -1, trainIdx = -1, imgIdx = -1;
    float distance = 0.f;
};
struct Mat {
    unsigned char* data = nullptr;
    int rows = 0, cols = 0, type_ = CV_32F_;
    int type() const { return type_; }
    bool isContinuous() const { return true; }
};
struct DescriptorMatcher {};
template <class T> using Ptr = std::shared_ptr<T>;
}  // namespace cv
#define CV_8U cv::CV_8U_
#define CV_32F cv::CV_32F_
#define CV_Assert(e) do { if (!(e)) throw std::runtime_error("CV_Assert: " #e); } while (0)

namespace photogrammetrie {
using std::shared_ptr;
using std::vector;
struct Features {
    vector<char> keypoints;   // unused by the adapter
    cv::Mat descriptors;
};
class CameraShot {
public:
    Features features;
    const Features& getFeatures() const { return features; }
};
class ShotMatches {
public:
    ShotMatches(const shared_ptr<CameraShot>& l, const shared_ptr<CameraShot>& r) : left(l), right(r) {}
    const vector<cv::DMatch>& getMatches() const { return matches; }
    void setMatches(const vector<cv::DMatch>& m) { matches = m; }
    shared_ptr<CameraShot> left, right;
    double homographyInlierRatio = -1;
private:
    vector<cv::DMatch> matches;
};
class Scene {
public:
    vector<shared_ptr<CameraShot>> shots;
    const vector<shared_ptr<CameraShot>>& getShots() const { return shots; }
};
class IFeatureMatchingStrategy {
public:
    virtual ~IFeatureMatchingStrategy() = default;
    virtual void calculateShotMatches(const Scene& scene, cv::Ptr<cv::DescriptorMatcher>& matcher,
                                      vector<ShotMatches>& matches) = 0;
};
}  // namespace photogrammetrie
