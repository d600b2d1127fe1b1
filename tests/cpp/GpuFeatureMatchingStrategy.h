// The IFeatureMatchingStrategy adapter of INTEGRATION.md §2, verbatim between the markers
// (tests/test_abi.py checks INTEGRATION.md holds the same text).  Compiled against
// tests/cpp/reference_stub.h here; in the reference it includes the real headers.
#pragma once
#include <sfmx.h>
// --- adapter begin ---
namespace photogrammetrie {
class GpuFeatureMatchingStrategy : public IFeatureMatchingStrategy {
public:
    enum class Pairs { Unordered, Video, Grid };
    GpuFeatureMatchingStrategy(Pairs p, int seq = 2, int rowLen = 0, int nGpus = 1)
        : pairs_(p), seq_(seq), rowLen_(rowLen), nGpus_(nGpus) {}

    void calculateShotMatches(const Scene& scene, cv::Ptr<cv::DescriptorMatcher>& matcher,
                              vector<ShotMatches>& out) override {
        const auto& shots = scene.getShots();
        const int n = (int)shots.size();
        // 1. pair list, same order as the reference strategies
        int64_t np = pairs_ == Pairs::Unordered ? sfmx_pairs_unordered(n, nullptr, 0)
                   : pairs_ == Pairs::Video     ? sfmx_pairs_video(n, seq_, nullptr, 0)
                                                : sfmx_pairs_grid(n, seq_, rowLen_, /*grid_mode*/0, nullptr, 0);
        std::vector<int32_t> pr(2 * np);
        if (pairs_ == Pairs::Unordered) sfmx_pairs_unordered(n, pr.data(), np);
        else if (pairs_ == Pairs::Video) sfmx_pairs_video(n, seq_, pr.data(), np);
        else sfmx_pairs_grid(n, seq_, rowLen_, 0, pr.data(), np);
        // 2. descriptor views (CV_32F N x 128 for SIFT, CV_8U N x 32 for ORB), no copies
        std::vector<sfmx_desc> d(n);
        for (int i = 0; i < n; ++i) {
            const cv::Mat& m = shots[i]->getFeatures().descriptors;      // CameraShot.h:41
            CV_Assert(m.isContinuous());
            d[i] = {m.data, m.rows, m.cols, m.type() == CV_32F ? SFMX_32F : SFMX_8U, 0};
        }
        // the norm follows the descriptor type exactly as the CLI's matcher factory
        // pairs them (PhotogrammetrieCli.cpp:359-392): SIFT (CV_32F) -> L2, ORB (CV_8U) -> Hamming
        (void)matcher;
        const int nt = (d.empty() || d[0].type == SFMX_32F) ? SFMX_NORM_L2 : SFMX_NORM_HAMMING;
        // 3. match all pairs in ONE call: 2-NN + Lowe 0.7 (UnorderedFeatureMatchingStrategy.cpp:55-64).
        //    Each query (left feature) yields at most one match, so sum(rows(left)) is a sufficient
        //    capacity.  distinct/min_count = 0 keeps the SfM filters on the host exactly where they
        //    are today; pass SfM's flags here to run them on the GPU instead (SfM.cpp:547-570).
        int64_t cap = 0;
        for (int64_t p = 0; p < np; ++p) cap += d[pr[2 * p]].rows;
        std::vector<cv::DMatch> all(cap);
        std::vector<int64_t> off(np + 1);
        int64_t got = 0;
        static_assert(sizeof(cv::DMatch) == sizeof(sfmx_dmatch), "layout");
        const int rc = sfmx_match_pairs(d.data(), n, pr.data(), (int32_t)np, nt, 0.7, 0, 0, nGpus_,
                                        reinterpret_cast<sfmx_dmatch*>(all.data()), cap, &got, off.data(), nullptr);
        if (rc != SFMX_OK) throw std::runtime_error(sfmx_last_error());
        // 4. ShotMatches in pair order (the reference's order is nondeterministic under OMP)
        for (int64_t p = 0; p < np; ++p) {
            ShotMatches sm(shots[pr[2 * p]], shots[pr[2 * p + 1]]);
            sm.setMatches(vector<cv::DMatch>(all.begin() + off[p], all.begin() + off[p + 1]));
            out.push_back(sm);
        }
    }
private:
    Pairs pairs_; int seq_, rowLen_, nGpus_;
};
}
// --- adapter end ---
