// Compiled caller of the C ABI: drives INTEGRATION.md §2's
// GpuFeatureMatchingStrategy through a reference-shaped Scene, as SfM.cpp:545 calls
// calculateShotMatches.  Input file (little-endian): int32 n, mode (0 unordered,
// 1 video, 2 grid), seq, rowLen; then per image int32 rows, cols, type (0 = CV_8U,
// 5 = CV_32F) and rows*cols elements.  Output file: int64 n_pairs, then per pair int32
// left, right, int64 count and count x 16-B cv::DMatch.  Exit code 0 on success.
#include <cstdio>
#include <cstring>
#include <string>
#include "reference_stub.h"
#include "GpuFeatureMatchingStrategy.h"

using namespace photogrammetrie;

static bool rd(FILE* f, void* p, size_t n) { return std::fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
    if (argc != 3) { std::fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 2; }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t hdr[4];
    if (!rd(f, hdr, sizeof hdr)) return 2;
    Scene scene;
    std::vector<std::vector<unsigned char>> store(hdr[0]);
    for (int i = 0; i < hdr[0]; ++i) {
        int32_t rct[3];
        if (!rd(f, rct, sizeof rct)) return 2;
        const size_t bytes = (size_t)rct[0] * rct[1] * (rct[2] == CV_32F ? 4 : 1);
        store[i].resize(bytes + 1);
        if (bytes && !rd(f, store[i].data(), bytes)) return 2;
        auto shot = std::make_shared<CameraShot>();
        shot->features.descriptors.data = store[i].data();
        shot->features.descriptors.rows = rct[0];
        shot->features.descriptors.cols = rct[1];
        shot->features.descriptors.type_ = rct[2];
        scene.shots.push_back(shot);
    }
    std::fclose(f);
    const auto mode = hdr[1] == 0 ? GpuFeatureMatchingStrategy::Pairs::Unordered
                    : hdr[1] == 1 ? GpuFeatureMatchingStrategy::Pairs::Video : GpuFeatureMatchingStrategy::Pairs::Grid;
    GpuFeatureMatchingStrategy strategy(mode, hdr[2], hdr[3], 1);
    IFeatureMatchingStrategy& iface = strategy;
    cv::Ptr<cv::DescriptorMatcher> matcher = std::make_shared<cv::DescriptorMatcher>();
    vector<ShotMatches> out;
    try {
        iface.calculateShotMatches(scene, matcher, out);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "calculateShotMatches: %s\n", e.what());
        return 1;
    }
    FILE* o = std::fopen(argv[2], "wb");
    if (!o) return 2;
    const int64_t np = (int64_t)out.size();
    std::fwrite(&np, 8, 1, o);
    for (const ShotMatches& sm : out) {
        int32_t lr[2] = {-1, -1};
        for (int i = 0; i < hdr[0]; ++i) {
            if (scene.shots[i] == sm.left) lr[0] = i;
            if (scene.shots[i] == sm.right) lr[1] = i;
        }
        const int64_t c = (int64_t)sm.getMatches().size();
        std::fwrite(lr, 4, 2, o);
        std::fwrite(&c, 8, 1, o);
        if (c) std::fwrite(sm.getMatches().data(), sizeof(cv::DMatch), (size_t)c, o);
    }
    std::fclose(o);
    std::printf("ok %lld pairs\n", (long long)np);
    return 0;
}
