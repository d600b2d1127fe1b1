// Phase timing of workgroup 0 of the homography RANSAC kernel (wall_clock64,
// 100 MHz) on a synthetic 1225-pair graph: 500 matches per pair, 75 % inliers.
#define SFMX_HOMOG_STAMPS
#include "../../sfm-mvs-pipeline_amd/csrc/homography.hip"
#include <cstdio>
#include <random>
void sfmx::set_last_error(const char*) {}
int main() {
    const int npairs = 1225, per = 500, nimg = 2;
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> ux(0, 720), uy(0, 405);
    std::normal_distribution<float> nz(0, 0.7f);
    std::vector<sfmx_point2f> k0(per), k1(per);
    for (int i = 0; i < per; ++i) {
        k0[i] = {ux(rng), uy(rng)};
        if (i < per * 3 / 4) k1[i] = {0.9f * k0[i].x + 0.1f * k0[i].y + 20 + nz(rng), -0.05f * k0[i].x + 1.05f * k0[i].y - 10 + nz(rng)};
        else k1[i] = {ux(rng), uy(rng)};
    }
    std::vector<sfmx_dmatch> m((size_t)npairs * per);
    std::vector<int64_t> off(npairs + 1);
    std::vector<int32_t> pairs(2 * npairs);
    for (int p = 0; p < npairs; ++p) {
        off[p] = (int64_t)p * per; pairs[2 * p] = 0; pairs[2 * p + 1] = 1;
        for (int i = 0; i < per; ++i) m[(size_t)p * per + i] = {i, i, 0, 1.f};
    }
    off[npairs] = (int64_t)npairs * per;
    const sfmx_point2f* kp[2] = {k0.data(), k1.data()};
    int32_t nk[2] = {per, per}, sz[4] = {720, 405, 720, 405};
    std::vector<double> out(npairs);
    for (int rep = 0; rep < 2; ++rep) {
        int zero = 0;
        hipMemcpyToSymbol(HIP_SYMBOL(g_h_nst), &zero, sizeof zero);
        int rc = sfmx_homography_ratios(kp, nk, nimg, sz, pairs.data(), npairs, m.data(), off.data(), -3.0, 2000, 0.995, 0, 0, nullptr, out.data());
        long long st[256]; int ns = 0;
        hipMemcpyFromSymbol(st, HIP_SYMBOL(g_h_stamps), sizeof st);
        hipMemcpyFromSymbol(&ns, HIP_SYMBOL(g_h_nst), sizeof ns);
        printf("rc %d kernel %.3f ms ratio %.4f | wg0:", rc, sfmx_homography_last_kernel_ms(), out[0]);
        for (int i = 1; i < ns; ++i) printf(" %lld:%lld", st[i] & 255, (st[i] >> 8) - (st[i - 1] >> 8));
        printf("\n");
    }
    return 0;
}
