// Phase timing of the BA dense solve's diagonal-tile inverse (chol_first) and one
// trailing step (chol_step) on a random SPD 1216x1216 system; wall_clock64 stamps.
#define SFMX_CHOL_STAMPS
#include "../../sfm-mvs-pipeline_amd/csrc/ba_kernels.hpp"
#include <cstdio>
#include <vector>
#include <random>
using namespace sfmx::ba;
int main() {
    const int npad = 1216, T = npad / NB;
    std::vector<double> h((size_t)npad * npad + npad);
    std::mt19937 rng(3);
    std::normal_distribution<double> nd;
    std::vector<double> B((size_t)npad * 40);
    for (auto& v : B) v = nd(rng);
    for (int i = 0; i < npad; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = (i == j) ? npad : 0.0;
            for (int k = 0; k < 40; ++k) s += B[i * 40 + k] * B[j * 40 + k];
            h[(size_t)i * npad + j] = h[(size_t)j * npad + i] = s;
        }
    for (int i = 0; i < npad; ++i) h[(size_t)npad * npad + i] = nd(rng);
    double *S, *W, *S0; int* fail;
    hipMalloc(&S, h.size() * 8); hipMalloc(&S0, h.size() * 8); hipMalloc(&W, 2 * NB * NB * 8); hipMalloc(&fail, 4);
    hipMemcpy(S0, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipMemset(fail, 0, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    long long st[64];
    for (int rep = 0; rep < 3; ++rep) {
        hipMemcpy(S, S0, h.size() * 8, hipMemcpyDeviceToDevice);
        double* rhs = S + (size_t)npad * npad;
        hipEventRecord(e0);
        chol_first<<<1, 256>>>(S, npad, W, rhs, fail);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpyFromSymbol(st, HIP_SYMBOL(g_chol_stamps), sizeof st);
        printf("chol_first %.2f us | load %lld", ms * 1e3, st[1] - st[0]);
        for (int s = 0; s < 4; ++s)
            printf(" | s%d panel->inner %lld inner %lld M %lld upd %lld", s, st[2 + 4 * s] - (s ? st[1 + 4 * s] : st[1]),
                   st[3 + 4 * s] - st[2 + 4 * s], st[4 + 4 * s] - st[3 + 4 * s], st[5 + 4 * s] - st[4 + 4 * s]);
        printf(" | store %lld rhs %lld  (ticks of 100 MHz wall clock)\n", st[20] - st[17], st[21] - st[20]);
        hipEventRecord(e0);
        const int m = T - 1;
        chol_step<<<m * (m + 1) / 2, 256>>>(S, npad, 0, W, rhs, fail, nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpyFromSymbol(st, HIP_SYMBOL(g_chol_stamps), sizeof st);
        printf("chol_step(0) %.2f us: load %lld gemm1 %lld store+gemm2 %lld -> inverse %lld | diag inverse %lld | GT %lld ticks\n", ms * 1e3,
               st[31] - st[30], st[32] - st[31], st[33] - st[32], st[0] - st[33], st[21] - st[0], st[34] - st[21]);
    }
    int hf; hipMemcpy(&hf, fail, 4, hipMemcpyDeviceToHost);
    printf("fail flag %d\n", hf);
    return 0;
}
