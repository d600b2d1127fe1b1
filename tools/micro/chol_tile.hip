// Phase timing of the BA solve's diagonal-tile inverse (chol_leaves, one leaf) and one level of
// trailing updates (chol_level: every tile below panel 0, natural order) on a random SPD 1216x1216
// system with 4 right-hand sides; wall_clock64 stamps.
#define SFMX_CHOL_STAMPS
#include "../../sfm-mvs-pipeline_amd/csrc/ba_chol.hpp"
#include <cstdio>
#include <vector>
#include <random>
using namespace sfmx::ba;
int main() {
    const int npad = 1216, T = npad / NB;
    constexpr int RW = 4;
    std::vector<double> h((size_t)npad * npad + (size_t)npad * RW);
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
    for (int i = 0; i < npad * RW; ++i) h[(size_t)npad * npad + i] = nd(rng);
    // level 0 of a natural-order plan: panel 0 updates every tile (a, b), 1 <= b <= a; (1, 1) inverts
    std::vector<int4> tasks;
    tasks.push_back(make_int4(1, 1, 0, 1));
    for (int a = 1; a < T; ++a)
        for (int b = 1; b <= a; ++b)
            if (a != 1 || b != 1) tasks.push_back(make_int4(a, b, 0, 1));
    int zero = 0;
    double *S, *W, *S0, *contrib; int *fail, *src, *leaves; int4* dt;
    hipMalloc(&S, h.size() * 8); hipMalloc(&S0, h.size() * 8); hipMalloc(&W, (size_t)T * NB * NB * 8); hipMalloc(&fail, 64);
    hipMalloc(&contrib, (size_t)T * 3 * RW * 8); hipMalloc(&src, 4); hipMalloc(&leaves, 4); hipMalloc(&dt, tasks.size() * 16);
    hipMemcpy(src, &zero, 4, hipMemcpyHostToDevice); hipMemcpy(leaves, &zero, 4, hipMemcpyHostToDevice);
    hipMemcpy(dt, tasks.data(), tasks.size() * 16, hipMemcpyHostToDevice);
    hipMemcpy(S0, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipMemset(fail, 0, 64);
    { const int one = 1; hipMemcpy(fail + 1, &one, 4, hipMemcpyHostToDevice); }   // the step gate open (ba_kernels.hpp step_gated)
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int* zpre; hipMalloc(&zpre, 4 * 64); hipMemset(zpre, 0, 4 * 64);   // no pre-swept panels
    long long st[64];
    for (int rep = 0; rep < 3; ++rep) {
        hipMemcpy(S, S0, h.size() * 8, hipMemcpyDeviceToDevice);
        double* R = S + (size_t)npad * npad;
        hipEventRecord(e0);
        chol_leaves<RW><<<1, 256>>>(S, npad, R, leaves, W, contrib, fail);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpyFromSymbol(st, HIP_SYMBOL(g_chol_stamps), sizeof st);
        printf("chol_leaves %.2f us | load %lld", ms * 1e3, st[1] - st[0]);
        for (int s = 0; s < 4; ++s)
            printf(" | s%d panel->inner %lld inner %lld M %lld upd %lld", s, st[2 + 4 * s] - (s ? st[1 + 4 * s] : st[1]),
                   st[3 + 4 * s] - st[2 + 4 * s], st[4 + 4 * s] - st[3 + 4 * s], st[5 + 4 * s] - st[4 + 4 * s]);
        printf(" | store %lld rhs %lld (w %lld sync %lld contrib %lld)  (ticks of 100 MHz wall clock)\n", st[20] - st[17], st[21] - st[20],
               st[22] - st[20], st[23] - st[22], st[21] - st[23]);
        hipEventRecord(e0);
        chol_level<RW><<<(unsigned)tasks.size(), 256>>>(S, npad, R, dt, src, 1, W, contrib, fail, zpre);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpyFromSymbol(st, HIP_SYMBOL(g_chol_stamps), sizeof st);
        printf("chol_level(0) %.2f us: load %lld gemm1 %lld store+gemm2 %lld -> inverse %lld | diag inverse %lld | GT %lld ticks\n", ms * 1e3,
               st[31] - st[30], st[32] - st[31], st[33] - st[32], st[0] - st[33], st[21] - st[0], st[34] - st[21]);
    }
    // the leaf inverse of tile 0 through the one-launch kernels: chol_factor (NW waves) vs chol_factor_w
    // (NW x NW waves), one item each (a leaf), 5 launches each, alternating
    {
        const int nver = T * (T + 1) / 2;
        int4 leaf = make_int4(0, -1, 0, 0), zero4 = make_int4(0, 0, 0, 0);
        int4 *items, *need; int *ctr, *tctr; double* pbuf;
        hipMalloc(&items, 16); hipMalloc(&need, 16); hipMalloc(&ctr, 4 * (nver + 4)); hipMalloc(&tctr, 64);
        hipMalloc(&pbuf, 8 * 8192);
        hipMemcpy(items, &leaf, 16, hipMemcpyHostToDevice); hipMemcpy(need, &zero4, 16, hipMemcpyHostToDevice);
        hipMemset(ctr, 0, 4 * (nver + 4)); hipMemset(tctr, 0, 64);
        double* R = S + (size_t)npad * npad;
        for (int rep = 0; rep < 5; ++rep)
            for (int wide = 0; wide < 2; ++wide) {
                hipMemcpy(S, S0, h.size() * 8, hipMemcpyDeviceToDevice);
                float ms;
                hipEventRecord(e0);
                if (wide) chol_factor_w<RW><<<1, NTW>>>(S, npad, R, dt, items, need, src, W, contrib, fail, pbuf, tctr, ctr, 1, nver, DAG_TIMEOUT);
                else chol_factor<RW><<<1, NTH>>>(S, npad, R, dt, items, need, src, W, contrib, fail, pbuf, tctr, ctr, 1, nver, DAG_TIMEOUT,
                                                 need /* all-zero row masks: a leaf with no padding panel */);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
                printf("leaf inverse via %s: %.2f us\n", wide ? "chol_factor_w (16 waves)" : "chol_factor (4 waves)  ", ms * 1e3);
            }
    }
    int hf; hipMemcpy(&hf, fail, 4, hipMemcpyDeviceToHost);
    printf("fail flag %d\n", hf);
    return 0;
}
