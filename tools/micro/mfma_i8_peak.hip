// Practical int8 MFMA ceiling on this part: register-resident v_mfma_i32_16x16x64_i8 chains (no LDS,
// no HBM), with and without the screen's v_max3 epilogue, on uniform-random and SIFT-like operand
// bytes.  Reports TOP/s, the fraction of the nominal 5033 TOP/s dense peak, and the shader clock
// the chip held (clock64 / wall_clock64 of one wave).  Measurement only, never in the product.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_i8_peak tools/micro/mfma_i8_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int NACC, bool MAX3>
__global__ __launch_bounds__(256, 2) void peak_kernel(const i32x4* __restrict__ src, int iters, int* __restrict__ out,
                                                      long long* __restrict__ clk) {
    const int lane = threadIdx.x & 63;
    const int base = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 * 8;
    i32x4 a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        a[k] = src[(base + k * 64 + lane) & ((1 << 20) - 1)];
        b[k] = src[(base + (k + 4) * 64 + lane) & ((1 << 20) - 1)];
    }
    i32x4 acc[NACC];
    int ch[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = i32x4{j, 0, 0, 0};
    const long long t0 = clock64(), w0 = wall_clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) {
            if (MAX3) {   // the screen: fresh C each pair of MFMAs, v_max3 folds the results
                i32x4 c = i32x4{it, j, 0, 0};
                c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[j & 3], b[(j + it) & 3], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[(j + 1) & 3], b[(j + 2) & 3], c, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 4; ++i) ch[i] = max(max(ch[i], c[i]), acc[j][i]);
                acc[j] = c;
            } else {
                acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[j & 3], b[(j + it) & 3], acc[j], 0, 0, 0);
            }
        }
    }
    const long long t1 = clock64(), w1 = wall_clock64();
    int s = ch[0] ^ ch[1] ^ ch[2] ^ ch[3];
#pragma unroll
    for (int j = 0; j < NACC; ++j) s ^= acc[j][0] ^ acc[j][1] ^ acc[j][2] ^ acc[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = w1 - w0;
    }
}

template <int NACC, bool MAX3>
void run(const char* name, const i32x4* d_src, int* d_out, long long* d_clk, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    peak_kernel<NACC, MAX3><<<blocks, 256>>>(d_src, iters / 10, d_out, d_clk);   // warm-up
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        hipEventRecord(e0);
        peak_kernel<NACC, MAX3><<<blocks, 256>>>(d_src, iters, d_out, d_clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    long long clk[2];
    hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost);
    const double mfmas = (double)blocks * 4 * iters * NACC * (MAX3 ? 2 : 1);
    const double tops = mfmas * 16 * 16 * 64 * 2 / (best * 1e-3) / 1e12;
    const double ghz = clk[1] > 0 ? (double)clk[0] / ((double)clk[1] / 100e6) / 1e9 : 0.0;
    printf("%-34s %8.3f ms  %7.1f TOP/s  %.3f of 5033  clock %.2f GHz\n", name, best, tops, tops / 5033.1648, ghz);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    const int blocks = 256 * 2 * 4;   // 4 rounds of 2 blocks x 4 waves per CU
    std::vector<int8_t> h(16u << 20);
    std::mt19937 rng(7);
    i32x4* d_src;
    int* d_out;
    long long* d_clk;
    hipMalloc(&d_src, h.size());
    hipMalloc(&d_out, (size_t)blocks * 256 * 4);
    hipMalloc(&d_clk, 16);
    for (int pattern = 0; pattern < 2; ++pattern) {
        // 0: uniform random bytes; 1: SIFT-like (u8 descriptor values, mostly small, stored as v - 128)
        std::exponential_distribution<double> ex(1.0 / 20.0);
        for (auto& v : h) v = pattern == 0 ? (int8_t)(rng() & 255) : (int8_t)(std::min(255.0, ex(rng)) - 128);
        hipMemcpy(d_src, h.data(), h.size(), hipMemcpyHostToDevice);
        printf("operands: %s\n", pattern == 0 ? "uniform random bytes" : "SIFT-like (v - 128, v ~ Exp(20))");
        run<8, false>("8 chains, MFMA only", d_src, d_out, d_clk, blocks, iters);
        run<4, false>("4 chains, MFMA only", d_src, d_out, d_clk, blocks, iters);
        run<8, true>("8 x (2 MFMA + 4 v_max3), screen-like", d_src, d_out, d_clk, blocks, iters / 2);
    }
    hipFree(d_src);
    hipFree(d_out);
    hipFree(d_clk);
    return 0;
}
