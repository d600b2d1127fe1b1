// Micro-benchmark: issue rate and semantics of v_lshl_add_u64 (shift 9) vs v_lshl_add_u32 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void sem(const unsigned long long* a, const unsigned long long* b, unsigned long long* o) {
    int i = threadIdx.x;
    unsigned long long d;
    asm volatile("v_lshl_add_u64 %0, %1, 9, %2" : "=v"(d) : "v"(a[i]), "v"(b[i]));
    o[i] = d;
}

template <int MODE>
__global__ __launch_bounds__(256) void rate(unsigned* out, int iters, long long* cyc) {
    unsigned long long x[8];
    unsigned y[16];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 7 + i;
    for (int i = 0; i < 16; ++i) y[i] = threadIdx.x * 3 + i;
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (MODE == 0) asm volatile("v_lshl_add_u64 %0, %0, 9, %1" : "+v"(x[i]) : "v"(x[(i + 1) & 7]));
            else if (MODE == 1) {
                asm volatile("v_lshl_add_u32 %0, %0, 9, %1" : "+v"(y[2 * i]) : "v"(y[(2 * i + 3) & 15]));
                asm volatile("v_lshl_add_u32 %0, %0, 9, %1" : "+v"(y[2 * i + 1]) : "v"(y[(2 * i + 4) & 15]));
            } else {
                asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(x[i]) : "v"(x[(i + 1) & 7]));
            }
        }
    }
    long long t1 = clock64();
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s ^= (unsigned)x[i] ^ (unsigned)(x[i] >> 32);
    for (int i = 0; i < 16; ++i) s ^= y[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    const int n = 64;
    unsigned long long ha[n], hb[n], ho[n];
    for (int i = 0; i < n; ++i) {
        ha[i] = ((unsigned long long)(0x3FFFFFu - i * 977) << 32) | (0x2FFFFFu + i * 1231);
        hb[i] = ((unsigned long long)(0x1000000u + i) << 32) | (0x20000000u - i * 5);
    }
    unsigned long long *da, *db, *dout;
    CHECK(hipMalloc(&da, sizeof ha)); CHECK(hipMalloc(&db, sizeof hb)); CHECK(hipMalloc(&dout, sizeof ho));
    CHECK(hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice));
    sem<<<1, n>>>(da, db, dout);
    CHECK(hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < n; ++i) if (ho[i] != (ha[i] << 9) + hb[i]) ++bad;
    printf("v_lshl_add_u64 shift 9 semantics: %s (%d mismatches; e.g. got %llx want %llx, shift1 %llx)\n",
           bad ? "MASKED/WRONG" : "exact", bad, ho[0], (ha[0] << 9) + hb[0], (ha[0] << 1) + hb[0]);
    unsigned* o; long long* cyc; CHECK(hipMalloc(&o, 4 << 20)); CHECK(hipMalloc(&cyc, 8));
    const int iters = 4096;
    const char* names[3] = {"v_lshl_add_u64 <<9 (8 per iter)", "v_lshl_add_u32 <<9 (16 per iter)", "v_lshl_add_u64 <<2 (8 per iter)"};
    for (int mode = 0; mode < 3; ++mode) {
        for (int waves = 1; waves <= 4; waves *= 2) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            // one block per CU, `waves` waves per SIMD
            dim3 grid(256), block(256 * waves > 1024 ? 1024 : 256 * waves);
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) rate<0><<<grid, block>>>(o, iters, cyc);
                else if (mode == 1) rate<1><<<grid, block>>>(o, iters, cyc);
                else rate<2><<<grid, block>>>(o, iters, cyc);
                hipEventRecord(e1);
                CHECK(hipEventSynchronize(e1));
            }
            long long c; CHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            float ms; hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_wave = (double)iters * (mode == 1 ? 16 : 8);
            printf("%-36s waves/SIMD=%d  clock64 cyc per instr per wave = %.2f  wall %.3f ms\n", names[mode], waves,
                   (double)c / instr_per_wave, ms);
        }
    }
    return 0;
}
