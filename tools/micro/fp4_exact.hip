// Micro-test: exactness of v_mfma_scale_f32_32x32x64_f8f6f4 (FP4 +-1 operands,
// unit scales) with a fractional C operand in [511, 1024): prints acc vs the
// exact value for one 32x32 tile (row i = train, col j = query).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cmath>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const uint32_t* A, const uint32_t* B, const float* C, float* D, int variant) {
    const int lane = threadIdx.x, h = lane >> 5, l32 = lane & 31;
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = C[(r / 4) * 8 + h * 4 + (r % 4)];
    for (int m = 0; m < 4; ++m) {
        const i32x4 a = *reinterpret_cast<const i32x4*>(A + l32 * 32 + 4 * (2 * m + h));
        const i32x4 b = *reinterpret_cast<const i32x4*>(B + l32 * 32 + 4 * (2 * m + h));
        i32x8 a8 = {a.x, a.y, a.z, a.w, 0, 0, 0, 0}, b8 = {b.x, b.y, b.z, b.w, 0, 0, 0, 0};
        if (variant == 0)
            acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc, 4, 4, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
        else   // reference: C added afterwards on the VALU
            acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc, 4, 4, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
    }
    for (int r = 0; r < 16; ++r) D[((r / 4) * 8 + h * 4 + (r % 4)) * 32 + l32] = acc[r];
}

static uint32_t enc(unsigned byte) { uint32_t w = 0; for (int b = 0; b < 8; ++b) w |= (((byte >> b) & 1u) ? 0x2u : 0xAu) << (4 * b); return w; }

int main() {
    srand(7);
    uint8_t t[32][32], q[32][32];
    for (int i = 0; i < 32; ++i) for (int c = 0; c < 32; ++c) t[i][c] = rand() & 255;
    for (int c = 0; c < 32; ++c) { t[9][c] = t[4][c]; t[30][c] = t[4][c]; }
    for (int j = 0; j < 32; ++j) for (int c = 0; c < 32; ++c) q[j][c] = (j == 0) ? (t[4][c] ^ 1) : (rand() & 255);
    uint32_t hA[32 * 32], hB[32 * 32]; float hC[32], hD[32 * 32];
    for (int i = 0; i < 32; ++i) for (int c = 0; c < 32; ++c) { hA[i * 32 + c] = enc(t[i][c]); hB[i * 32 + c] = enc(q[i][c]); }
    for (int i = 0; i < 32; ++i) hC[i] = (float)(767 * 16384 + 16383 - i) / 16384.0f;
    uint32_t *dA, *dB; float *dC, *dD;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC); hipMalloc(&dD, sizeof hD);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dA, dB, dC, dD, 0);
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    int bad = 0, badint = 0;
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
        int hd = 0; for (int c = 0; c < 32; ++c) hd += __builtin_popcount(t[i][c] ^ q[j][c]);
        const double exact = (double)hC[i] + (256 - 2 * hd);
        const float got = hD[i * 32 + j];
        if ((double)got != exact) { if (bad < 8) printf("row %d col %d: got %.8f exact %.8f (hd %d)\n", i, j, got, exact, hd); ++bad; }
        if (floorf(got) != floor(exact)) ++badint;
    }
    printf("mismatches %d / 1024 (integer part wrong: %d)\n", bad, badint);
    for (int i : {4, 9, 30}) printf("row %2d col 0: %.8f bits %08x\n", i, hD[i * 32], *(uint32_t*)&hD[i * 32]);
    return 0;
}
