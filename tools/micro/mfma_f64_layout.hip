// Operand/result lane layout of v_mfma_f64_16x16x4f64: infer (row, col) of each
// result register from a product with distinct entries.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* D) {
    const int l = threadIdx.x;
    const double a = A[(l % 16) * 4 + l / 16];     // A[m][k], m = l % 16, k = l / 16
    const double b = B[(l / 16) * 16 + l % 16];    // B[k][n], k = l / 16, n = l % 16
    f64x4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[l * 4 + r] = acc[r];
}
int main() {
    double hA[64], hB[64], hD[256], ref[256];
    for (int i = 0; i < 16; ++i) for (int kk = 0; kk < 4; ++kk) hA[i * 4 + kk] = (kk == 0) ? i : 0;          // row index in k=0
    for (int kk = 0; kk < 4; ++kk) for (int j = 0; j < 16; ++j) hB[kk * 16 + j] = (kk == 0) ? 1000.0 : 0;  // D[i][j] = 1000 i
    for (int i = 0; i < 16; ++i) { hA[i * 4 + 1] = 1; }
    for (int j = 0; j < 16; ++j) { hB[16 + j] = j; }                                                       // + j
    double *A, *B, *D;
    hipMalloc(&A, 512); hipMalloc(&B, 512); hipMalloc(&D, 2048);
    hipMemcpy(A, hA, 512, hipMemcpyHostToDevice); hipMemcpy(B, hB, 512, hipMemcpyHostToDevice);
    k<<<1, 64>>>(A, B, D);
    hipMemcpy(hD, D, 2048, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l += 1) {
        if (l % 16 > 2 && l % 16 < 15) continue;
        printf("lane %2d:", l);
        for (int r = 0; r < 4; ++r) { int v = (int)lrint(hD[l * 4 + r]); printf(" (%d,%d)", v / 1000, v % 1000); }
        printf("\n");
    }
    (void)ref;
    return 0;
}
