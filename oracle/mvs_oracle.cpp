// SPDX-License-Identifier: MIT
// TEST INFRASTRUCTURE ONLY (see oracle/README.md): CPU restatement of the
// image undistortion OpenMvsUtils::toOpenMVS runs before the openMVS export
// (util/OpenMvsUtils.cpp:142-150 -> ICamera::undistort, common/ICamera.cpp:72-80
// -> cv::undistort of OpenCV 4.5.1, an external dependency absent here).
//
// Restated from OpenCV's published scalar code paths, loop for loop:
//   cv::undistort           (imgproc/src/undistort.dispatch.cpp)  stripes of
//                            max(1, 4096/cols) rows, Ar(1,2) = v0 - y per stripe
//   initUndistortRectifyMap (same file + undistort.simd.hpp scalar tail)
//                            iR = (Ar*R)^-1 by cv::invert's 3x3 det/adjugate
//                            formulas, running sums _x += ir[0] ..., the
//                            rational/tangential/thin-prism/tilt model with the
//                            unused coefficients at 0, CV_16SC2 + CV_16UC1 maps
//                            (INTER_BITS = 5, cvRound = round half to even,
//                            INT_MIN when out of range as cvtsd2si does)
//   cv::remap INTER_LINEAR  (imgproc/src/imgwarp.cpp remapBilinear with
//                            FixedPtCast<int, uchar, 15>), BORDER_CONSTANT 0:
//                            the inlier fast path and the border path
//   initInterTab2D          bilinear table in float, saturate_cast<short>(v * 32768)
//                            (the (0,0) entry saturates to 32767; for 8-bit pixels
//                            (32767 v + 16384) >> 15 == v, so the sum fix-up that
//                            OpenCV applies to that entry cannot change a pixel and
//                            is not restated)
// Parity against OpenCV itself is unpinned (OpenCV is not available here); an
// AVX2-dispatched initUndistortRectifyMap sums _x in a different order and can
// differ from this scalar path by one 1/32-px map step where u*32 sits within
// an ulp of a half-integer.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

int cv_round(double v) {
    const double r = std::nearbyint(v);
    if (!(r >= -2147483648.0 && r <= 2147483647.0)) return INT_MIN;
    return (int)r;
}

// cv::invert, n == 3, CV_64F: det3 and the adjugate
bool invert3(const double* m, double* t) {
#define Sd(y, x) m[(y) * 3 + (x)]
    double d = Sd(0, 0) * (Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) - Sd(0, 1) * (Sd(1, 0) * Sd(2, 2) - Sd(1, 2) * Sd(2, 0)) +
               Sd(0, 2) * (Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0));
    if (d == 0.) { for (int i = 0; i < 9; ++i) t[i] = 0; return false; }
    d = 1. / d;
    t[0] = (Sd(1, 1) * Sd(2, 2) - Sd(1, 2) * Sd(2, 1)) * d;
    t[1] = (Sd(0, 2) * Sd(2, 1) - Sd(0, 1) * Sd(2, 2)) * d;
    t[2] = (Sd(0, 1) * Sd(1, 2) - Sd(0, 2) * Sd(1, 1)) * d;
    t[3] = (Sd(1, 2) * Sd(2, 0) - Sd(1, 0) * Sd(2, 2)) * d;
    t[4] = (Sd(0, 0) * Sd(2, 2) - Sd(0, 2) * Sd(2, 0)) * d;
    t[5] = (Sd(0, 2) * Sd(1, 0) - Sd(0, 0) * Sd(1, 2)) * d;
    t[6] = (Sd(1, 0) * Sd(2, 1) - Sd(1, 1) * Sd(2, 0)) * d;
    t[7] = (Sd(0, 1) * Sd(2, 0) - Sd(0, 0) * Sd(2, 1)) * d;
    t[8] = (Sd(0, 0) * Sd(1, 1) - Sd(0, 1) * Sd(1, 0)) * d;
#undef Sd
    return true;
}

void matmul3(const double* a, const double* b, double* c) {   // Mat_<double> * Mat_<double>
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += a[i * 3 + k] * b[k * 3 + j];
            c[i * 3 + j] = s;
        }
}

// initUndistortRectifyMap(A, dist, R = I, Ar, Size(W, rows), CV_16SC2, map1, map2)
void init_map(const double* A, const double* dist, const double* Ar, int W, int rows, int16_t* m1, uint16_t* m2) {
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double AR[9], ir[9];
    matmul3(Ar, I, AR);
    invert3(AR, ir);
    const double u0 = A[2], v0 = A[5], fx = A[0], fy = A[4];
    const double k1 = dist[0], k2 = dist[1], p1 = dist[2], p2 = dist[3], k3 = dist[4];
    const double k4 = 0, k5 = 0, k6 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0;
    const double matTilt[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int i = 0; i < rows; ++i) {
        int16_t* M1 = m1 + (size_t)i * W * 2;
        uint16_t* M2 = m2 + (size_t)i * W;
        double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
        for (int j = 0; j < W; ++j, _x += ir[0], _y += ir[3], _w += ir[6]) {
            double w = 1. / _w, x = _x * w, y = _y * w;
            double x2 = x * x, y2 = y * y;
            double r2 = x2 + y2, _2xy = 2 * x * y;
            double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            double xd = (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2);
            double yd = (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2);
            double vt[3];
            const double vin[3] = {xd, yd, 1};
            for (int a = 0; a < 3; ++a) {
                double s = 0;
                for (int k = 0; k < 3; ++k) s += matTilt[a * 3 + k] * vin[k];
                vt[a] = s;
            }
            double invProj = vt[2] ? 1. / vt[2] : 1;
            double u = fx * invProj * vt[0] + u0;
            double v = fy * invProj * vt[1] + v0;
            int iu = cv_round(u * 32);
            int iv = cv_round(v * 32);
            M1[j * 2] = (int16_t)(iu >> 5);
            M1[j * 2 + 1] = (int16_t)(iv >> 5);
            M2[j] = (uint16_t)((iv & 31) * 32 + (iu & 31));
        }
    }
}

struct Tab {
    int16_t w[32 * 32][4];
    Tab() {
        float t1[32][2];
        for (int i = 0; i < 32; ++i) {
            const float x = i * (1.f / 32);
            t1[i][0] = 1.f - x;
            t1[i][1] = x;
        }
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j)
                for (int k1 = 0; k1 < 2; ++k1)
                    for (int k2 = 0; k2 < 2; ++k2) {
                        const float v = t1[i][k1] * t1[j][k2];
                        const int r = (int)std::nearbyint(v * 32768.f);
                        w[i * 32 + j][k1 * 2 + k2] = (int16_t)std::min(std::max(r, -32768), 32767);
                    }
    }
};

uint8_t fixcast(int v) { v = (v + (1 << 14)) >> 15; return (uint8_t)std::min(std::max(v, 0), 255); }

int border_const(int p, int len) { return (p >= 0 && p < len) ? p : -1; }   // borderInterpolate, BORDER_CONSTANT

// remapBilinear<FixedPtCast<int, uchar, 15>, ..., short>, BORDER_CONSTANT, cval 0
void remap_rows(const uint8_t* S0, int64_t sstep, int W, int H, int cn, uint8_t* dst, int64_t dstep, int rows,
                const int16_t* m1, const uint16_t* m2) {
    static const Tab tab;
    const unsigned width1 = (unsigned)std::max(W - 1, 0), height1 = (unsigned)std::max(H - 1, 0);
    for (int dy = 0; dy < rows; ++dy) {
        uint8_t* D = dst + dy * dstep;
        const int16_t* XY = m1 + (size_t)dy * W * 2;
        const uint16_t* FXY = m2 + (size_t)dy * W;
        for (int dx = 0; dx < W; ++dx) {
            const int sx = XY[dx * 2], sy = XY[dx * 2 + 1];
            const int16_t* w = tab.w[FXY[dx]];
            uint8_t* d = D + dx * cn;
            if ((unsigned)sx < width1 && (unsigned)sy < height1) {
                const uint8_t* S = S0 + sy * sstep + sx * cn;
                for (int k = 0; k < cn; ++k)
                    d[k] = fixcast(S[k] * w[0] + S[k + cn] * w[1] + S[sstep + k] * w[2] + S[sstep + k + cn] * w[3]);
            } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
                for (int k = 0; k < cn; ++k) d[k] = 0;
            } else {
                const int sx0 = border_const(sx, W), sx1 = border_const(sx + 1, W);
                const int sy0 = border_const(sy, H), sy1 = border_const(sy + 1, H);
                for (int k = 0; k < cn; ++k) {
                    const int v0 = sx0 >= 0 && sy0 >= 0 ? S0[sy0 * sstep + sx0 * cn + k] : 0;
                    const int v1 = sx1 >= 0 && sy0 >= 0 ? S0[sy0 * sstep + sx1 * cn + k] : 0;
                    const int v2 = sx0 >= 0 && sy1 >= 0 ? S0[sy1 * sstep + sx0 * cn + k] : 0;
                    const int v3 = sx1 >= 0 && sy1 >= 0 ? S0[sy1 * sstep + sx1 * cn + k] : 0;
                    d[k] = fixcast(v0 * w[0] + v1 * w[1] + v2 * w[2] + v3 * w[3]);
                }
            }
        }
    }
}

}  // namespace

extern "C" {

// cv::undistort(src, dst, K, dist) for one W x H x cn 8-bit image, packed rows.
void orc_undistort(const uint8_t* src, uint8_t* dst, int W, int H, int cn, const double* K, const double* dist) {
    const int stripe0 = std::min(std::max(1, (1 << 12) / std::max(W, 1)), H);
    double A[9], Ar[9];
    std::memcpy(A, K, sizeof(A));
    std::memcpy(Ar, K, sizeof(Ar));
    const double v0 = Ar[5];
    std::vector<int16_t> m1((size_t)stripe0 * W * 2);
    std::vector<uint16_t> m2((size_t)stripe0 * W);
    const int64_t step = (int64_t)W * cn;
    for (int y = 0; y < H; y += stripe0) {
        const int rows = std::min(stripe0, H - y);
        Ar[5] = v0 - y;
        init_map(A, dist, Ar, W, rows, m1.data(), m2.data());
        remap_rows(src, step, W, H, cn, dst + y * step, step, rows, m1.data(), m2.data());
    }
}

// the same over a batch of images (OpenMP over images, as OpenMvsUtils.cpp:141)
void orc_undistort_batch(const uint8_t* const* src, uint8_t* const* dst, const int32_t* W, const int32_t* H,
                         const int32_t* cn, const double* K, const double* dist, int n, int nthreads) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int i = 0; i < n; ++i) orc_undistort(src[i], dst[i], W[i], H[i], cn[i], K + 9 * i, dist + 5 * i);
}

}  // extern "C"
