// SPDX-License-Identifier: MIT
// sfmx SIFT feature extraction for gfx950.
//
//   sfmx_sift_detect_compute   featureDetector->detect + descriptorExtractor->compute
//                              of SfM::extractFeatures (sfm/SfM.cpp:577-597) with
//                              cv::SIFT::create(featureLimit, 3, 0.09)
//                              (cli/PhotogrammetrieCli.cpp:354): OpenCV 4.5.1's
//                              SIFT::detectAndCompute, restated.
//
// Pipeline (one image, all on the device except the keypoint filter):
//   up2_kernel          u8 -> float, 2x INTER_LINEAR (horizontal then vertical taps)
//   blur_row/col        GaussianBlur: getGaussianKernel taps (host, double), row
//                       filter in tap order then the symmetric column filter,
//                       BORDER_REFLECT_101 -- base image and 5 layers per octave
//   half_nn_kernel      INTER_NEAREST half of layer 3 -> next octave
//   dog_kernel          DoG layers
//   extrema_kernel      26-neighbour extrema above floor(0.5 c / 3 * 255)
//   refine_kernel       adjustLocalExtrema (Cramer solve, <= 5 steps, contrast + edge)
//   orient_kernel       one wave per refined point: 36-bin orientation histogram,
//                       smoothing, 80 % peaks -> keypoints
//   host                removeDuplicatedSorted order, retainBest(nfeatures), 2x rescale
//   descriptor_kernel   one block per keypoint: 4x4x8 trilinear histogram,
//                       0.2 clamp, 512 / norm, saturate_cast<uchar>
// Float expressions follow oracle/sift_oracle.cpp operation for operation; the
// file is built with -ffp-contract=off.  exp / sin / cos are the fixed float
// formulas both sides share (sx_expf, sx_sincosf); histogram bins accumulate in
// 2^-30 fixed point with 64-bit LDS atomics, which makes the sums independent
// of the order the lanes add them.  Result: keypoints and descriptors
// bit-identical to the oracle.
#include <hip/hip_runtime.h>
#include "diag.hpp"
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sfmx_features.h"
#include "match_common.hpp"
#include "xcd.hpp"

namespace sfmx {
namespace sift {

constexpr int IMG_BORDER = 5, MAX_INTERP = 5, ORI_BINS = 36, DD = 4, NB = 8;
constexpr int HIST_LEN = (DD + 2) * (DD + 2) * (NB + 2);
constexpr float ORI_SIG = 1.5f, ORI_RADIUS = 3 * ORI_SIG, ORI_PEAK = 0.8f, DESCR_SCL = 3.f, DESCR_MAG_THR = 0.2f,
                INT_DESCR = 512.f, INIT_SIGMA = 0.5f;
constexpr double FIX = 1073741824.0;   // 2^30

struct Layer { float* p; int w, h; };
struct Cand { int o, layer, r, c; };
struct Refined { int o, layer, r, c; float x, y, size, response; int octave, _pad; };
struct Kp { float x, y, size, angle, response; int32_t octave, class_id; };
static_assert(sizeof(Kp) == sizeof(sfmx_keypoint), "cv::KeyPoint layout");

__host__ __device__ inline int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

__device__ __forceinline__ int round_f(float v) { return (int)rintf(v); }
__device__ __forceinline__ int round_d(double v) { return (int)rint(v); }

__device__ float sx_expf(float x) {
    if (!(x > -80.f)) return 0.f;
    if (x > 88.f) x = 88.f;
    const float k = rintf(x * 1.44269504088896341f);
    const float r = (x - k * 0.693145751953125f) - k * 1.42860682030941723e-6f;
    float p = 1.38888889e-3f;
    p = p * r + 8.33333333e-3f;
    p = p * r + 4.16666667e-2f;
    p = p * r + 1.66666667e-1f;
    p = p * r + 0.5f;
    p = p * r + 1.0f;
    p = p * r + 1.0f;
    return ldexpf(p, (int)k);
}

__device__ void sx_sincosf(float a, float* s, float* c) {
    const float q = rintf(a * 0.636619772367581343f);
    const float r = (a - q * 1.5703125f) - q * 4.83826794897e-4f;
    const float r2 = r * r;
    float sp = -1.9515295891e-4f;
    sp = sp * r2 + 8.3321608736e-3f;
    sp = sp * r2 - 1.6666654611e-1f;
    const float sr = r + r * (r2 * sp);
    float cp = 2.443315711809948e-5f;
    cp = cp * r2 - 1.388731625493765e-3f;
    cp = cp * r2 + 4.166664568298827e-2f;
    const float cr = (1.f - 0.5f * r2) + (r2 * r2) * cp;
    switch (((int)q) & 3) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
    }
}

__device__ float atan2_deg(float y, float x) {   // cv::fastAtan2
    constexpr float R2D = (float)(180 / 3.14159265358979323846);
    constexpr float P1 = 0.9997878412794807f * R2D, P3 = -0.3258083974640975f * R2D, P5 = 0.1555786518463281f * R2D,
                    P7 = -0.04432655554792128f * R2D;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((P7 * c2 + P5) * c2 + P3) * c2 + P1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((P7 * c2 + P5) * c2 + P3) * c2 + P1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

__device__ __forceinline__ long long fixp(float v) { return (long long)(v * 1073741824.f); }

// ------------------------------------------------------------------ pyramid
__device__ __forceinline__ void lin_coef(int d, int ssize, int& s, float& f0, float& f1) {
    float fx = (float)((d + 0.5) * 0.5 - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx >= ssize - 1) { fx = 0; sx = ssize - 1; }
    s = sx;
    f0 = 1.f - fx;
    f1 = fx;
}

__global__ void up2_kernel(const uint8_t* __restrict__ img, int W, int H, int64_t pitch, float* __restrict__ dst) {
    const int X = blockIdx.x * blockDim.x + threadIdx.x, Y = blockIdx.y;
    if (X >= 2 * W) return;
    int sy, sx;
    float b0, b1, a0, a1;
    lin_coef(Y, H, sy, b0, b1);
    lin_coef(X, W, sx, a0, a1);
    const int sy1 = min(sy + 1, H - 1), sx1 = min(sx + 1, W - 1);
    const float h0 = (float)img[sy * pitch + sx] * a0 + (float)img[sy * pitch + sx1] * a1;
    const float h1 = (float)img[sy1 * pitch + sx] * a0 + (float)img[sy1 * pitch + sx1] * a1;
    dst[(int64_t)Y * (2 * W) + X] = h0 * b0 + h1 * b1;
}

// img.convertTo(CV_32F) of createInitialImage's un-doubled branch (compute() with firstOctave = 0)
__global__ void to_float_kernel(const uint8_t* __restrict__ img, int W, int H, int64_t pitch, float* __restrict__ dst) {
    const int X = blockIdx.x * blockDim.x + threadIdx.x, Y = blockIdx.y;
    if (X >= W) return;
    dst[(int64_t)Y * W + X] = (float)img[Y * pitch + X];
}

__global__ void blur_row_kernel(const float* __restrict__ src, float* __restrict__ dst, int w, int h,
                                const float* __restrict__ f, int n) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= w) return;
    const int r = n / 2;
    const float* row = src + (int64_t)y * w;
    float s = f[0] * row[reflect101(x - r, w)];
    for (int k = 1; k < n; ++k) s += f[k] * row[reflect101(x - r + k, w)];
    dst[(int64_t)y * w + x] = s;
}

__global__ void blur_col_kernel(const float* __restrict__ src, float* __restrict__ dst, int w, int h,
                                const float* __restrict__ f, int n) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= w) return;
    const int r = n / 2;
    float s = f[r] * src[(int64_t)y * w + x];
    for (int k = 1; k <= r; ++k)
        s += f[r + k] * (src[(int64_t)reflect101(y + k, h) * w + x] + src[(int64_t)reflect101(y - k, h) * w + x]);
    dst[(int64_t)y * w + x] = s;
}

// Fused separable blur on a TX x TY output tile: the reflected source halo is
// staged in LDS once, the row filter runs into LDS (taps in order, as
// blur_row_kernel), then the symmetric column filter (as blur_col_kernel) --
// the same operations on the same values, so the result equals the two-pass
// kernels bit for bit.  With `dog` set it also writes the DoG layer
// dst - src at each pixel (src is the previous pyramid layer).
constexpr int TX = 64, TY = 32, RMAX = 16;
__global__ __launch_bounds__(256)
void blur_tile_kernel(const float* __restrict__ src, float* __restrict__ dst, float* __restrict__ dog, int w, int h,
                      const float* __restrict__ fk, int n, int xcd) {
    __shared__ float in[(TY + 2 * RMAX) * (TX + 2 * RMAX)];
    __shared__ float rowf[(TY + 2 * RMAX) * TX];
    __shared__ float f[2 * RMAX + 1];
    const int r = n / 2;
    int bx, by, bz;
    xcd_grid(xcd, bx, by, bz);
    const int x0 = bx * TX, y0 = by * TY;
    const int IW = TX + 2 * r, IH = TY + 2 * r;
    if (threadIdx.x < n) f[threadIdx.x] = fk[threadIdx.x];
    for (int q = threadIdx.x; q < IW * IH; q += 256) {
        const int iy = q / IW, ix = q % IW;
        const int sy = reflect101(y0 - r + iy, h), sx = reflect101(x0 - r + ix, w);
        in[iy * IW + ix] = src[(int64_t)sy * w + sx];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < IH * TX; q += 256) {
        const int iy = q / TX, x = q % TX;
        const float* row = in + iy * IW + x;
        float s = f[0] * row[0];
        for (int k = 1; k < n; ++k) s += f[k] * row[k];
        rowf[iy * TX + x] = s;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < TY * TX; q += 256) {
        const int ty = q / TX, x = q % TX;
        const int gx = x0 + x, gy = y0 + ty;
        if (gx >= w || gy >= h) continue;
        const float* col = rowf + (ty + r) * TX + x;
        float s = f[r] * col[0];
        for (int k = 1; k <= r; ++k) s += f[r + k] * (col[k * TX] + col[-k * TX]);
        dst[(int64_t)gy * w + gx] = s;
        if (dog) dog[(int64_t)gy * w + gx] = s - in[(ty + r) * IW + x + r];
    }
}

// blur_tile_kernel specialised on the tap count N (the reference setting uses
// N = 11, 13, 17, 21, 27) with 4 outputs per thread in both passes: the row
// pass slides an (N + 3)-value window through registers, the column pass a
// (2r + 4)-value one, giving 4 independent chains per thread.  Every output is
// still the same sequence of float operations as blur_row/col_kernel.
template <int N>
__global__ __launch_bounds__(256)
void blur_tile_n_kernel(const float* __restrict__ src, float* __restrict__ dst, float* __restrict__ dog, int w, int h,
                        const float* __restrict__ fk, int xcd) {
    constexpr int R = N / 2, IW = TX + 2 * R, IH = TY + 2 * R;
    __shared__ float in[IH * IW];
    __shared__ float rowf[IH * TX];
    int bx, by, bz;
    xcd_grid(xcd, bx, by, bz);
    const int x0 = bx * TX, y0 = by * TY;
    float f[N];
#pragma unroll
    for (int k = 0; k < N; ++k) f[k] = fk[k];
    for (int q = threadIdx.x; q < IW * IH; q += 256) {
        const int iy = q / IW, ix = q % IW;
        const int sy = reflect101(y0 - R + iy, h), sx = reflect101(x0 - R + ix, w);
        in[iy * IW + ix] = src[(int64_t)sy * w + sx];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < IH * (TX / 4); q += 256) {   // row pass: 4 consecutive x per thread
        const int iy = q / (TX / 4), x = (q % (TX / 4)) * 4;
        const float* row = in + iy * IW + x;
        float v[N + 3];
#pragma unroll
        for (int t = 0; t < N + 3; ++t) v[t] = row[t];
        float s[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] = f[0] * v[j];
#pragma unroll
        for (int k = 1; k < N; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) s[j] += f[k] * v[j + k];
#pragma unroll
        for (int j = 0; j < 4; ++j) rowf[iy * TX + x + j] = s[j];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < (TY / 4) * TX; q += 256) {   // column pass: 4 consecutive y per thread
        const int ty = (q / TX) * 4, x = q % TX;
        const float* col = rowf + ty * TX + x;                  // rowf row ty holds source row ty - R
        float c[2 * R + 4];
#pragma unroll
        for (int t = 0; t < 2 * R + 4; ++t) c[t] = col[t * TX];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gx = x0 + x, gy = y0 + ty + j;
            float a = f[R] * c[j + R];
#pragma unroll
            for (int k = 1; k <= R; ++k) a += f[R + k] * (c[j + R + k] + c[j + R - k]);
            if (gx < w && gy < h) {
                dst[(int64_t)gy * w + gx] = a;
                if (dog) dog[(int64_t)gy * w + gx] = a - in[(ty + j + R) * IW + x + R];
            }
        }
    }
}

// The small octaves of one image in ONE workgroup (1024 threads): octaves o_s .. nOct - 1 (each of
// at most SMALL_PX pixels), in order: INTER_NEAREST half of the previous octave's layer L, then per
// layer the row filter (taps in order, as blur_row_kernel) into `rf`, the symmetric column filter
// (as blur_col_kernel) into the layer and its DoG against the previous layer, then the octave's
// 26-neighbour extrema (as extrema_kernel).  The same operations on the same values as the
// per-octave launches (tile blur, half_nn_kernel, extrema_kernel), so every layer, DoG and candidate
// is bit-identical; ~7 launches per small octave become one launch for all of them.  Everything goes
// through global memory (L1/L2-resident at these sizes); __syncthreads orders the passes.
constexpr int SMALL_PX = 2048, SMALL_MAXL = 8;   // r02q sweep: 512 / 2048 +3 %, 8192 -7 %, 32768 -40 %
struct SmallTaps { const float* p[SMALL_MAXL]; int n[SMALL_MAXL]; };
__global__ __launch_bounds__(1024)
void small_octaves_kernel(const Layer* __restrict__ gp, const Layer* __restrict__ dog, int L, int o_s, int nOct,
                          SmallTaps taps, float* __restrict__ rf, int threshold, Cand* __restrict__ out,
                          int* __restrict__ count, int cap) {
    const int tid = threadIdx.x;
    for (int o = o_s; o < nOct; ++o) {
        const Layer base = gp[o * (L + 3)];
        const int w = base.w, h = base.h, npx = w * h;
        {   // layer 0: INTER_NEAREST half of the previous octave's layer L
            const Layer src = gp[(o - 1) * (L + 3) + L];
            const double ifx = 1. / ((double)w / src.w), ify = 1. / ((double)h / src.h);
            for (int e = tid; e < npx; e += 1024) {
                const int y = e / w, x = e % w;
                const int sy = min((int)floor(y * ify), src.h - 1), sx = min((int)floor(x * ifx), src.w - 1);
                base.p[e] = src.p[(int64_t)sy * src.w + sx];
            }
        }
        __syncthreads();
        for (int i = 1; i < L + 3; ++i) {
            const float* src = gp[o * (L + 3) + i - 1].p;
            float* dst = gp[o * (L + 3) + i].p;
            float* dg = dog[o * (L + 2) + i - 1].p;
            const float* f = taps.p[i];
            const int n = taps.n[i], r = n / 2;
            for (int e = tid; e < npx; e += 1024) {   // row filter
                const int y = e / w, x = e % w;
                const float* row = src + (int64_t)y * w;
                float sm = f[0] * row[reflect101(x - r, w)];
                for (int k = 1; k < n; ++k) sm += f[k] * row[reflect101(x - r + k, w)];
                rf[e] = sm;
            }
            __syncthreads();
            for (int e = tid; e < npx; e += 1024) {   // column filter + DoG
                const int y = e / w, x = e % w;
                float sm = f[r] * rf[e];
                for (int k = 1; k <= r; ++k)
                    sm += f[r + k] * (rf[(int64_t)reflect101(y + k, h) * w + x] + rf[(int64_t)reflect101(y - k, h) * w + x]);
                dst[e] = sm;
                dg[e] = sm - src[e];
            }
            __syncthreads();
        }
        if (w > 2 * IMG_BORDER && h > 2 * IMG_BORDER) {   // extrema of layers 1 .. L
            const int iw = w - 2 * IMG_BORDER, ih = h - 2 * IMG_BORDER, m = iw * ih;
            for (int e = tid; e < L * m; e += 1024) {
                const int layer = 1 + e / m, q0 = e % m, rr = q0 / iw + IMG_BORDER, c = q0 % iw + IMG_BORDER;
                const float* prev = dog[o * (L + 2) + layer - 1].p;
                const float* img = dog[o * (L + 2) + layer].p;
                const float* next = dog[o * (L + 2) + layer + 1].p;
                const float val = img[(int64_t)rr * w + c];
                if (!(fabsf(val) > threshold)) continue;
                bool mx = val > 0, mn = val < 0;
#pragma unroll
                for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                    for (int dx = -1; dx <= 1; ++dx) {
                        const int64_t q = (int64_t)(rr + dy) * w + c + dx;
                        const float a = img[q], b = prev[q], ee = next[q];
                        mx = mx && val >= a && val >= b && val >= ee;
                        mn = mn && val <= a && val <= b && val <= ee;
                    }
                if (!mx && !mn) continue;
                const int slot = atomicAdd(count, 1);
                if (slot < cap) out[slot] = Cand{o, layer, rr, c};
            }
        }
        __syncthreads();   // the next octave halves this octave's layer L
    }
}

inline bool small_octaves_on() {   // SFMX_SIFT_SMALL=0: every octave as per-octave launches (A/B, tests)
    const char* e = SFMX_DIAG_ENV("SFMX_SIFT_SMALL");
    return !(e && e[0] == '0');
}
inline int small_px() {   // SFMX_SIFT_SMALL_PX: the largest octave (pixels) the fused launch takes (tuning)
    const char* e = SFMX_DIAG_ENV("SFMX_SIFT_SMALL_PX");
    return e ? std::atoi(e) : SMALL_PX;
}

__global__ void half_nn_kernel(const float* __restrict__ src, int sw, int sh, float* __restrict__ dst, int dw, int dh,
                               double ifx, double ify) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= dw) return;
    const int sy = min((int)floor(y * ify), sh - 1), sx = min((int)floor(x * ifx), sw - 1);
    dst[(int64_t)y * dw + x] = src[(int64_t)sy * sw + sx];
}

__global__ void dog_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ d, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = b[i] - a[i];
}

// ------------------------------------------------------------------ detection
// One launch per octave: blockIdx.z picks the inner DoG layer 1 + z of dog[o * (L + 2) ..],
// so a small octave's three scans fill the chip together.  Candidate slots come from
// one atomic counter in any order; the host filter sorts them (as before).
// r05: each thread scans `rows` (<= EX_ROWS) rows of its column, their values loaded together: one row
// per workgroup (r01-r04) made the octave-0 launch ~97k short workgroups (51.7 us per 1080p image on
// one stream; 8 rows: 40.9 us, r05zh), while the smaller octaves run faster with one row (their launches
// have few workgroups, r05zh: 8 rows made octave 1 24.3 -> 27.4 us).
constexpr int EX_ROWS = 8;
__global__ void extrema_kernel(const Layer* __restrict__ dog, int L, int w, int h, int threshold, int o,
                               Cand* __restrict__ out, int* __restrict__ count, int cap, int xcd, int rows) {
    int bx, by, bz;
    xcd_grid(xcd, bx, by, bz);
    const int c = bx * blockDim.x + threadIdx.x + IMG_BORDER, r0 = by * rows + IMG_BORDER;
    if (c >= w - IMG_BORDER || r0 >= h - IMG_BORDER) return;
    const int layer = 1 + bz;
    const float* __restrict__ prev = dog[o * (L + 2) + layer - 1].p;
    const float* __restrict__ img = dog[o * (L + 2) + layer].p;
    const float* __restrict__ next = dog[o * (L + 2) + layer + 1].p;
    const int nr = min(rows, h - IMG_BORDER - r0);
    float vals[EX_ROWS];
#pragma unroll
    for (int k = 0; k < EX_ROWS; ++k) vals[k] = k < nr ? img[(int64_t)(r0 + k) * w + c] : 0.f;
#pragma unroll
    for (int k = 0; k < EX_ROWS; ++k) {
        const float val = vals[k];
        if (k >= nr || !(fabsf(val) > threshold)) continue;
        const int r = r0 + k;
        bool mx = val > 0, mn = val < 0;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const int64_t q = (int64_t)(r + dy) * w + c + dx;
                const float a = img[q], b = prev[q], e = next[q];
                mx = mx && val >= a && val >= b && val >= e;
                mn = mn && val <= a && val <= b && val <= e;
            }
        if (!mx && !mn) continue;
        const int slot = atomicAdd(count, 1);
        if (slot < cap) out[slot] = Cand{o, layer, r, c};
    }
}

__device__ __forceinline__ float at(const Layer& L, int r, int c) { return L.p[(int64_t)r * L.w + c]; }

// adjustLocalExtrema; dog[o * (L + 2) + i]
__global__ void refine_kernel(const Cand* __restrict__ cands, const int* __restrict__ ncand_p, int cap,
                              const Layer* __restrict__ dog, int L, float contrastThreshold, float edgeThreshold,
                              float sigma, Refined* __restrict__ out, int* __restrict__ count, int out_cap) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= min(*ncand_p, cap)) return;
    const Cand cd = cands[t];
    const int octv = cd.o;
    int layer = cd.layer, r = cd.r, c = cd.c;
    const float img_scale = 1.f / 255, deriv_scale = img_scale * 0.5f, second_deriv_scale = img_scale,
                cross_deriv_scale = img_scale * 0.25f;
    float xi = 0, xr = 0, xc = 0, contr = 0;
    int i = 0;
    for (; i < MAX_INTERP; i++) {
        const int idx = octv * (L + 2) + layer;
        const Layer img = dog[idx], prev = dog[idx - 1], next = dog[idx + 1];
        const float d0 = (at(img, r, c + 1) - at(img, r, c - 1)) * deriv_scale;
        const float d1 = (at(img, r + 1, c) - at(img, r - 1, c)) * deriv_scale;
        const float d2 = (at(next, r, c) - at(prev, r, c)) * deriv_scale;
        const float v2 = at(img, r, c) * 2;
        const float dxx = (at(img, r, c + 1) + at(img, r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (at(img, r + 1, c) + at(img, r - 1, c) - v2) * second_deriv_scale;
        const float dss = (at(next, r, c) + at(prev, r, c) - v2) * second_deriv_scale;
        const float dxy = (at(img, r + 1, c + 1) - at(img, r + 1, c - 1) - at(img, r - 1, c + 1) + at(img, r - 1, c - 1)) *
                          cross_deriv_scale;
        const float dxs = (at(next, r, c + 1) - at(next, r, c - 1) - at(prev, r, c + 1) + at(prev, r, c - 1)) *
                          cross_deriv_scale;
        const float dys = (at(next, r + 1, c) - at(next, r - 1, c) - at(prev, r + 1, c) + at(prev, r - 1, c)) *
                          cross_deriv_scale;
        const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs, a21 = dys, a22 = dss;
        float x0 = 0, x1 = 0, x2 = 0;
        float det = a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
        if (det != 0) {
            det = 1 / det;
            x0 = det * (d0 * (a11 * a22 - a12 * a21) - a01 * (d1 * a22 - a12 * d2) + a02 * (d1 * a21 - a11 * d2));
            x1 = det * (a00 * (d1 * a22 - a12 * d2) - d0 * (a10 * a22 - a12 * a20) + a02 * (a10 * d2 - d1 * a20));
            x2 = det * (a00 * (a11 * d2 - d1 * a21) - a01 * (a10 * d2 - d1 * a20) + d0 * (a10 * a21 - a11 * a20));
        }
        xi = -x2; xr = -x1; xc = -x0;
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) || fabsf(xc) > (float)(INT_MAX / 3)) return;
        c += round_f(xc);
        r += round_f(xr);
        layer += round_f(xi);
        if (layer < 1 || layer > L || c < IMG_BORDER || c >= img.w - IMG_BORDER || r < IMG_BORDER || r >= img.h - IMG_BORDER)
            return;
    }
    if (i >= MAX_INTERP) return;
    const int idx = octv * (L + 2) + layer;
    const Layer img = dog[idx], prev = dog[idx - 1], next = dog[idx + 1];
    {
        const float d0 = (at(img, r, c + 1) - at(img, r, c - 1)) * deriv_scale;
        const float d1 = (at(img, r + 1, c) - at(img, r - 1, c)) * deriv_scale;
        const float d2 = (at(next, r, c) - at(prev, r, c)) * deriv_scale;
        float tt = 0;
        tt += d0 * xc;
        tt += d1 * xr;
        tt += d2 * xi;
        contr = at(img, r, c) * img_scale + tt * 0.5f;
        if (fabsf(contr) * L < contrastThreshold) return;
        const float v2 = at(img, r, c) * 2.f;
        const float dxx = (at(img, r, c + 1) + at(img, r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (at(img, r + 1, c) + at(img, r - 1, c) - v2) * second_deriv_scale;
        const float dxy = (at(img, r + 1, c + 1) - at(img, r + 1, c - 1) - at(img, r - 1, c + 1) + at(img, r - 1, c - 1)) *
                          cross_deriv_scale;
        const float tr = dxx + dyy;
        const float det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * edgeThreshold >= (edgeThreshold + 1) * (edgeThreshold + 1) * det) return;
    }
    Refined R;
    R.o = octv; R.layer = layer; R.r = r; R.c = c;
    R.x = (c + xc) * (1 << octv);
    R.y = (r + xr) * (1 << octv);
    R.octave = octv + (layer << 8) + (round_d((xi + 0.5) * 255) << 16);
    R.size = sigma * sx_expf(((layer + xi) / L) * 0.693147180559945309f) * (1 << octv) * 2;
    R.response = fabsf(contr);
    R._pad = 0;
    const int slot = atomicAdd(count, 1);
    if (slot < out_cap) out[slot] = R;
}

// calcOrientationHist + peak emission; one wave per refined point
__global__ __launch_bounds__(64)
void orient_kernel(const Refined* __restrict__ refs, const int* __restrict__ nref_p, int cap,
                   const Layer* __restrict__ gp, int L, Kp* __restrict__ out, int* __restrict__ count, int out_cap) {
    __shared__ unsigned long long acc[ORI_BINS];
    const int t = blockIdx.x;
    if (t >= min(*nref_p, cap)) return;
    const Refined R = refs[t];
    const Layer img = gp[R.o * (L + 3) + R.layer];
    const float scl_octv = R.size * 0.5f / (1 << R.o);
    const int radius = round_f(ORI_RADIUS * scl_octv);
    const float sigma = ORI_SIG * scl_octv;
    const float expf_scale = -1.f / (2.f * sigma * sigma);
    const int n = ORI_BINS;
    for (int b = threadIdx.x; b < n; b += 64) acc[b] = 0;
    __syncthreads();
    const int side = 2 * radius + 1;
    for (int q = threadIdx.x; q < side * side; q += 64) {
        const int i = q / side - radius, j = q % side - radius;
        const int y = R.r + i, x = R.c + j;
        if (y <= 0 || y >= img.h - 1 || x <= 0 || x >= img.w - 1) continue;
        const float dx = at(img, y, x + 1) - at(img, y, x - 1);
        const float dy = at(img, y - 1, x) - at(img, y + 1, x);
        const float w = sx_expf((i * i + j * j) * expf_scale);
        const float ori = atan2_deg(dy, dx);
        const float mag = sqrtf(dx * dx + dy * dy);
        int bin = round_f((n / 360.f) * ori);
        if (bin >= n) bin -= n;
        if (bin < 0) bin += n;
        atomicAdd(&acc[bin], (unsigned long long)fixp(w * mag));
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    float t_[ORI_BINS + 4];
    float* temphist = t_ + 2;
    float hist[ORI_BINS];
    for (int b = 0; b < n; ++b) temphist[b] = (float)((double)(long long)acc[b] * (1.0 / FIX));
    temphist[-1] = temphist[n - 1];
    temphist[-2] = temphist[n - 2];
    temphist[n] = temphist[0];
    temphist[n + 1] = temphist[1];
    for (int b = 0; b < n; b++)
        hist[b] = (temphist[b - 2] + temphist[b + 2]) * (1.f / 16.f) + (temphist[b - 1] + temphist[b + 1]) * (4.f / 16.f) +
                  temphist[b] * (6.f / 16.f);
    float omax = hist[0];
    for (int b = 1; b < n; b++) omax = fmaxf(omax, hist[b]);
    const float mag_thr = omax * ORI_PEAK;
    for (int j = 0; j < n; j++) {
        const int l = j > 0 ? j - 1 : n - 1, r2 = j < n - 1 ? j + 1 : 0;
        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
            float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
            bin = bin < 0 ? n + bin : bin >= n ? bin - n : bin;
            Kp k;
            k.x = R.x; k.y = R.y; k.size = R.size; k.response = R.response; k.octave = R.octave; k.class_id = -1;
            k.angle = 360.f - (float)((360.f / n) * bin);
            if (fabsf(k.angle - 360.f) < FLT_EPSILON) k.angle = 0.f;
            const int slot = atomicAdd(count, 1);
            if (slot < out_cap) out[slot] = k;
        }
    }
}

// calcSIFTDescriptor; one block per (final, rescaled) keypoint
constexpr int DESC_THREADS = 256;
__global__ __launch_bounds__(DESC_THREADS)
void descriptor_kernel(const Kp* __restrict__ kps, int nkp, const Layer* __restrict__ gp, int L, int firstOctave,
                       float* __restrict__ desc) {
    __shared__ unsigned long long hist[HIST_LEN];
    __shared__ float dst[DD * DD * NB];
    const int q = blockIdx.x;
    if (q >= nkp) return;
    const Kp kp = kps[q];
    int octave = kp.octave & 255;
    const int layer = (kp.octave >> 8) & 255;
    octave = octave < 128 ? octave : (-128 | octave);
    const float scale = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
    const float size = kp.size * scale;
    const float ptx = kp.x * scale, pty = kp.y * scale;
    const Layer img = gp[(octave - firstOctave) * (L + 3) + layer];
    float ori = 360.f - kp.angle;
    if (fabsf(ori - 360.f) < FLT_EPSILON) ori = 0.f;
    const float scl = size * 0.5f;
    const int d = DD, n = NB;
    const int ptX = round_f(ptx), ptY = round_f(pty);
    float sin_t, cos_t;
    sx_sincosf(ori * (float)(3.14159265358979323846 / 180), &sin_t, &cos_t);
    const float bins_per_rad = n / 360.f;
    const float exp_scale = -1.f / (d * d * 0.5f);
    const float hist_width = DESCR_SCL * scl;
    int radius = round_f(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
    radius = min(radius, (int)sqrt(((double)img.w) * img.w + ((double)img.h) * img.h));
    cos_t /= hist_width;
    sin_t /= hist_width;
    for (int b = threadIdx.x; b < HIST_LEN; b += DESC_THREADS) hist[b] = 0;
    __syncthreads();
    const int side = 2 * radius + 1;
    for (int k = threadIdx.x; k < side * side; k += DESC_THREADS) {
        const int i = k / side - radius, j = k % side - radius;
        const float c_rot = j * cos_t - i * sin_t;
        const float r_rot = j * sin_t + i * cos_t;
        float rbin = r_rot + d / 2 - 0.5f;
        float cbin = c_rot + d / 2 - 0.5f;
        const int r = ptY + i, c = ptX + j;
        if (!(rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < img.h - 1 && c > 0 && c < img.w - 1)) continue;
        const float dx = at(img, r, c + 1) - at(img, r, c - 1);
        const float dy = at(img, r - 1, c) - at(img, r + 1, c);
        const float w = sx_expf((c_rot * c_rot + r_rot * r_rot) * exp_scale);
        const float o = atan2_deg(dy, dx);
        const float m = sqrtf(dx * dx + dy * dy);
        float obin = (o - ori) * bins_per_rad;
        const float mag = m * w;
        const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
        int o0 = (int)floorf(obin);
        rbin -= r0;
        cbin -= c0;
        obin -= o0;
        if (o0 < 0) o0 += n;
        if (o0 >= n) o0 -= n;
        const float v_r1 = mag * rbin, v_r0 = mag - v_r1;
        const float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
        const float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
        const float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
        const float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
        const float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
        const float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
        const int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
        atomicAdd(&hist[idx], (unsigned long long)fixp(v_rco000));
        atomicAdd(&hist[idx + 1], (unsigned long long)fixp(v_rco001));
        atomicAdd(&hist[idx + (n + 2)], (unsigned long long)fixp(v_rco010));
        atomicAdd(&hist[idx + (n + 3)], (unsigned long long)fixp(v_rco011));
        atomicAdd(&hist[idx + (d + 2) * (n + 2)], (unsigned long long)fixp(v_rco100));
        atomicAdd(&hist[idx + (d + 2) * (n + 2) + 1], (unsigned long long)fixp(v_rco101));
        atomicAdd(&hist[idx + (d + 3) * (n + 2)], (unsigned long long)fixp(v_rco110));
        atomicAdd(&hist[idx + (d + 3) * (n + 2) + 1], (unsigned long long)fixp(v_rco111));
    }
    __syncthreads();
    if (threadIdx.x < d * d) {   // circular fold of each cell's orientation bins
        const int i = threadIdx.x / d, j = threadIdx.x % d;
        const int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
        const long long h0 = (long long)hist[idx] + (long long)hist[idx + n];
        const long long h1 = (long long)hist[idx + 1] + (long long)hist[idx + n + 1];
        for (int k = 0; k < n; k++) {
            const long long v = k == 0 ? h0 : (k == 1 ? h1 : (long long)hist[idx + k]);
            dst[(i * d + j) * n + k] = (float)((double)v * (1.0 / FIX));
        }
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    const int len = d * d * n;
    float nrm2 = 0;
    for (int k = 0; k < len; k++) nrm2 += dst[k] * dst[k];
    const float thr = sqrtf(nrm2) * DESCR_MAG_THR;
    nrm2 = 0;
    for (int k = 0; k < len; k++) {
        const float val = fminf(dst[k], thr);
        dst[k] = val;
        nrm2 += val * val;
    }
    nrm2 = INT_DESCR / fmaxf(sqrtf(nrm2), FLT_EPSILON);
    float* out = desc + (int64_t)q * 128;
    for (int k = 0; k < len; k++) out[k] = (float)min(max(round_f(dst[k] * nrm2), 0), 255);
}

// ------------------------------------------------------------------ host
static int host_round(double v) { return (int)std::nearbyint(v); }

std::vector<float> gauss_kernel(double sigma) {   // getGaussianKernel(cvRound(8 sigma + 1) | 1, sigma, CV_32F)
    const int n = host_round(sigma * 4 * 2 + 1) | 1;
    std::vector<float> cf(n);
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < n; i++) {
        const double x = i - (n - 1) * 0.5;
        const double t = std::exp(scale2X * x * x);
        cf[i] = (float)t;
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; i++) cf[i] = (float)(cf[i] * sum);
    return cf;
}

static bool kp_less(const Kp& a, const Kp& b) {   // KeyPointsFilter::removeDuplicatedSorted's order
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle < b.angle;
    if (a.response != b.response) return a.response > b.response;
    if (a.octave != b.octave) return a.octave > b.octave;
    return a.class_id > b.class_id;
}

// removeDuplicatedSorted + retainBest + firstOctave = -1 rescale
static void filter_keypoints(std::vector<Kp>& kps, int nfeatures) {
    std::sort(kps.begin(), kps.end(), kp_less);
    if (kps.size() > 1) {
        size_t w = 0;
        for (size_t j = 1; j < kps.size(); ++j) {
            const Kp &a = kps[w], &b = kps[j];
            if (a.x != b.x || a.y != b.y || a.size != b.size || a.angle != b.angle) kps[++w] = kps[j];
        }
        kps.resize(w + 1);
    }
    // KeyPointsFilter::retainBest (OpenCV 4.5.1): nth_element on the keypoint vector itself with
    // KeypointResponseGreater, then std::partition of the tail by response >= the boundary response. Both
    // reorder the kept keypoints in place (libstdc++ algorithms, as OpenCV's build), and descriptor rows follow.
    if (nfeatures > 0 && (int)kps.size() > nfeatures) {
        std::nth_element(kps.begin(), kps.begin() + nfeatures - 1, kps.end(),
                         [](const Kp& a, const Kp& b) { return a.response > b.response; });
        const float amb = kps[nfeatures - 1].response;
        auto new_end = std::partition(kps.begin() + nfeatures, kps.end(), [amb](const Kp& q) { return q.response >= amb; });
        kps.resize(new_end - kps.begin());
    }
    for (Kp& q : kps) {
        q.octave = (q.octave & ~255) | ((q.octave - 1) & 255);
        q.x *= 0.5f;
        q.y *= 0.5f;
        q.size *= 0.5f;
    }
}

thread_local float g_last_ms = -1.f;

struct Arena {                 // per-thread device scratch, grown on demand
    int dev = -1;
    char* p = nullptr;
    size_t cap = 0, used = 0;
    bool overflow = false;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    void release() {   // frees on the device the arena was made for
        if (dev < 0) return;
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev);
        if (p) (void)hipFree(p);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (prev >= 0) (void)hipSetDevice(prev);
        p = nullptr; cap = 0; e0 = e1 = nullptr; dev = -1;
    }
    bool reserve(int device, size_t bytes) {
        if (dev != device) {
            release();
            (void)hipSetDevice(device);
            dev = device;
        }
        used = 0;
        overflow = false;
        if (bytes > cap) {
            if (p) (void)hipFree(p);
            p = nullptr;
            cap = 0;
            if (hipMalloc(&p, bytes) != hipSuccess) return false;
            cap = bytes;
        }
        if (!e0 && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) return false;
        return true;
    }
    template <class T> T* take(size_t n) {   // callers check `overflow` before the first launch
        T* r = reinterpret_cast<T*>(p + used);
        used += (sizeof(T) * n + 255) & ~(size_t)255;
        if (used > cap) overflow = true;
        return r;
    }
};
thread_local Arena g_arena;

bool is_gfx950(int device) {
    static std::atomic<int> state[64];
    if (device < 0 || device >= 64) return false;
    int v = state[device].load();
    if (v == 0) {
        hipDeviceProp_t prop;
        v = (hipGetDeviceProperties(&prop, device) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) ? 1 : 2;
        state[device].store(v);
    }
    return v == 1;
}

}  // namespace sift
}  // namespace sfmx

using namespace sfmx;
using namespace sfmx::sift;

#define FCHK(expr) do { if ((expr) != hipSuccess) { rc = SFMX_EDEVICE; set_last_error("HIP error in " #expr); goto done; } } while (0)

extern "C" {

void sfmx_sift_default_params(sfmx_sift_params* p) {
    if (!p) return;
    p->nfeatures = 0;
    p->n_octave_layers = 3;
    p->contrast_threshold = 0.09;
    p->edge_threshold = 10;
    p->sigma = 1.6;
}

float sfmx_sift_last_kernel_ms(void) { return g_last_ms; }

}  // extern "C"

namespace {

// One image through the whole pipeline on `stream`, scratch from `arena`;
// *last_ms = device time of the kernels (HIP events on the stream).
int detect_compute_impl(const uint8_t* image, int32_t width, int32_t height, int64_t pitch,
                        const sfmx_sift_params* params, int32_t inputs_on_device, int32_t device, void* stream,
                        sfmx_keypoint* keypoints, float* descriptors, int32_t capacity, int32_t* n_keypoints,
                        Arena& arena, float* last_ms) {
    if (!image || !params || !n_keypoints || capacity < 0 || (capacity > 0 && !keypoints)) {
        set_last_error("null argument");
        return SFMX_EINVAL;
    }
    if (width < 1 || height < 1 || pitch < width || width > 16384 || height > 16384) {
        set_last_error("image size must be 1..16384 with pitch >= width");
        return SFMX_EINVAL;
    }
    const int L = params->n_octave_layers;
    if (L < 1 || L > 16 || params->nfeatures < 0 || !(params->sigma > 0) || !(params->contrast_threshold >= 0) ||
        !(params->edge_threshold > 0)) {
        set_last_error("bad SIFT parameters");
        return SFMX_EINVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { set_last_error("no HIP device visible"); return SFMX_EDEVICE; }
    if (device < 0 || device >= ndev) { set_last_error("device index out of range"); return SFMX_EINVAL; }
    if (!is_gfx950(device)) { set_last_error("sfmx kernels are built for gfx950 only"); return SFMX_EDEVICE; }
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    const hipStream_t st = (hipStream_t)stream;
    int rc = SFMX_OK;
    {
        const float sigma = (float)params->sigma;
        const int BW = 2 * width, BH = 2 * height;
        const int nOct = host_round(std::log((double)std::min(BW, BH)) / std::log(2.) - 2) + 1;
        std::vector<double> sig(L + 3);
        sig[0] = sigma;
        const double k = std::pow(2., 1. / L);
        for (int i = 1; i < L + 3; i++) {
            const double sig_prev = std::pow(k, (double)(i - 1)) * sigma;
            const double sig_total = sig_prev * k;
            sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
        }
        const float sig_diff = std::sqrt(std::max(sigma * sigma - INIT_SIGMA * INIT_SIGMA * 4, 0.01f));
        // kern[L + 3]: createInitialImage's blur without doubling (compute() with firstOctave = 0)
        const float sig_diff0 = std::sqrt(std::max(sigma * sigma - INIT_SIGMA * INIT_SIGMA, 0.01f));
        std::vector<std::vector<float>> kern(L + 4);
        kern[0] = gauss_kernel(sig_diff);
        for (int i = 1; i < L + 3; i++) kern[i] = gauss_kernel(sig[i]);
        kern[L + 3] = gauss_kernel(sig_diff0);
        if (nOct < 1) {   // 1-pixel-high or -wide image: no octave, no keypoints (as OpenCV)
            *n_keypoints = 0;
            if (prev >= 0) (void)hipSetDevice(prev);
            return SFMX_OK;
        }
        std::vector<int> ow(nOct), oh(nOct);
        size_t px = 0;
        for (int o = 0; o < nOct; ++o) {
            ow[o] = o == 0 ? BW : ow[o - 1] / 2;
            oh[o] = o == 0 ? BH : oh[o - 1] / 2;
            px += (size_t)ow[o] * oh[o];
        }
        const int CAND_CAP = 1 << 20, REF_CAP = 1 << 19, KP_CAP = 1 << 20;
        size_t kbytes = 0;
        for (auto& kk : kern) kbytes += (kk.size() * 4 + 255) & ~(size_t)255;
        // the take() sequence below, each take rounded up to 256 B: the 2L + 5 layers per octave, tmp and up
        // (two BW x BH float buffers), the kernels, the layer tables, the candidate / keypoint buffers, the
        // staged host image and the staged descriptors
        const size_t ntakes = (size_t)nOct * (2 * L + 5) + (L + 4) + 12;
        const size_t need = px * 4 * (size_t)(2 * L + 5) + 2 * ((size_t)BW * BH * 4) + (size_t)width * height +
                            kbytes + sizeof(Cand) * CAND_CAP + sizeof(Refined) * REF_CAP + sizeof(Kp) * KP_CAP * 2 +
                            (size_t)KP_CAP * 128 * 4 + 16 + (size_t)nOct * (2 * L + 5) * sizeof(Layer) + 256 * ntakes;
        if (!arena.reserve(device, need)) { rc = SFMX_ENOMEM; set_last_error("device allocation failed"); goto done; }
        {
            Arena& A = arena;
            std::vector<Layer> hgp((size_t)nOct * (L + 3)), hdog((size_t)nOct * (L + 2));
            for (int o = 0; o < nOct; ++o) {
                for (int i = 0; i < L + 3; ++i) hgp[o * (L + 3) + i] = Layer{A.take<float>((size_t)ow[o] * oh[o]), ow[o], oh[o]};
                for (int i = 0; i < L + 2; ++i) hdog[o * (L + 2) + i] = Layer{A.take<float>((size_t)ow[o] * oh[o]), ow[o], oh[o]};
            }
            float* tmp = A.take<float>((size_t)BW * BH);
            float* up = A.take<float>((size_t)BW * BH);
            std::vector<float*> dk(L + 4);
            for (int i = 0; i < L + 4; ++i) dk[i] = A.take<float>(kern[i].size());
            Layer* dgp = A.take<Layer>(hgp.size());
            Layer* ddog = A.take<Layer>(hdog.size());
            Cand* cands = A.take<Cand>(CAND_CAP);
            Refined* refs = A.take<Refined>(REF_CAP);
            Kp* raw = A.take<Kp>(KP_CAP);
            Kp* fin = A.take<Kp>(KP_CAP);
            int* counters = A.take<int>(4);
            const uint8_t* dimg = image;
            int64_t dpitch = pitch;
            uint8_t* t = inputs_on_device ? nullptr : A.take<uint8_t>((size_t)width * height);
            float* dd_stage = inputs_on_device || !descriptors ? nullptr : A.take<float>((size_t)KP_CAP * 128);
            if (A.overflow) { set_last_error("internal: SIFT scratch arena too small"); rc = SFMX_ECAPACITY; goto done; }
            if (!inputs_on_device) {
                FCHK(hipMemcpy2DAsync(t, width, image, pitch, width, height, hipMemcpyHostToDevice, st));
                dimg = t;
                dpitch = width;
            }
            for (int i = 0; i < L + 4; ++i)
                FCHK(hipMemcpyAsync(dk[i], kern[i].data(), kern[i].size() * 4, hipMemcpyHostToDevice, st));
            FCHK(hipMemcpyAsync(dgp, hgp.data(), sizeof(Layer) * hgp.size(), hipMemcpyHostToDevice, st));
            FCHK(hipMemcpyAsync(ddog, hdog.data(), sizeof(Layer) * hdog.size(), hipMemcpyHostToDevice, st));
            FCHK(hipMemsetAsync(counters, 0, 16, st));
            FCHK(hipEventRecord(A.e0, st));
            // the tile blurs on XCD-contiguous block ranges (xcd.hpp: a tile's halo lines from the XCD's own
            // L2).  r05zd/ze (features leg, 150 images): the leg's counter traffic 1565 -> 1051 MB per image
            // (blurs 1.22 GB -> 0.69), one-stream blur 17.9 -> 17.4 us a launch; the extrema scan took
            // 18.2 -> 23.3 us on the same order for 115 -> 92 MB, so it keeps the plain grid.  A/B:
            // SFMX_SIFT_XCD (blurs), SFMX_SIFT_XCD_EXTREMA.
            int xcd = -1, xcd_ext = 0;
            if (const char* v = SFMX_DIAG_ENV("SFMX_SIFT_XCD")) xcd = std::atoi(v);
            if (const char* v = SFMX_DIAG_ENV("SFMX_SIFT_XCD_EXTREMA")) xcd_ext = std::atoi(v);
            // blur (+ the DoG of the new layer against its source layer when `dg` is set)
            auto blur = [&](const float* src, float* dst, float* dg, int w, int h, int ki) {
                const int n = (int)kern[ki].size();
                const dim3 tg((w + TX - 1) / TX, (h + TY - 1) / TY);
                if (n == 11) blur_tile_n_kernel<11><<<tg, 256, 0, st>>>(src, dst, dg, w, h, dk[ki], xcd);
                else if (n == 13) blur_tile_n_kernel<13><<<tg, 256, 0, st>>>(src, dst, dg, w, h, dk[ki], xcd);
                else if (n == 17) blur_tile_n_kernel<17><<<tg, 256, 0, st>>>(src, dst, dg, w, h, dk[ki], xcd);
                else if (n == 21) blur_tile_n_kernel<21><<<tg, 256, 0, st>>>(src, dst, dg, w, h, dk[ki], xcd);
                else if (n == 27) blur_tile_n_kernel<27><<<tg, 256, 0, st>>>(src, dst, dg, w, h, dk[ki], xcd);
                else if (n / 2 <= RMAX) {
                    blur_tile_kernel<<<tg, 256, 0, st>>>(src, dst, dg, w, h, dk[ki], n, xcd);
                } else {
                    const dim3 g((w + 255) / 256, h);
                    blur_row_kernel<<<g, 256, 0, st>>>(src, tmp, w, h, dk[ki], n);
                    blur_col_kernel<<<g, 256, 0, st>>>(tmp, dst, w, h, dk[ki], n);
                    if (dg) {
                        const int64_t m = (int64_t)w * h;
                        dog_kernel<<<(unsigned)((m + 255) / 256), 256, 0, st>>>(src, dst, dg, m);
                    }
                }
            };
            up2_kernel<<<dim3((BW + 255) / 256, BH), 256, 0, st>>>(dimg, width, height, dpitch, up);
            blur(up, hgp[0].p, nullptr, BW, BH, 0);
            // the trailing octaves of at most SMALL_PX pixels run in one launch (small_octaves_kernel)
            int o_small = nOct;
            if (small_octaves_on() && L + 3 <= SMALL_MAXL)
                while (o_small > 1 && (int64_t)ow[o_small - 1] * oh[o_small - 1] <= small_px()) --o_small;
            for (int o = 0; o < o_small; ++o)
                for (int i = 0; i < L + 3; ++i) {
                    if (o == 0 && i == 0) continue;
                    Layer& dst = hgp[o * (L + 3) + i];
                    if (i == 0) {
                        const Layer& src = hgp[(o - 1) * (L + 3) + L];
                        half_nn_kernel<<<dim3((dst.w + 255) / 256, dst.h), 256, 0, st>>>(
                            src.p, src.w, src.h, dst.p, dst.w, dst.h, 1. / ((double)dst.w / src.w), 1. / ((double)dst.h / src.h));
                    } else {
                        blur(hgp[o * (L + 3) + i - 1].p, dst.p, hdog[o * (L + 2) + i - 1].p, dst.w, dst.h, i);
                    }
                }
            const int threshold = (int)std::floor(0.5 * params->contrast_threshold / L * 255);
            if (o_small < nOct) {
                SmallTaps tp{};
                for (int i = 0; i < L + 3; ++i) { tp.p[i] = dk[i]; tp.n[i] = (int)kern[i].size(); }
                small_octaves_kernel<<<1, 1024, 0, st>>>(dgp, ddog, L, o_small, nOct, tp, tmp, threshold, cands, counters + 0,
                                                         CAND_CAP);
            }
            for (int o = 0; o < o_small; ++o) {
                const int w = ow[o], h = oh[o];
                if (w <= 2 * IMG_BORDER || h <= 2 * IMG_BORDER || L < 1) continue;
                const int nbx = (w - 2 * IMG_BORDER + 255) / 256, hr = h - 2 * IMG_BORDER;
                int rows = (int64_t)nbx * hr * L >= 65536 ? EX_ROWS : 1;   // (rows per thread, above)
                if (const char* v = SFMX_DIAG_ENV("SFMX_SIFT_EX_ROWS")) if (rows > 1) rows = std::max(1, std::min(EX_ROWS, std::atoi(v)));
                extrema_kernel<<<dim3(nbx, (hr + rows - 1) / rows, L), 256, 0, st>>>(ddog, L, w, h, threshold, o, cands,
                                                                                    counters + 0, CAND_CAP, xcd_ext, rows);
            }
            refine_kernel<<<CAND_CAP / 256, 256, 0, st>>>(cands, counters + 0, CAND_CAP, ddog, L,
                                                          (float)params->contrast_threshold, (float)params->edge_threshold,
                                                          sigma, refs, counters + 1, REF_CAP);
            FCHK(hipGetLastError());
            int hc[4] = {0, 0, 0, 0};
            FCHK(hipMemcpyAsync(hc, counters, 16, hipMemcpyDeviceToHost, st));
            FCHK(hipStreamSynchronize(st));
            if (hc[0] > CAND_CAP || hc[1] > REF_CAP) { set_last_error("too many extrema for the candidate buffers"); rc = SFMX_ECAPACITY; goto done; }
            if (hc[1] > 0) orient_kernel<<<hc[1], 64, 0, st>>>(refs, counters + 1, REF_CAP, dgp, L, raw, counters + 2, KP_CAP);
            FCHK(hipGetLastError());
            FCHK(hipMemcpyAsync(hc, counters, 16, hipMemcpyDeviceToHost, st));
            FCHK(hipStreamSynchronize(st));
            if (hc[2] > KP_CAP) { set_last_error("too many keypoints for the buffer"); rc = SFMX_ECAPACITY; goto done; }
            std::vector<Kp> kps(hc[2]);
            if (hc[2]) FCHK(hipMemcpyAsync(kps.data(), raw, sizeof(Kp) * hc[2], hipMemcpyDeviceToHost, st));
            FCHK(hipStreamSynchronize(st));
            filter_keypoints(kps, params->nfeatures);
            const int n = (int)kps.size();
            *n_keypoints = n;
            const int m = std::min(n, (int)capacity);
            if (m > 0) {
                FCHK(hipMemcpyAsync(fin, kps.data(), sizeof(Kp) * m, hipMemcpyHostToDevice, st));
                if (descriptors) {
                    // compute() after detect() (SfM.cpp:586-587): firstOctave = min(0, min kept octave). When no kept
                    // keypoint is from the doubled octave the pyramid is rebuilt un-doubled for the descriptors; its
                    // octave o has exactly the size of the doubled pyramid's octave o + 1, so it reuses those slots.
                    int cFirst = 0, cMaxOct = INT_MIN;
                    for (int q = 0; q < n; ++q) {
                        int o = kps[q].octave & 255;
                        o = o < 128 ? o : (-128 | o);
                        cFirst = std::min(cFirst, o);
                        cMaxOct = std::max(cMaxOct, o);
                    }
                    const Layer* dgp_desc = dgp;
                    int first_desc = -1;
                    if (cFirst == 0) {
                        const int nOc = cMaxOct + 1;   // <= nOct - 1: detection octaves are < nOct in doubled numbering
                        to_float_kernel<<<dim3((width + 255) / 256, height), 256, 0, st>>>(dimg, width, height, dpitch, up);
                        blur(up, hgp[L + 3].p, nullptr, width, height, L + 3);
                        for (int o = 0; o < nOc; ++o)
                            for (int i = 0; i < L + 3; ++i) {
                                if (o == 0 && i == 0) continue;
                                Layer& dst = hgp[(o + 1) * (L + 3) + i];
                                if (i == 0) {
                                    const Layer& src = hgp[o * (L + 3) + L];   // rebuilt octave o - 1, layer L
                                    half_nn_kernel<<<dim3((dst.w + 255) / 256, dst.h), 256, 0, st>>>(
                                        src.p, src.w, src.h, dst.p, dst.w, dst.h, 1. / ((double)dst.w / src.w), 1. / ((double)dst.h / src.h));
                                } else {
                                    blur(hgp[(o + 1) * (L + 3) + i - 1].p, dst.p, nullptr, dst.w, dst.h, i);
                                }
                            }
                        dgp_desc = dgp + (L + 3);
                        first_desc = 0;
                    }
                    float* dd = inputs_on_device ? descriptors : dd_stage;
                    descriptor_kernel<<<m, DESC_THREADS, 0, st>>>(fin, m, dgp_desc, L, first_desc, dd);
                    FCHK(hipGetLastError());
                    if (!inputs_on_device)
                        FCHK(hipMemcpyAsync(descriptors, dd, sizeof(float) * 128 * m, hipMemcpyDeviceToHost, st));
                }
                if (inputs_on_device) FCHK(hipMemcpyAsync(keypoints, fin, sizeof(Kp) * m, hipMemcpyDeviceToDevice, st));
                else std::memcpy(keypoints, kps.data(), sizeof(Kp) * m);
            }
            FCHK(hipEventRecord(A.e1, st));
            FCHK(hipStreamSynchronize(st));
            float ms = -1.f;
            (void)hipEventElapsedTime(&ms, A.e0, A.e1);
            *last_ms = ms;
            if (n > capacity) { set_last_error("keypoint capacity too small"); rc = SFMX_ECAPACITY; }
        }
    done:;
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
}

// Batch workers: one host thread and one non-blocking HIP stream per slot,
// each with its own scratch arena, kept for the life of the process.
struct BatchSlot {
    Arena arena;
    hipStream_t stream = nullptr;
    int device = -1;
};
std::mutex g_batch_mu;
std::vector<std::unique_ptr<BatchSlot>> g_slots;

}  // namespace

extern "C" {

int sfmx_sift_detect_compute(const uint8_t* image, int32_t width, int32_t height, int64_t pitch,
                             const sfmx_sift_params* params, int32_t inputs_on_device, int32_t device, void* stream,
                             sfmx_keypoint* keypoints, float* descriptors, int32_t capacity, int32_t* n_keypoints) {
    return detect_compute_impl(image, width, height, pitch, params, inputs_on_device, device, stream, keypoints,
                               descriptors, capacity, n_keypoints, g_arena, &g_last_ms);
}

int sfmx_sift_detect_compute_batch(const sfmx_gray_image* images, int32_t n_images, const sfmx_sift_params* params,
                                   int32_t inputs_on_device, int32_t device, int32_t n_streams,
                                   sfmx_keypoint* const* keypoints, float* const* descriptors,
                                   const int32_t* capacities, int32_t* n_keypoints, int32_t* status) {
    if (n_images < 0 || (n_images > 0 && (!images || !keypoints || !capacities || !n_keypoints)) || !params) {
        set_last_error("null argument");
        return SFMX_EINVAL;
    }
    if (n_streams < 1 || n_streams > 16) { set_last_error("n_streams must be 1..16"); return SFMX_EINVAL; }
    if (n_images == 0) { g_last_ms = 0.f; return SFMX_OK; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { set_last_error("no HIP device visible"); return SFMX_EDEVICE; }
    if (device < 0 || device >= ndev) { set_last_error("device index out of range"); return SFMX_EINVAL; }
    std::lock_guard<std::mutex> lock(g_batch_mu);
    const int ns = std::min<int>(n_streams, n_images);
    while ((int)g_slots.size() < ns) g_slots.emplace_back(new BatchSlot());
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    for (int i = 0; i < ns; ++i) {
        BatchSlot& sl = *g_slots[i];
        if (sl.device != device) {
            if (sl.stream) (void)hipStreamDestroy(sl.stream);
            sl.stream = nullptr;
            if (hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess) {
                if (prev >= 0) (void)hipSetDevice(prev);
                set_last_error("hipStreamCreate failed");
                return SFMX_EDEVICE;
            }
            sl.device = device;
        }
    }
    std::atomic<int> next{0};
    std::vector<int> rcs(n_images, SFMX_OK);
    std::vector<float> kms(ns, 0.f);
    std::vector<std::string> errs(n_images);
    auto work = [&](int slot) {
        (void)hipSetDevice(device);
        BatchSlot& sl = *g_slots[slot];
        for (int i; (i = next.fetch_add(1)) < n_images;) {
            float ms = 0.f;
            const sfmx_gray_image& im = images[i];
            rcs[i] = detect_compute_impl(im.data, im.width, im.height, im.pitch, params, inputs_on_device, device,
                                         sl.stream, keypoints[i], descriptors ? descriptors[i] : nullptr,
                                         capacities[i], &n_keypoints[i], sl.arena, &ms);
            if (rcs[i] != SFMX_OK) errs[i] = sfmx_last_error();
            kms[slot] += ms;
        }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < ns; ++i) th.emplace_back(work, i);
    work(0);
    for (auto& t : th) t.join();
    if (prev >= 0) (void)hipSetDevice(prev);
    float total = 0.f;
    for (float k : kms) total += k;
    g_last_ms = total / n_images;
    int rc = SFMX_OK;
    for (int i = 0; i < n_images; ++i) {
        if (status) status[i] = rcs[i];
        if (rcs[i] != SFMX_OK && rc == SFMX_OK) {   // first failing image decides the return code
            rc = rcs[i];
            set_last_error(("image " + std::to_string(i) + ": " + errs[i]).c_str());
        }
    }
    return rc;
}

}  // extern "C"
