// SPDX-License-Identifier: MIT
// sfmx bundle adjustment kernels for gfx950 (MI355X / CDNA4), fp64.
//
// One Levenberg-Marquardt iteration of the reference's Ceres problem
// (BundleAdjustment.cpp:29-91 solved by CeresUtils::solve, DENSE_SCHUR):
//   ba_linearize      residual + Jacobian of every observation by forward-mode
//                     dual numbers (what ceres::AutoDiffCostFunction does for the
//                     reference functors SimpleRadialCamera.cpp:79-115,
//                     SimpleCamera.cpp:73-103, DistortionCamera.cpp:72-110)
//   column kernels    J^T r and squared column norms (Jacobi scaling, LM diagonal)
//   ba_point_blocks   per 3-dof point block: E = Je^T Je + D_e^2, E^-1, and the
//                     per-observation factors the Schur complement needs
//   ba_cam_blocks     per camera: pose-pose diagonal, pose-intrinsics coupling, rhs
//   ba_pair_blocks    per co-visible camera pair: -sum W_a^T E^-1 W_b, one
//                     workgroup per 6x6 block, fixed-order tree sums (deterministic)
//   ba_assemble       dense reduced camera system S ((6C+k) padded to 64)
//   chol_*            block LDL^T of S (64x64 tiles, one launch per panel) + solves
//   ba_backsub / ba_step / ba_model / ba_cost
// Layout in HBM: parameters x = [points 3P | poses 6C | intrinsics k]; the
// Jacobian is stored per observation, J[o][f] (f = r0,r1, Je 2x3, Jc 2x6, Ji 2xk,
// stride jst(K) = 20 + 2k): every gather (by point, by camera) reads whole records.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cfloat>

namespace sfmx {
namespace ba {

constexpr int NB = 64;   // Cholesky tile
// Bijective XCD-contiguous block remap (blocks b, b+8, ... land on one XCD;
// speed only, never correctness).
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}
__host__ __device__ constexpr int jst(int K) { return 20 + 2 * K; }   // Jacobian record stride

// ---- dual numbers --------------------------------------------------------
template <int N>
struct DJet {
    double a;
    double v[N];
};
template <int N> __device__ __forceinline__ DJet<N> jconst(double x) { DJet<N> r; r.a = x;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = 0.0; return r; }
template <int N> __device__ __forceinline__ DJet<N> jvar(double x, int k) { DJet<N> r = jconst<N>(x);
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = (i == k) ? 1.0 : 0.0; return r; }
template <int N> __device__ __forceinline__ DJet<N> operator+(const DJet<N>& f, const DJet<N>& g) { DJet<N> r; r.a = f.a + g.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = f.v[i] + g.v[i]; return r; }
template <int N> __device__ __forceinline__ DJet<N> operator-(const DJet<N>& f, const DJet<N>& g) { DJet<N> r; r.a = f.a - g.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = f.v[i] - g.v[i]; return r; }
template <int N> __device__ __forceinline__ DJet<N> operator*(const DJet<N>& f, const DJet<N>& g) { DJet<N> r; r.a = f.a * g.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = f.a * g.v[i] + f.v[i] * g.a; return r; }
template <int N> __device__ __forceinline__ DJet<N> operator*(double s, const DJet<N>& f) { DJet<N> r; r.a = s * f.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i]; return r; }
template <int N> __device__ __forceinline__ DJet<N> operator/(const DJet<N>& f, const DJet<N>& g) {
    const double gi = 1.0 / g.a, fg = f.a * gi;
    DJet<N> r; r.a = f.a * gi;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = (f.v[i] - fg * g.v[i]) * gi;
    return r;
}
template <int N> __device__ __forceinline__ DJet<N> jsqrt(const DJet<N>& f) {
    const double s = sqrt(f.a), t = 1.0 / (2.0 * s);
    DJet<N> r; r.a = s;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = t * f.v[i]; return r;
}
template <int N> __device__ __forceinline__ void jsincos(const DJet<N>& f, DJet<N>& sn, DJet<N>& cs) {
    double s, c;
    sincos(f.a, &s, &c);
    sn.a = s; cs.a = c;
#pragma unroll
    for (int i = 0; i < N; ++i) { sn.v[i] = c * f.v[i]; cs.v[i] = -s * f.v[i]; }
}

// ceres::AngleAxisRotatePoint (Ceres 1.14 rotation.h) on dual numbers.
template <int N>
__device__ __forceinline__ void rotate(const DJet<N> aa[3], const DJet<N> pt[3], DJet<N> res[3]) {
    const DJet<N> theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
    if (theta2.a > DBL_EPSILON) {
        const DJet<N> theta = jsqrt(theta2);
        DJet<N> st, ct;
        jsincos(theta, st, ct);
        const DJet<N> ti = jconst<N>(1.0) / theta;
        const DJet<N> w[3] = {aa[0] * ti, aa[1] * ti, aa[2] * ti};
        const DJet<N> wx[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
        const DJet<N> tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (jconst<N>(1.0) - ct);
#pragma unroll
        for (int i = 0; i < 3; ++i) res[i] = pt[i] * ct + wx[i] * st + w[i] * tmp;
    } else {
        const DJet<N> wx[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]};
#pragma unroll
        for (int i = 0; i < 3; ++i) res[i] = pt[i] + wx[i];
    }
}

// The reference functors' arithmetic (same operation order).
template <int K, int N>
__device__ __forceinline__ void project(const DJet<N> X[3], const DJet<N> ps[6], const DJet<N> in[K], double ox, double oy,
                                        double cx, double cy, DJet<N> res[2]) {
    DJet<N> p[3];
    rotate(ps, X, p);
    p[0] = p[0] + ps[3]; p[1] = p[1] + ps[4]; p[2] = p[2] + ps[5];
    const DJet<N> xp = p[0] / p[2];
    const DJet<N> yp = p[1] / p[2];
    const DJet<N> xd = in[0] * xp;
    const DJet<N> yd = in[0] * yp;
    if constexpr (K == 1) {
        res[0] = xd - jconst<N>(ox - cx);
        res[1] = yd - jconst<N>(oy - cy);
    } else if constexpr (K == 3) {
        const DJet<N> r2 = (xp * xp) + (yp * yp);
        const DJet<N> r4 = r2 * r2;
        const DJet<N> rad = in[1] * r2 + in[2] * r4;
        res[0] = (xd + xd * rad) - (jconst<N>(ox) - jconst<N>(cx));
        res[1] = (yd + yd * rad) - (jconst<N>(oy) - jconst<N>(cy));
    } else {
        const DJet<N> r2 = (xp * xp) + (yp * yp);
        const DJet<N> r4 = r2 * r2;
        const DJet<N> rad = in[3] * r2 + in[4] * r4;
        const DJet<N> xu = xd + xd * rad + (in[5] * (r2 + 2.0 * (xd * xd)) + 2.0 * in[6] * xd * yd);
        const DJet<N> yu = yd + yd * rad + (2.0 * in[5] * xd * yd + in[6] * (r2 + 2.0 * (yd * yd)));
        res[0] = xu - (jconst<N>(ox) - in[1]);
        res[1] = yu - (jconst<N>(oy) - in[2]);
    }
}

// ---- block reduction helper (256 threads, fixed order) -------------------
__device__ __forceinline__ double block_sum(double v, double* sh) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    double s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sh[w];
    return s;   // valid in thread 0
}

// ---- linearization --------------------------------------------------------
// Fields of the field-major Jacobian store: 0,1 r; 2..7 Je (row-major 2x3);
// 8..19 Jc (2x6); 20..20+2K Ji (2xK).
template <int K, bool JAC>
__global__ __launch_bounds__(256)
void ba_linearize(int O, const int* __restrict__ obs_point, const int* __restrict__ obs_cam,
                  const double* __restrict__ obs_xy, double cx, double cy, const double* __restrict__ pts,
                  const double* __restrict__ poses, const double* __restrict__ intr, double* __restrict__ J,
                  double* __restrict__ partial) {
    __shared__ double sh[8];
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    double c2 = 0.0;
    if (o < O) {
        const int p = obs_point[o], c = obs_cam[o];
        const double ox = obs_xy[2 * (size_t)o], oy = obs_xy[2 * (size_t)o + 1];
        if constexpr (JAC) {
            constexpr int N = 9 + K;
            DJet<N> X[3], ps[6], in[K], res[2];
#pragma unroll
            for (int i = 0; i < 3; ++i) X[i] = jvar<N>(pts[3 * (size_t)p + i], i);
#pragma unroll
            for (int i = 0; i < 6; ++i) ps[i] = jvar<N>(poses[6 * (size_t)c + i], 3 + i);
#pragma unroll
            for (int i = 0; i < K; ++i) in[i] = jvar<N>(intr[i], 9 + i);
            project<K, N>(X, ps, in, ox, oy, cx, cy, res);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                J[(size_t)o * jst(K) + j] = res[j].a;
#pragma unroll
                for (int i = 0; i < 3; ++i) J[(size_t)o * jst(K) + (2 + 3 * j + i)] = res[j].v[i];
#pragma unroll
                for (int i = 0; i < 6; ++i) J[(size_t)o * jst(K) + (8 + 6 * j + i)] = res[j].v[3 + i];
#pragma unroll
                for (int i = 0; i < K; ++i) J[(size_t)o * jst(K) + (20 + K * j + i)] = res[j].v[9 + i];
            }
            c2 = res[0].a * res[0].a + res[1].a * res[1].a;
        } else {
            DJet<0> X[3], ps[6], in[K], res[2];
#pragma unroll
            for (int i = 0; i < 3; ++i) X[i].a = pts[3 * (size_t)p + i];
#pragma unroll
            for (int i = 0; i < 6; ++i) ps[i].a = poses[6 * (size_t)c + i];
#pragma unroll
            for (int i = 0; i < K; ++i) in[i].a = intr[i];
            project<K, 0>(X, ps, in, ox, oy, cx, cy, res);
            c2 = res[0].a * res[0].a + res[1].a * res[1].a;
        }
    }
    const double s = block_sum(c2, sh);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// Deterministic final sum of `n` partials (one block); out[0] = scale * sum.
__global__ __launch_bounds__(256)
void ba_sum(const double* __restrict__ partial, int n, double scale, double* __restrict__ out) {
    __shared__ double sh[8];
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) v += partial[i];
    const double s = block_sum(v, sh);
    if (threadIdx.x == 0) out[0] = scale * s;
}

// Squared column norms (unscaled) and gradient J^T r.
// Points: one thread per point over its observations (CSR).
template <int K>
__global__ __launch_bounds__(256)
void ba_point_cols(int P, int O, const int* __restrict__ pt_start, const int* __restrict__ pt_obs,
                   const double* __restrict__ J, double* __restrict__ colsq, double* __restrict__ grad) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    double cs[3] = {0, 0, 0}, g[3] = {0, 0, 0};
    for (int a = pt_start[p]; a < pt_start[p + 1]; ++a) {
        const int o = pt_obs[a];
        const double r0 = J[(size_t)o * jst(K)], r1 = J[(size_t)o * jst(K) + 1];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double j0 = J[(size_t)o * jst(K) + (2 + i)], j1 = J[(size_t)o * jst(K) + (5 + i)];
            cs[i] += j0 * j0 + j1 * j1;
            g[i] += j0 * r0 + j1 * r1;
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) { colsq[3 * (size_t)p + i] = cs[i]; grad[3 * (size_t)p + i] = g[i]; }
}

// Cameras: one block per camera over its observations; intrinsics: per-block
// partials over observation ranges (cam-major), summed by ba_intr_cols_final.
template <int K>
__global__ __launch_bounds__(256)
void ba_cam_cols(int O, const int* __restrict__ cam_start, const int* __restrict__ cam_obs, const double* __restrict__ J,
                 double* __restrict__ colsq, double* __restrict__ grad, double* __restrict__ ipart) {
    __shared__ double sh[8];
    const int c = blockIdx.x;
    double v[12 + 2 * K];
#pragma unroll
    for (int i = 0; i < 12 + 2 * K; ++i) v[i] = 0.0;
    for (int a = cam_start[c] + threadIdx.x; a < cam_start[c + 1]; a += blockDim.x) {
        const int o = cam_obs[a];
        const double r0 = J[(size_t)o * jst(K)], r1 = J[(size_t)o * jst(K) + 1];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double j0 = J[(size_t)o * jst(K) + (8 + i)], j1 = J[(size_t)o * jst(K) + (14 + i)];
            v[i] += j0 * j0 + j1 * j1;
            v[6 + i] += j0 * r0 + j1 * r1;
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const double j0 = J[(size_t)o * jst(K) + (20 + i)], j1 = J[(size_t)o * jst(K) + (20 + K + i)];
            v[12 + i] += j0 * j0 + j1 * j1;
            v[12 + K + i] += j0 * r0 + j1 * r1;
        }
    }
#pragma unroll
    for (int i = 0; i < 12 + 2 * K; ++i) {
        const double s = block_sum(v[i], sh);
        if (threadIdx.x == 0) {
            if (i < 6) colsq[6 * (size_t)c + i] = s;
            else if (i < 12) grad[6 * (size_t)c + i - 6] = s;
            else ipart[(size_t)c * 2 * K + (i - 12)] = s;
        }
    }
}

template <int K>
__global__ void ba_intr_cols_final(int C, const double* __restrict__ ipart, double* __restrict__ colsq,
                                   double* __restrict__ grad) {
    const int i = threadIdx.x;
    if (i >= 2 * K) return;
    double s = 0;
    for (int c = 0; c < C; ++c) s += ipart[(size_t)c * 2 * K + i];
    if (i < K) colsq[i] = s; else grad[i - K] = s;
}

// scale = 1 / (1 + sqrt(colsq)) (iteration 0 only, Ceres jacobi_scaling)
__global__ void ba_scale(int n, const double* __restrict__ colsq, double* __restrict__ scale) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) scale[i] = 1.0 / (1.0 + sqrt(colsq[i]));
}
// LM diagonal from the scaled Jacobian: clamp(colsq * scale^2, min, max);
// also max |grad| partials for the gradient tolerance.
__global__ __launch_bounds__(256)
void ba_diag(int n, const double* __restrict__ colsq, const double* __restrict__ scale, double dmin, double dmax,
             double* __restrict__ diag, const double* __restrict__ grad, double* __restrict__ gpart) {
    __shared__ double sh[8];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double g = 0.0;
    if (i < n) {
        const double s = scale[i];
        diag[i] = fmin(fmax(colsq[i] * s * s, dmin), dmax);
        g = fabs(grad[i]);
    }
    for (int o = 32; o > 0; o >>= 1) g = fmax(g, __shfl_xor(g, o));
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) sh[wid] = g;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = fmax(m, sh[w]);
        gpart[blockIdx.x] = m;
    }
}
__global__ __launch_bounds__(256)
void ba_max(const double* __restrict__ part, int n, double* __restrict__ out) {
    __shared__ double sh[8];
    double g = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) g = fmax(g, part[i]);
    for (int o = 32; o > 0; o >>= 1) g = fmax(g, __shfl_xor(g, o));
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = g;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = fmax(m, sh[w]);
        out[0] = m;
    }
}

// ---- Schur complement -------------------------------------------------------
// D = sqrt(diag / radius) (LevenbergMarquardtStrategy::ComputeStep [ext]).
__global__ void ba_lm_d(int n, const double* __restrict__ diag, double radius, double* __restrict__ D) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) D[i] = sqrt(diag[i] / radius);
}

__device__ __forceinline__ bool inv3_spd(const double* A, double* Ai) {
    double l00 = A[0];
    if (!(l00 > 0)) return false;
    l00 = sqrt(l00);
    const double l10 = A[3] / l00, l20 = A[6] / l00;
    double l11 = A[4] - l10 * l10;
    if (!(l11 > 0)) return false;
    l11 = sqrt(l11);
    const double l21 = (A[7] - l20 * l10) / l11;
    double l22 = A[8] - l20 * l20 - l21 * l21;
    if (!(l22 > 0)) return false;
    l22 = sqrt(l22);
    const double i00 = 1 / l00, i11 = 1 / l11, i22 = 1 / l22;
    const double i10 = -l10 * i00 * i11;
    const double i21 = -l21 * i11 * i22;
    const double i20 = -(l20 * i00 + l21 * i10) * i22;
    const double Li[9] = {i00, 0, 0, i10, i11, 0, i20, i21, i22};
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            double s = 0;
#pragma unroll
            for (int m = 0; m < 3; ++m) s += Li[m * 3 + a] * Li[m * 3 + b];
            Ai[a * 3 + b] = s;
        }
    return true;
}

// Per-observation records written by ba_point_blocks (AoS, so the gathers of
// the Schur kernels touch whole cache lines instead of one line per field):
//   R1[o]          (point-major, stride r1s(K) = 24 + 2K): Je_s 2x3 | U = Einv Je_s^T 3x2 | Jc_s 2x6 | Ji_s 2xK
//   R2[campos(o)]  (camera-major, stride r2s(K) = 14 + 4K): Jc_s 2x6 | Ji_s 2xK | T = Je_s Einv V 2xK | r - q 2
__host__ __device__ constexpr int r1s(int K) { return 24 + 2 * K; }
__host__ __device__ constexpr int r2s(int K) { return 14 + 4 * K; }

// Per point: E = sum Je_s^T Je_s + D_e^2, g_e = sum Je_s^T r, Einv, EinvG = Einv g_e,
// V = sum Je_s^T Ji_s (3xK); per observation the R1/R2 records (q = Je_s EinvG);
// per-block partials of sum_p V^T Einv V (KxK) for the intrinsics block.
template <int K>
__global__ __launch_bounds__(256)
void ba_point_blocks(int P, int O, int C, const int* __restrict__ pt_start, const int* __restrict__ pt_obs,
                     const int* __restrict__ obs_cam, const int* __restrict__ campos, const double* __restrict__ J,
                     const double* __restrict__ scale, const double* __restrict__ D, double* __restrict__ Einv,
                     double* __restrict__ EinvG, double* __restrict__ R1, double* __restrict__ R2,
                     double* __restrict__ vzpart, int* __restrict__ fail, const int* __restrict__ plist, int nlist) {
    __shared__ double sh[8];
    const int gi = blockIdx.x * blockDim.x + threadIdx.x;
    const int p = plist ? (gi < nlist ? plist[gi] : P) : gi;   // plist: only these points (see ba_point_blocks_lds)
    const size_t ne = 3 * (size_t)P, ni = ne + 6 * (size_t)C;   // first camera / intrinsics column
    double VZ[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) VZ[i] = 0.0;
    if (p < P) {
        const double sp[3] = {scale[3 * (size_t)p], scale[3 * (size_t)p + 1], scale[3 * (size_t)p + 2]};
        double si[K];
#pragma unroll
        for (int i = 0; i < K; ++i) si[i] = scale[ni + i];
        double E[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0}, V[3 * K];
#pragma unroll
        for (int i = 0; i < 3 * K; ++i) V[i] = 0.0;
        const int a0 = pt_start[p], a1 = pt_start[p + 1];
        for (int a = a0; a < a1; ++a) {
            const int o = pt_obs[a];
            const double r[2] = {J[(size_t)o * jst(K)], J[(size_t)o * jst(K) + 1]};
            double je[2][3], ji[2][K];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int u = 0; u < 3; ++u) je[j][u] = J[(size_t)o * jst(K) + (2 + 3 * j + u)] * sp[u];
#pragma unroll
                for (int i = 0; i < K; ++i) ji[j][i] = J[(size_t)o * jst(K) + (20 + K * j + i)] * si[i];
            }
#pragma unroll
            for (int u = 0; u < 3; ++u) {
#pragma unroll
                for (int v = 0; v < 3; ++v) E[u * 3 + v] += je[0][u] * je[0][v] + je[1][u] * je[1][v];
                g[u] += je[0][u] * r[0] + je[1][u] * r[1];
#pragma unroll
                for (int i = 0; i < K; ++i) V[u * K + i] += je[0][u] * ji[0][i] + je[1][u] * ji[1][i];
            }
        }
        const double d0 = D[3 * (size_t)p], d1 = D[3 * (size_t)p + 1], d2 = D[3 * (size_t)p + 2];
        E[0] += d0 * d0; E[4] += d1 * d1; E[8] += d2 * d2;
        double Ei[9];
        if (!inv3_spd(E, Ei)) {
            atomicOr(fail, 1);
#pragma unroll
            for (int i = 0; i < 9; ++i) Ei[i] = 0.0;
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) Einv[9 * (size_t)p + i] = Ei[i];
        double eg[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            eg[u] = Ei[u * 3] * g[0] + Ei[u * 3 + 1] * g[1] + Ei[u * 3 + 2] * g[2];
            EinvG[3 * (size_t)p + u] = eg[u];
        }
        double Z[3 * K];   // Einv V
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int i = 0; i < K; ++i) Z[u * K + i] = Ei[u * 3] * V[i] + Ei[u * 3 + 1] * V[K + i] + Ei[u * 3 + 2] * V[2 * K + i];
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int l = 0; l < K; ++l) VZ[i * K + l] = V[i] * Z[l] + V[K + i] * Z[K + l] + V[2 * K + i] * Z[2 * K + l];
        for (int a = a0; a < a1; ++a) {
            const int o = pt_obs[a];
            const size_t nc = ne + 6 * (size_t)obs_cam[o];
            double* r1 = R1 + (size_t)o * r1s(K);
            double* r2 = R2 + (size_t)campos[o] * r2s(K);
            double je[2][3];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int u = 0; u < 3; ++u) { je[j][u] = J[(size_t)o * jst(K) + (2 + 3 * j + u)] * sp[u]; r1[3 * j + u] = je[j][u]; }
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double v = J[(size_t)o * jst(K) + (8 + 6 * j + i)] * scale[nc + i];
                    r1[12 + 6 * j + i] = v;
                    r2[6 * j + i] = v;
                }
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const double v = J[(size_t)o * jst(K) + (20 + K * j + i)] * si[i];
                    r1[24 + K * j + i] = v;
                    r2[12 + K * j + i] = v;
                }
            }
#pragma unroll
            for (int u = 0; u < 3; ++u)
#pragma unroll
                for (int j = 0; j < 2; ++j) r1[6 + u * 2 + j] = Ei[u * 3] * je[j][0] + Ei[u * 3 + 1] * je[j][1] + Ei[u * 3 + 2] * je[j][2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int i = 0; i < K; ++i) r2[12 + 2 * K + K * j + i] = je[j][0] * Z[i] + je[j][1] * Z[K + i] + je[j][2] * Z[2 * K + i];
                const double qj = je[j][0] * eg[0] + je[j][1] * eg[1] + je[j][2] * eg[2];
                r2[12 + 4 * K + j] = J[(size_t)o * jst(K) + j] - qj;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < K * K; ++i) {
        const double s = block_sum(VZ[i], sh);
        if (threadIdx.x == 0) vzpart[(size_t)blockIdx.x * K * K + i] = s;
    }
}

// Same outputs as ba_point_blocks, LDS-staged so that every HBM access is a
// coalesced stream: one workgroup per host-built point group (points bp[2b] ..
// bp[2b+1]: at most PB_MAXP points whose observations, contiguous in the
// point-major internal order, number at most PB_CAPO).
//   1. the group's Jacobian records J[o0 .. o1) are copied into LDS (16-B loads)
//   2. one thread per point: E, g, V from LDS; Einv, Einv g, Z = Einv V -> LDS
//   3. one thread per observation: its R1 and R2 records in registers
//   4. R1[o0 .. o1) staged in LDS and stored contiguously; then the R2 records
//      staged and stored record by record at their camera-major slots.
// Points with more than CAPO observations go to ba_point_blocks (point list).
constexpr int PB_CAPO = 256;   // observations per group (= threads: one per observation)
constexpr int PB_MAXP = 64;    // points per group
template <int K>
__global__ __launch_bounds__(256)
void ba_point_blocks_lds(const int* __restrict__ bp, int P, int C, const int* __restrict__ pt_start,
                         const int* __restrict__ obs_cam, const int* __restrict__ campos, const double* __restrict__ J,
                         const double* __restrict__ scale, const double* __restrict__ D, double* __restrict__ Einv,
                         double* __restrict__ EinvG, double* __restrict__ R1, double* __restrict__ R2,
                         double* __restrict__ vzpart, int* __restrict__ fail) {
    constexpr int JS = jst(K), RS1 = r1s(K), RS2 = r2s(K);
    constexpr int BUF = PB_CAPO * (RS1 > JS ? RS1 : JS);
    constexpr int PD = 12 + 3 * K;                       // per point: Ei (9) | Einv g (3) | Z = Einv V (3K)
    static_assert(JS % 2 == 0 && RS1 % 2 == 0 && RS2 % 2 == 0, "records must be whole 16-B pieces");
    __shared__ __attribute__((aligned(16))) double buf[BUF];
    __shared__ double pd[PB_MAXP * PD];
    __shared__ int opt[PB_CAPO];                         // observation -> point slot in the group
    __shared__ double sh[8];
    const int tid = threadIdx.x, b = blockIdx.x;
    const int p0 = bp[2 * b], np = bp[2 * b + 1] - p0;
    const int o0 = pt_start[p0], no = pt_start[p0 + np] - o0;
    const size_t ne = 3 * (size_t)P, ni = ne + 6 * (size_t)C;   // first camera / intrinsics column
    {   // 1. J records of the group -> LDS
        const double2* src = reinterpret_cast<const double2*>(J + (size_t)o0 * JS);
        double2* dst = reinterpret_cast<double2*>(buf);
        for (int i = tid; i < no * (JS / 2); i += 256) dst[i] = src[i];
    }
    double si[K];
#pragma unroll
    for (int i = 0; i < K; ++i) si[i] = scale[ni + i];
    __syncthreads();
    // 2. one thread per point
    double VZ[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) VZ[i] = 0.0;
    if (tid < np) {
        const int p = p0 + tid;
        const int a0 = pt_start[p] - o0, a1 = pt_start[p + 1] - o0;
        const double sp[3] = {scale[3 * (size_t)p], scale[3 * (size_t)p + 1], scale[3 * (size_t)p + 2]};
        double E[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0}, V[3 * K];
#pragma unroll
        for (int i = 0; i < 3 * K; ++i) V[i] = 0.0;
        for (int a = a0; a < a1; ++a) {
            opt[a] = tid;
            const double* jr = buf + a * JS;
            const double r[2] = {jr[0], jr[1]};
            double je[2][3], ji[2][K];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int u = 0; u < 3; ++u) je[j][u] = jr[2 + 3 * j + u] * sp[u];
#pragma unroll
                for (int i = 0; i < K; ++i) ji[j][i] = jr[20 + K * j + i] * si[i];
            }
#pragma unroll
            for (int u = 0; u < 3; ++u) {
#pragma unroll
                for (int v = 0; v < 3; ++v) E[u * 3 + v] += je[0][u] * je[0][v] + je[1][u] * je[1][v];
                g[u] += je[0][u] * r[0] + je[1][u] * r[1];
#pragma unroll
                for (int i = 0; i < K; ++i) V[u * K + i] += je[0][u] * ji[0][i] + je[1][u] * ji[1][i];
            }
        }
        const double d0 = D[3 * (size_t)p], d1 = D[3 * (size_t)p + 1], d2 = D[3 * (size_t)p + 2];
        E[0] += d0 * d0; E[4] += d1 * d1; E[8] += d2 * d2;
        double Ei[9];
        if (!inv3_spd(E, Ei)) {
            atomicOr(fail, 1);
#pragma unroll
            for (int i = 0; i < 9; ++i) Ei[i] = 0.0;
        }
        double* q = pd + tid * PD;
#pragma unroll
        for (int i = 0; i < 9; ++i) { Einv[9 * (size_t)p + i] = Ei[i]; q[i] = Ei[i]; }
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const double eg = Ei[u * 3] * g[0] + Ei[u * 3 + 1] * g[1] + Ei[u * 3 + 2] * g[2];
            EinvG[3 * (size_t)p + u] = eg;
            q[9 + u] = eg;
        }
        double Z[3 * K];
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int i = 0; i < K; ++i) {
                Z[u * K + i] = Ei[u * 3] * V[i] + Ei[u * 3 + 1] * V[K + i] + Ei[u * 3 + 2] * V[2 * K + i];
                q[12 + u * K + i] = Z[u * K + i];
            }
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int l = 0; l < K; ++l) VZ[i * K + l] = V[i] * Z[l] + V[K + i] * Z[K + l] + V[2 * K + i] * Z[2 * K + l];
    }
    __syncthreads();
    // 3. one thread per observation: R1 / R2 records in registers
    double r1[RS1], r2[RS2];
    const int a = tid;
    if (a < no) {
        const int o = o0 + a, lp = opt[a], p = p0 + lp;
        const double* jr = buf + a * JS;
        const double* q = pd + lp * PD;
        const size_t nc = ne + 6 * (size_t)obs_cam[o];
        const double sp[3] = {scale[3 * (size_t)p], scale[3 * (size_t)p + 1], scale[3 * (size_t)p + 2]};
        double je[2][3];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int u = 0; u < 3; ++u) { je[j][u] = jr[2 + 3 * j + u] * sp[u]; r1[3 * j + u] = je[j][u]; }
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double v = jr[8 + 6 * j + i] * scale[nc + i];
                r1[12 + 6 * j + i] = v;
                r2[6 * j + i] = v;
            }
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const double v = jr[20 + K * j + i] * si[i];
                r1[24 + K * j + i] = v;
                r2[12 + K * j + i] = v;
            }
        }
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int j = 0; j < 2; ++j) r1[6 + u * 2 + j] = q[u * 3] * je[j][0] + q[u * 3 + 1] * je[j][1] + q[u * 3 + 2] * je[j][2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                r2[12 + 2 * K + K * j + i] = je[j][0] * q[12 + i] + je[j][1] * q[12 + K + i] + je[j][2] * q[12 + 2 * K + i];
            const double qj = je[j][0] * q[9] + je[j][1] * q[10] + je[j][2] * q[11];
            r2[12 + 4 * K + j] = jr[j] - qj;
        }
    }
    __syncthreads();   // every J read is done: buf is free
    // 4. R1 (point-major, contiguous for the group) through LDS
    if (a < no) {
#pragma unroll
        for (int i = 0; i < RS1; ++i) buf[a * RS1 + i] = r1[i];
    }
    __syncthreads();
    {
        const double2* src = reinterpret_cast<const double2*>(buf);
        double2* dst = reinterpret_cast<double2*>(R1 + (size_t)o0 * RS1);
        for (int i = tid; i < no * (RS1 / 2); i += 256) dst[i] = src[i];
    }
    __syncthreads();
    if (a < no) {
#pragma unroll
        for (int i = 0; i < RS2; ++i) buf[a * RS2 + i] = r2[i];
    }
    __syncthreads();
    {   // R2 records at their camera-major slots, RS2/2 lanes per record
        const double2* src = reinterpret_cast<const double2*>(buf);
        for (int i = tid; i < no * (RS2 / 2); i += 256) {
            const int rec = i / (RS2 / 2), e = i - rec * (RS2 / 2);
            reinterpret_cast<double2*>(R2 + (size_t)campos[o0 + rec] * RS2)[e] = src[i];
        }
    }
#pragma unroll
    for (int i = 0; i < K * K; ++i) {
        const double s = block_sum(VZ[i], sh);
        if (threadIdx.x == 0) vzpart[(size_t)blockIdx.x * K * K + i] = s;
    }
}

// Per camera c (one block) over its contiguous R2 records:
// Scc = sum Jc^T Jc (6x6), Spi = sum Jc^T (Ji - T) (6xK), rc = sum Jc^T (r - q);
// per-camera partials of sum Ji^T Ji (upper KxK) and sum Ji^T (r - q) (K).
template <int K>
__global__ __launch_bounds__(256)
void ba_cam_blocks(int C, const int* __restrict__ cam_start, const double* __restrict__ R2, double* __restrict__ Scc,
                   double* __restrict__ Spi, double* __restrict__ rc, double* __restrict__ ipart) {
    __shared__ double sh[8];
    constexpr int NV = 21 + 6 * K + 6 + (K * (K + 1)) / 2 + K;   // upper 6x6, 6xK, 6, upper KxK, K
    constexpr int NI = (K * (K + 1)) / 2 + K;
    const int c = blockIdx.x;
    double v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = 0.0;
    for (int a = cam_start[c] + threadIdx.x; a < cam_start[c + 1]; a += blockDim.x) {
        const double* r2 = R2 + (size_t)a * r2s(K);
        double jc[2][6], ji[2][K], T[2][K], rq[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int i = 0; i < 6; ++i) jc[j][i] = r2[6 * j + i];
#pragma unroll
            for (int i = 0; i < K; ++i) { ji[j][i] = r2[12 + K * j + i]; T[j][i] = r2[12 + 2 * K + K * j + i]; }
            rq[j] = r2[12 + 4 * K + j];
        }
        int e = 0;
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
            for (int w = u; w < 6; ++w) v[e++] += jc[0][u] * jc[0][w] + jc[1][u] * jc[1][w];
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
            for (int i = 0; i < K; ++i) v[e++] += jc[0][u] * (ji[0][i] - T[0][i]) + jc[1][u] * (ji[1][i] - T[1][i]);
#pragma unroll
        for (int u = 0; u < 6; ++u) v[e++] += jc[0][u] * rq[0] + jc[1][u] * rq[1];
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int l = i; l < K; ++l) v[e++] += ji[0][i] * ji[0][l] + ji[1][i] * ji[1][l];
#pragma unroll
        for (int i = 0; i < K; ++i) v[e++] += ji[0][i] * rq[0] + ji[1][i] * rq[1];
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const double s = block_sum(v[i], sh);
        if (threadIdx.x == 0) {
            if (i < 21) {
                int u = 0, e = i;
                while (e >= 6 - u) { e -= 6 - u; ++u; }
                const int w = u + e;
                Scc[36 * (size_t)c + u * 6 + w] = s;
                Scc[36 * (size_t)c + w * 6 + u] = s;
            } else if (i < 21 + 6 * K) {
                Spi[(size_t)c * 6 * K + (i - 21)] = s;
            } else if (i < 27 + 6 * K) {
                rc[6 * (size_t)c + (i - 21 - 6 * K)] = s;
            } else {
                ipart[(size_t)c * NI + (i - 27 - 6 * K)] = s;
            }
        }
    }
}

// Intrinsics block, one 256-thread block per output (fixed-order tree sums):
// outputs 0..K*K-1: Sii = sum_c JiJi - sym(sum_blocks V^T Einv V); K*K..K*K+K-1: ri.
template <int K>
__global__ __launch_bounds__(256)
void ba_intr_final(int C, int nvz, const double* __restrict__ ipart, const double* __restrict__ vzpart,
                   double* __restrict__ Sii, double* __restrict__ ri) {
    __shared__ double sh[8];
    constexpr int NI = (K * (K + 1)) / 2 + K;
    const int t = blockIdx.x;
    if (t < K * K) {
        const int i = t / K, l = t % K;
        const int a = i < l ? i : l, b = i < l ? l : i;
        int e = 0;
        for (int u = 0; u < a; ++u) e += K - u;
        e += b - a;
        double s = 0.0, z = 0.0;
        for (int c = threadIdx.x; c < C; c += blockDim.x) s += ipart[(size_t)c * NI + e];
        for (int bk = threadIdx.x; bk < nvz; bk += blockDim.x)
            z += 0.5 * (vzpart[(size_t)bk * K * K + i * K + l] + vzpart[(size_t)bk * K * K + l * K + i]);
        const double tot = block_sum(s - z, sh);
        if (threadIdx.x == 0) Sii[t] = tot;
    } else {
        const int i = t - K * K;
        double s = 0.0;
        for (int c = threadIdx.x; c < C; c += blockDim.x) s += ipart[(size_t)c * NI + (K * (K + 1)) / 2 + i];
        const double tot = block_sum(s, sh);
        if (threadIdx.x == 0) ri[i] = tot;
    }
}

// Pose blocks: for block b = (c1 <= c2) with its segment of ordered observation
// pairs (o1 in c1, o2 in c2, same point):
//   Spp_b = - sum Jc_s(o1)^T [Je_s(o1) U(o2)] Jc_s(o2)     (U = Einv Je_s^T)
// one workgroup per block, fixed-order tree sum (deterministic); R1 gathers.
template <int K>
__global__ __launch_bounds__(256)
void ba_pair_blocks(const int* __restrict__ blk_start, const int2* __restrict__ trip, const double* __restrict__ R1,
                    double* __restrict__ Spp) {
    __shared__ double sh[8];
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    double acc[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) acc[i] = 0.0;
    for (int t = blk_start[b] + threadIdx.x; t < blk_start[b + 1]; t += blockDim.x) {
        const int2 tr = trip[t];
        const double* x1 = R1 + (size_t)tr.x * r1s(K);
        const double* x2 = R1 + (size_t)tr.y * r1s(K);
        double je1[6], u2[6], a1[12], a2[12];
#pragma unroll
        for (int i = 0; i < 6; ++i) { je1[i] = x1[i]; u2[i] = x2[6 + i]; }
#pragma unroll
        for (int i = 0; i < 12; ++i) { a1[i] = x1[12 + i]; a2[i] = x2[12 + i]; }
        double M[2][2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int l = 0; l < 2; ++l) M[j][l] = je1[3 * j] * u2[l] + je1[3 * j + 1] * u2[2 + l] + je1[3 * j + 2] * u2[4 + l];
        double T[2][6];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 6; ++i) T[j][i] = M[j][0] * a2[i] + M[j][1] * a2[6 + i];
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
            for (int w = 0; w < 6; ++w) acc[u * 6 + w] += a1[u] * T[0][w] + a1[6 + u] * T[1][w];
    }
#pragma unroll
    for (int i = 0; i < 36; ++i) {
        const double s = block_sum(acc[i], sh);
        if (threadIdx.x == 0) Spp[36 * (size_t)b + i] = -s;
    }
}

// Dense reduced camera system, row-major npad x npad (npad multiple of NB),
// assembled by three ordered launches over a zeroed S (no two workgroups of one
// launch touch the same element):
//   ba_assemble_pairs  Spp(c1,c2) into the (c1,c2) block and its transpose
//   ba_assemble_diag   += Scc on each pose diagonal block
//   ba_assemble_rest   pose-intrinsics Spi, intrinsics Sii, + D^2 on the
//                      diagonal (added once, after any cross-rank all-reduce),
//                      identity on the padding, rhs = [rc ; ri].
__global__ void ba_assemble_pairs(int npad, const int* __restrict__ blk_cam, const double* __restrict__ Spp,
                                  double* __restrict__ S) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (t >= 36) return;
    const int u = t / 6, w = t % 6;
    const int c1 = blk_cam[2 * b], c2 = blk_cam[2 * b + 1];
    const double v = Spp[36 * (size_t)b + t];
    S[(size_t)(6 * c1 + u) * npad + 6 * c2 + w] = v;
    if (c1 != c2) S[(size_t)(6 * c2 + w) * npad + 6 * c1 + u] = v;
}

__global__ void ba_assemble_diag(int npad, const double* __restrict__ Scc, double* __restrict__ S) {
    const int c = blockIdx.x, t = threadIdx.x;
    if (t >= 36) return;
    const int u = t / 6, w = t % 6;
    S[(size_t)(6 * c + u) * npad + 6 * c + w] += Scc[36 * (size_t)c + t];
}

__global__ void ba_assemble_rest(int C, int K, int nf, int npad, const double* __restrict__ Spi,
                                 const double* __restrict__ Sii, const double* __restrict__ rc,
                                 const double* __restrict__ ri, double* __restrict__ S, double* __restrict__ rhs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npad) return;
    if (i < 6 * C) {
        const int c = i / 6, u = i % 6;
        for (int l = 0; l < K; ++l) {
            const double v = Spi[(size_t)c * 6 * K + u * K + l];
            S[(size_t)i * npad + 6 * C + l] = v;
            S[(size_t)(6 * C + l) * npad + i] = v;
        }
        rhs[i] = rc[i];
    } else if (i < nf) {
        const int l = i - 6 * C;
        for (int m = 0; m < K; ++m) S[(size_t)i * npad + 6 * C + m] = Sii[l * K + m];
        rhs[i] = ri[l];
    } else {
        S[(size_t)i * npad + i] = 1.0;
        rhs[i] = 0.0;
    }
}

// + D_f^2 on the reduced system's diagonal (after the cross-rank all-reduce).
__global__ void ba_add_damping(int P, int nf, int npad, const double* __restrict__ D, double* __restrict__ S) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const double d = D[3 * (size_t)P + i];
    S[(size_t)i * npad + i] += d * d;
}

// ---- dense factorisation of the reduced camera system, NB x NB tiles -----
// Block LDL^T, right-looking, one launch per panel: A = L~ D~ L~^T with
// D~_k the (updated) diagonal tile and L~_ak = A_ak W_k, W_k = D~_k^-1.  A
// pivot of D~_k is a pivot of the scalar Cholesky, so "not positive definite"
// is detected exactly where LLT (Ceres DENSE_SCHUR) fails.  Storage in S
// (row-major, npad x npad):
//   lower tiles (a, b), a > b : A, updated in place until consumed
//   upper tile (k, a), a > k  : L~_ak^T (for the back solve)
// W_k lives in a ping-pong buffer; rhs is overwritten with w = D~^-1 L~^-1 b
// during the factorisation, then with x by the back solve.
constexpr int LDT = NB + 2;   // LDS row stride (doubles): 16-B aligned rows
typedef double f64x4 __attribute__((ext_vector_type(4)));

// 64x64 fp64 tiles on the matrix cores: v_mfma_f64_16x16x4f64 (operands: lane
// m + 16k holds A[m][k] and B[k][n = m]; result register r of lane l is
// D[l/16 + 4r][l%16], checked by tools/micro/mfma_f64_layout.hip).  Wave w of
// the 256-thread block owns the row strip 16w..16w+15 and four 16x16 column
// tiles: acc[c][r] = out[16w + l/16 + 4r][16c + l%16].
__device__ __forceinline__ int trow(int r) { return ((threadIdx.x & 63) >> 4) + 4 * r; }   // row in the strip
__device__ __forceinline__ int tcol() { return threadIdx.x & 15; }

__device__ __forceinline__ void tile_load(double (*dst)[LDT], const double* __restrict__ src, int ld) {
#pragma unroll
    for (int q = 0; q < NB * NB / 512; ++q) {
        const int e = q * 512 + 2 * threadIdx.x;
        *reinterpret_cast<double2*>(&dst[e / NB][e % NB]) = *reinterpret_cast<const double2*>(src + (size_t)(e / NB) * ld + e % NB);
    }
}

// acc[c] = A[strip] * B          (A, B row-major 64x64 in LDS)
__device__ __forceinline__ void mfma_nn(const double (*A)[LDT], const double (*B)[LDT], f64x4 acc[4]) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, m = l & 15, kq = l >> 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int st = 0; st < NB / 4; ++st) {
        const double av = A[16 * w + m][4 * st + kq];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, B[4 * st + kq][16 * c + m], acc[c], 0, 0, 0);
    }
}
// acc[c] = A[strip] * X^T        (A, X row-major 64x64 in LDS)
__device__ __forceinline__ void mfma_nt(const double (*A)[LDT], const double (*X)[LDT], f64x4 acc[4]) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, m = l & 15, kq = l >> 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int st = 0; st < NB / 4; ++st) {
        const double av = A[16 * w + m][4 * st + kq];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, X[16 * c + m][4 * st + kq], acc[c], 0, 0, 0);
    }
}

// 1/d: hardware estimate + two Newton steps (within an ulp or so of the divide).
__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

// W_k = D~_k^-1 by symmetric block sweeps.  Sweeping the pivot block B with
// Q = A_BB^-1:  a_il -= A_iB Q A_Bl (i, l not in B), A_iB <- A_iB Q,
// A_Bl <- Q A_Bl, A_BB <- -Q; after all blocks the tile holds -A^-1.
// Two levels (256 threads, the tile in registers in the MFMA layout above):
//   outer: 4 sweeps of 16-wide pivot blocks — the column panel A_:B goes
//          through LDS; M = A_:B Q (per wave, its own strip) and the rank-16
//          update of the other column tiles run on the fp64 matrix cores;
//   inner: Qn = -A_BB^-1 (16x16) by wave 0 alone (no barriers): 8 sweeps of
//          2x2 pivot blocks, each lane holding a 2x2 block; the 2x2 pivot
//          inverse is closed-form and its two scalar pivots (a, det/a) are the
//          scalar Cholesky pivots, i.e. exactly where LLT would fail.
// Then rhs_k <- W_k rhs_k.
constexpr int LDP = 18;   // LDS row stride of the 16-wide panels (16-B aligned rows)
#ifdef SFMX_CHOL_STAMPS   // tools/micro/chol_tile.hip: phase timestamps of block 0 (never in the product build)
__device__ long long g_chol_stamps[64];
#define CHOL_STAMP(i) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_chol_stamps[i] = wall_clock64(); } while (0)
#else
#define CHOL_STAMP(i) do { } while (0)
#endif

__device__ __forceinline__ void inner_inverse16(const double* __restrict__ Pc, int s, double* __restrict__ Qn,
                                                double* __restrict__ ipan, bool& bad) {
    // wave 0 only: Qn = -(Pc[16s + i][j])^-1, i, j < 16
    const int lane = threadIdx.x & 63, r = lane >> 3, c = lane & 7;
    double p[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int w = 0; w < 2; ++w) p[u][w] = Pc[(16 * s + 2 * r + u) * LDP + 2 * c + w];
    for (int j = 0; j < 8; ++j) {
        if (c == j) {   // column panel of the pivot block: rows 2r.., cols 2j..
            *reinterpret_cast<double2*>(&ipan[(2 * r) * 2]) = make_double2(p[0][0], p[0][1]);
            *reinterpret_cast<double2*>(&ipan[(2 * r + 1) * 2]) = make_double2(p[1][0], p[1][1]);
        }
        __builtin_amdgcn_wave_barrier();
        const double2 b0 = *reinterpret_cast<const double2*>(&ipan[(2 * j) * 2]);
        const double2 b1 = *reinterpret_cast<const double2*>(&ipan[(2 * j + 1) * 2]);
        const double2 i0 = *reinterpret_cast<const double2*>(&ipan[(2 * r) * 2]);
        const double2 i1 = *reinterpret_cast<const double2*>(&ipan[(2 * r + 1) * 2]);
        const double2 l0 = *reinterpret_cast<const double2*>(&ipan[(2 * c) * 2]);
        const double2 l1 = *reinterpret_cast<const double2*>(&ipan[(2 * c + 1) * 2]);
        __builtin_amdgcn_wave_barrier();
        // q = -[a b; b d]^-1
        const double a = b0.x, bb = b0.y, d = b1.y;
        double det = fma(a, d, -bb * bb);
        if (!(a > 0.0) || !isfinite(a) || !(det > 0.0) || !isfinite(det)) { bad = true; det = 1.0; }
        const double rd = rcp_nr(det);
        const double q00 = -d * rd, q01 = bb * rd, q11 = -a * rd;   // q10 = q01
        const bool rowB = (r == j), colB = (c == j);
        double m[2][2];
        {
            const double ai[2][2] = {{i0.x, i0.y}, {i1.x, i1.y}};
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const double v0 = -(ai[u][0] * q00 + ai[u][1] * q01), v1 = -(ai[u][0] * q01 + ai[u][1] * q11);
                m[u][0] = rowB ? (u == 0 ? q00 : q01) : v0;
                m[u][1] = rowB ? (u == 0 ? q01 : q11) : v1;
            }
        }
        const double al[2][2] = {{l0.x, l0.y}, {l1.x, l1.y}};   // al[w][b] = A_(2c+w),(2j+b) = A_Bl[b][w]
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                if (colB) p[u][w] = m[u][w];
                else p[u][w] = (rowB ? 0.0 : p[u][w]) - (m[u][0] * al[w][0] + m[u][1] * al[w][1]);
            }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int w = 0; w < 2; ++w) Qn[(2 * r + u) * LDP + 2 * c + w] = p[u][w];
}

// t: the (updated) diagonal tile k in registers (MFMA layout); rk: rhs_k in LDS.
// workspace: >= 2624 doubles of LDS (buf = 64 x LDT)
__device__ __forceinline__ void chol_diag_tile(f64x4 (&t)[4], int k, double* __restrict__ Wout,
                                               double* __restrict__ rhs, const double* __restrict__ rk,
                                               int* __restrict__ fail, double (*buf)[LDT]) {
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, m = l & 15, kq = l >> 4, k0 = k * NB;
    double* ws = &buf[0][0];
    double* Pc = ws;                       // [64][LDP]  column panel A_:B
    double* Qn = ws + NB * LDP;            // [16][LDP]  -A_BB^-1
    double* ipan = Qn + 16 * LDP;          // [16][2]    inner column panel
    double* Mw = ipan + 32 + 16 * LDP * w; // [16][LDP]  this wave's -M strip
    CHOL_STAMP(0);
    bool bad = false;
    CHOL_STAMP(1);
#pragma unroll
    for (int s = 0; s < NB / 16; ++s) {
        const bool rowB = (w == s);
#pragma unroll
        for (int r = 0; r < 4; ++r) Pc[(16 * w + trow(r)) * LDP + tcol()] = t[s][r];
        __syncthreads();
        CHOL_STAMP(2 + 4 * s);
        if (tid < 64) inner_inverse16(Pc, s, Qn, ipan, bad);
        __syncthreads();
        CHOL_STAMP(3 + 4 * s);
        // M = A_(strip),B Q on the matrix cores; rows in B take Q itself (-Qn)
        f64x4 mm = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 4; ++st)
            mm = __builtin_amdgcn_mfma_f64_16x16x4f64(Pc[(16 * w + m) * LDP + 4 * st + kq], Qn[(4 * st + kq) * LDP + m], mm, 0, 0, 0);
        f64x4 mv;
#pragma unroll
        for (int r = 0; r < 4; ++r) mv[r] = rowB ? Qn[trow(r) * LDP + tcol()] : -mm[r];   // M (Qn = -Q)
        t[s] = mv;                                                         // A_iB <- A_iB Q, A_BB <- -Q
#pragma unroll
        for (int r = 0; r < 4; ++r) Mw[trow(r) * LDP + tcol()] = -mv[r];   // -M as the A operand
        __builtin_amdgcn_wave_barrier();
        CHOL_STAMP(4 + 4 * s);
        // a_il -= M[i][:] A_l,B for the other column tiles (rows in B start from 0)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c == s) continue;
            f64x4 acc = rowB ? f64x4{0.0, 0.0, 0.0, 0.0} : t[c];
#pragma unroll
            for (int st = 0; st < 4; ++st)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Mw[m * LDP + 4 * st + kq], Pc[(16 * c + m) * LDP + 4 * st + kq], acc, 0, 0, 0);
            t[c] = acc;
        }
        __syncthreads();   // Pc is rewritten by the next sweep
        CHOL_STAMP(5 + 4 * s);
    }
    if (bad) atomicOr(fail, 1);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * w + trow(r), j = 16 * c + tcol();
            buf[i][j] = -t[c][r];
            Wout[i * NB + j] = -t[c][r];
        }
    __syncthreads();
    CHOL_STAMP(20);
    {   // rhs_k <- W_k rhs_k: 4 threads per row, 16 terms each
        const int i = tid >> 2, q = tid & 3;
        double sum = 0.0;
#pragma unroll
        for (int c = 0; c < 16; ++c) sum = fma(buf[i][4 * c + q], rk[4 * c + q], sum);
        sum += __shfl_xor(sum, 1);
        sum += __shfl_xor(sum, 2);
        if (q == 0) rhs[k0 + i] = sum;
    }
    CHOL_STAMP(21);
}

struct alignas(16) CholLds {
    double a[NB][LDT], m[NB][LDT], n[NB][LDT];
    double rk[NB], ra[NB];   // rhs_k (= w_k after panel k's inverse), rhs_a
};

__device__ __forceinline__ void tile_regs(f64x4 (&t)[4], const double* __restrict__ src, int ld) {
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) t[c][r] = src[(size_t)(16 * w + trow(r)) * ld + 16 * c + tcol()];
}

__global__ __launch_bounds__(256)
void chol_first(double* __restrict__ S, int npad, double* __restrict__ W, double* __restrict__ rhs,
                int* __restrict__ fail) {
    __shared__ CholLds sm;
    f64x4 t[4];
    tile_regs(t, S, npad);
    if (threadIdx.x < NB) sm.rk[threadIdx.x] = rhs[threadIdx.x];
    __syncthreads();
    chol_diag_tile(t, 0, W, rhs, sm.rk, fail, sm.a);
}

// Panel k: one block per trailing lower tile (a, b), k < b <= a.  Block 0 is
// (k+1, k+1); after its update it inverts that tile for panel k+1 (its updated
// value never goes back to S: only W_{k+1} is needed later).
//   G = A_ak W_k
//   b <  a : A_ab -= G A_bk^T
//   b == a : A_aa -= G A_ak^T;  G^T -> upper tile (k, a);  rhs_a -= A_ak w_k
// The destination tile is prefetched into registers before the GEMMs.
__global__ __launch_bounds__(256)
void chol_step(double* __restrict__ S, int npad, int k, double* __restrict__ W, double* __restrict__ rhs,
               int* __restrict__ fail, const int2* __restrict__ tl) {
    __shared__ CholLds sm;
    const int tid = threadIdx.x, w = tid >> 6;
    int a = k + 1, b = k + 1;
    if (tl) {               // tile-sparse: this step's structurally nonzero updates, tl[0] = (k+1, k+1)
        const int2 ab = tl[blockIdx.x];
        a = ab.x; b = ab.y;
    } else if (blockIdx.x > 0) {   // dense: tile rows a >= k + 2 hold a - k tiles (b = k+1 .. a)
        int rem = blockIdx.x - 1;
        for (a = k + 2; rem >= a - k; ++a) rem -= a - k;
        b = k + 1 + rem;
    }
    const int k0 = k * NB, a0 = a * NB, b0 = b * NB;
    const bool diagblk = (a == b);
    CHOL_STAMP(30);
    f64x4 t[4];
    double* dst = S + (size_t)a0 * npad + b0;
    tile_regs(t, dst, npad);                                             // A_ab (prefetch)
    tile_load(sm.a, S + (size_t)a0 * npad + k0, npad);                   // A_ak
    tile_load(sm.m, W + (size_t)(k & 1) * NB * NB, NB);                  // W_k
    if (!diagblk) tile_load(sm.n, S + (size_t)b0 * npad + k0, npad);     // A_bk
    else if (tid < NB) { sm.rk[tid] = rhs[k0 + tid]; sm.ra[tid] = rhs[a0 + tid]; }
    __syncthreads();
    CHOL_STAMP(31);
    f64x4 g[4];
    mfma_nn(sm.a, sm.m, g);   // G = A_ak W_k
    __syncthreads();
    CHOL_STAMP(32);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.m[16 * w + trow(r)][16 * c + tcol()] = g[c][r];
    __syncthreads();
    f64x4 upd[4];
    mfma_nt(sm.m, diagblk ? sm.a : sm.n, upd);   // G X^T
#pragma unroll
    for (int c = 0; c < 4; ++c) t[c] -= upd[c];
    CHOL_STAMP(33);
    if (diagblk) {
        {   // rhs_a -= A_ak w_k: 4 threads per row
            const int i = tid >> 2, q = tid & 3;
            double sum = 0.0;
#pragma unroll
            for (int c = 0; c < 16; ++c) sum = fma(sm.a[i][4 * c + q], sm.rk[4 * c + q], sum);
            sum += __shfl_xor(sum, 1);
            sum += __shfl_xor(sum, 2);
            if (q == 0) sm.ra[i] -= sum;
        }
        __syncthreads();
        if (blockIdx.x == 0) chol_diag_tile(t, k + 1, W + (size_t)((k + 1) & 1) * NB * NB, rhs, sm.ra, fail, sm.n);
        else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int r = 0; r < 4; ++r) dst[(size_t)(16 * w + trow(r)) * npad + 16 * c + tcol()] = t[c][r];
            if (tid < NB) rhs[a0 + tid] = sm.ra[tid];
        }
        // upper tile (k, a): row k0 + j, column a0 + i holds G[i][j]
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) S[(size_t)(k0 + 16 * c + tcol()) * npad + a0 + 16 * w + trow(r)] = g[c][r];
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(size_t)(16 * w + trow(r)) * npad + 16 * c + tcol()] = t[c][r];
    }
    CHOL_STAMP(34);
}

// Back substitution L~^T x = w, panel k (descending): x_k = rhs_k is final;
// block 0 stores it (rows < nf) into xout, every block i < k does
// rhs_i -= L~_ki^T x_k (upper tile (i, k)).
__global__ __launch_bounds__(256)
void chol_back(const double* __restrict__ S, int npad, int nf, int k, double* __restrict__ rhs,
               double* __restrict__ xout) {
    __shared__ double xk[NB];
    const int tid = threadIdx.x, k0 = k * NB;
    if (tid < NB) {
        const double v = rhs[k0 + tid];
        xk[tid] = v;
        if (blockIdx.x == 0 && k0 + tid < nf) xout[k0 + tid] = v;
    }
    __syncthreads();
    if (blockIdx.x >= k) return;
    const int i0 = blockIdx.x * NB, r = tid >> 2, qq = tid & 3;
    const double* U = S + (size_t)(i0 + r) * npad + k0;
    double t = 0.0;
#pragma unroll 4
    for (int m = 0; m < NB / 4; ++m) t = fma(U[4 * m + qq], xk[4 * m + qq], t);
    t += __shfl_xor(t, 1);
    t += __shfl_xor(t, 2);
    if (qq == 0) rhs[i0 + r] -= t;
}

// Tile-sparse back substitution L~^T x = w in one workgroup: panels descending; for panel k only
// the structurally nonzero upper tiles (i, k), i < k (list ut[ut_start[k] .. ut_start[k+1])) update
// rhs_i -= U(i, k) x_k.  rhs lives in LDS (npad <= 16384).
__global__ __launch_bounds__(256)
void chol_back_sparse(const double* __restrict__ S, int npad, int nf, int T, const double* __restrict__ rhs_in,
                      const int* __restrict__ ut_start, const int* __restrict__ ut, double* __restrict__ xout) {
    extern __shared__ double r[];
    const int tid = threadIdx.x;
    for (int i = tid; i < npad; i += 256) r[i] = rhs_in[i];
    __syncthreads();
    for (int k = T - 1; k >= 0; --k) {
        const int k0 = k * NB;
        for (int i = tid; i < NB; i += 256)
            if (k0 + i < nf) xout[k0 + i] = r[k0 + i];
        const int e0 = ut_start[k], e1 = ut_start[k + 1];
        // 4 threads per row, 64 rows per pass over the listed tiles' rows
        for (int e = e0; e < e1; ++e) {
            const int i0 = ut[e] * NB, rr = tid >> 2, qq = tid & 3;
            const double* U = S + (size_t)(i0 + rr) * npad + k0;
            double t = 0.0;
#pragma unroll
            for (int m = 0; m < NB / 4; ++m) t = fma(U[4 * m + qq], r[k0 + 4 * m + qq], t);
            t += __shfl_xor(t, 1);
            t += __shfl_xor(t, 2);
            if (qq == 0) r[i0 + rr] -= t;
        }
        __syncthreads();
    }
}

// x_e = EinvG - sum_o U_o (F_o x_f), F_o = [Jc_s | Ji_s]   (R1 records)
template <int K>
__global__ __launch_bounds__(256)
void ba_backsub(int P, int C, const int* __restrict__ pt_start, const int* __restrict__ pt_obs,
                const int* __restrict__ obs_cam, const double* __restrict__ R1, const double* __restrict__ EinvG,
                const double* __restrict__ xf, double* __restrict__ xe) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    double xi[K];
#pragma unroll
    for (int i = 0; i < K; ++i) xi[i] = xf[6 * C + i];
    double v[3] = {EinvG[3 * (size_t)p], EinvG[3 * (size_t)p + 1], EinvG[3 * (size_t)p + 2]};
    for (int a = pt_start[p]; a < pt_start[p + 1]; ++a) {
        const int o = pt_obs[a], c = obs_cam[o];
        const double* r1 = R1 + (size_t)o * r1s(K);
        double f[2] = {0, 0};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int i = 0; i < 6; ++i) f[j] += r1[12 + 6 * j + i] * xf[6 * c + i];
#pragma unroll
            for (int i = 0; i < K; ++i) f[j] += r1[24 + K * j + i] * xi[i];
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) v[u] -= r1[6 + u * 2] * f[0] + r1[6 + u * 2 + 1] * f[1];
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) xe[3 * (size_t)p + u] = v[u];
}

// step_s = -sol; delta = step_s * scale; cand = x + delta; partials of ||delta||^2 and finiteness.
__global__ __launch_bounds__(256)
void ba_step(int n, const double* __restrict__ sol, const double* __restrict__ scale, const double* __restrict__ x,
             double* __restrict__ step, double* __restrict__ cand, double* __restrict__ part) {
    __shared__ double sh[8];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double d2 = 0.0;
    if (i < n) {
        const double st = -sol[i];
        step[i] = st;
        const double d = st * scale[i];
        cand[i] = x[i] + d;
        d2 = isfinite(d) ? (x[i] - cand[i]) * (x[i] - cand[i]) : INFINITY;
    }
    const double s = block_sum(d2, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// model cost change partials: sum_o m . (r + m/2), m = J_s step
template <int K>
__global__ __launch_bounds__(256)
void ba_model(int P, int O, int C, const int* __restrict__ obs_point, const int* __restrict__ obs_cam,
              const double* __restrict__ J, const double* __restrict__ scale, const double* __restrict__ step,
              double* __restrict__ part) {
    __shared__ double sh[8];
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t ne = 3 * (size_t)P;
    double acc = 0.0;
    if (o < O) {
        const int p = obs_point[o], c = obs_cam[o];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            double m = 0;
#pragma unroll
            for (int i = 0; i < 3; ++i) m += J[(size_t)o * jst(K) + (2 + 3 * j + i)] * scale[3 * (size_t)p + i] * step[3 * (size_t)p + i];
#pragma unroll
            for (int i = 0; i < 6; ++i) m += J[(size_t)o * jst(K) + (8 + 6 * j + i)] * scale[ne + 6 * (size_t)c + i] * step[ne + 6 * (size_t)c + i];
#pragma unroll
            for (int i = 0; i < K; ++i) m += J[(size_t)o * jst(K) + (20 + K * j + i)] * scale[ne + 6 * (size_t)C + i] * step[ne + 6 * (size_t)C + i];
            acc += m * (J[(size_t)o * jst(K) + j] + m / 2.0);
        }
    }
    const double s = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256)
void ba_sumsq(int n, const double* __restrict__ x, double* __restrict__ part) {
    __shared__ double sh[8];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const double v = i < n ? x[i] * x[i] : 0.0;
    const double s = block_sum(v, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

}  // namespace ba
}  // namespace sfmx
