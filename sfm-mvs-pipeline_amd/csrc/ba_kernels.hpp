// SPDX-License-Identifier: MIT
// sfmx bundle adjustment kernels for gfx950 (MI355X / CDNA4), fp64.
//
// Shared pieces of the Levenberg-Marquardt solver of the reference's Ceres problem
// (BundleAdjustment.cpp:29-91 solved by CeresUtils::solve, DENSE_SCHUR):
//   DJet / project    forward-mode dual numbers and the reference functors' arithmetic (what
//                     ceres::AutoDiffCostFunction evaluates for SimpleRadialCamera.cpp:79-115,
//                     SimpleCamera.cpp:73-103, DistortionCamera.cpp:72-110)
//   ba_linearize      residual + Jacobian of every observation (sfmx_ba_jacobian); the solver's
//                     own linearization is fused into the point-group kernels (ba_group.hpp)
//   ba_sum, ba_scale  deterministic sums, Jacobi scaling
// Layout in HBM: parameters x = [points 3P | poses 6C | intrinsics k]; the Jacobian record of
// an observation is J[o][f] (f = r0,r1, Je 2x3, Jc 2x6, Ji 2xk, stride jst(K) = 20 + 2k).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cfloat>

namespace sfmx {
namespace ba {

// LM scalars of one step (ba_finalize -> host / ba_decide)
enum { SC_COST = 0, SC_MODEL = 1, SC_STEPN = 2, SC_XN = 3, SC_GMAX = 4, SC_FAIL = 5, SC_STEPN_F = 6, SC_XN_F = 7, SC_N = 8 };
// Tile of the reduced camera system (ba_chol.hpp, ba_plan.hpp PLAN_NB): NB x NB, factored by
// workgroups of NW = NB / 16 waves (NTH threads), wave w owning the 16-row strip 16w.
#ifndef SFMX_BA_NB
#define SFMX_BA_NB 64
#endif
constexpr int NB = SFMX_BA_NB;
constexpr int NW = NB / 16, NTH = 64 * NW;
static_assert(NB == 32 || NB == 64, "tile size 32 or 64");
__host__ __device__ constexpr int jst(int K) { return 20 + 2 * K; }   // Jacobian record stride

// fp64 matrix-core tiles: v_mfma_f64_16x16x4f64 (operands: lane m + 16k holds A[m][k] and
// B[k][n = m]; result register r of lane l is D[l/16 + 4r][l%16], checked by
// tools/micro/mfma_f64_layout.hip).  Wave w of a 256-thread block owns the row strip
// 16w..16w+15: acc[c][r] = out[16w + l/16 + 4r][16c + l%16].
typedef double f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int trow(int r) { return ((threadIdx.x & 63) >> 4) + 4 * r; }   // row in the strip
__device__ __forceinline__ int tcol() { return threadIdx.x & 15; }

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

// Several cameras (BundleAdjustment.cpp:81-89: each residual takes its shot's camera block):
// the intrinsics columns of x are the border [0, K) holding every referenced block back to
// back.  Per pose, pim = model | (first border column << 4) and pcc = the block's (cx, cy).
// The observation's own block enters the jets at derivative slots 9 + off ..; every other
// border column gets a zero derivative, so the J record's Ji row is the observation's block
// scattered into K columns.  Only models that fit the border are instantiated.
template <int K, int N>
__device__ __forceinline__ void project_blk(const DJet<N> X[3], const DJet<N> ps[6], const double* __restrict__ intr,
                                            int pim, double2 pcc, double ox, double oy, DJet<N> res[2]) {
    const int model = pim & 15, off = pim >> 4;
    if constexpr (K >= 7) {
        if (model == 7) {
            DJet<N> in[7];
#pragma unroll
            for (int i = 0; i < 7; ++i) in[i] = N ? jvar<N>(intr[off + i], 9 + off + i) : jconst<N>(intr[off + i]);
            project<7, N>(X, ps, in, ox, oy, pcc.x, pcc.y, res);
            return;
        }
    }
    if constexpr (K >= 3) {
        if (model == 3) {
            DJet<N> in[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) in[i] = N ? jvar<N>(intr[off + i], 9 + off + i) : jconst<N>(intr[off + i]);
            project<3, N>(X, ps, in, ox, oy, pcc.x, pcc.y, res);
            return;
        }
    }
    DJet<N> in[1];
    in[0] = N ? jvar<N>(intr[off], 9 + off) : jconst<N>(intr[off]);
    project<1, N>(X, ps, in, ox, oy, pcc.x, pcc.y, res);
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
                  double* __restrict__ partial, const int* __restrict__ pim, const double2* __restrict__ pcc) {
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
            if (pim) {
                project_blk<K, N>(X, ps, intr, pim[c], pcc[c], ox, oy, res);
            } else {
#pragma unroll
                for (int i = 0; i < K; ++i) in[i] = jvar<N>(intr[i], 9 + i);
                project<K, N>(X, ps, in, ox, oy, cx, cy, res);
            }
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
            if (pim) {
                project_blk<K, 0>(X, ps, intr, pim[c], pcc[c], ox, oy, res);
            } else {
#pragma unroll
                for (int i = 0; i < K; ++i) in[i].a = intr[i];
                project<K, 0>(X, ps, in, ox, oy, cx, cy, res);
            }
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

// The step gate (speculative LM, ba_solver.hip): every kernel of an LM step returns at once when
// the gate word is 0.  ba_decide sets it to 1 only when the step it judged was accepted and the
// minimisation continues, so the next step, enqueued by the host before it knows the outcome (with
// the accepted step's buffers), runs exactly then; after a rejection the host re-opens the gate and
// enqueues the step again on the unchanged buffers.  Outside the speculative mode it stays 1.
__device__ __forceinline__ bool step_gated(const int* __restrict__ gate) { return gate && *gate == 0; }

// LM controller state on the device (speculative mode), doubles so it publishes with the scalars.
enum { LM_COST = 0, LM_GMAX, LM_XNORM, LM_RADIUS, LM_DECREASE, LM_ITER, LM_SUCC, LM_UNSUCC, LM_INVALID, LM_CONSEC,
       LM_SUCCESSFUL, LM_TERM, LM_ACCEPTED, LM_TRACE, LM_ERROR, LM_N = 16 };
constexpr double LM_RUNNING = -1.0;
struct LmOpt {
    double ptol, ftol, minrel, maxr, gtol, minr;
    int maxit, maxinv, term_conv, term_noconv, term_fail;
};
// (2 rho - 1)^3 of the radius update (Ceres: std::pow(2 rho - 1, 3)): the cube with the errors of both
// products carried (fma) and one final rounding, so the host and the device get the same bits.
__host__ __device__ inline double lm_cube(double y) {
#pragma clang fp contract(off)   // host and device must not fuse t + ... into an fma differently
    const double p = y * y, pe = fma(y, y, -p);
    const double t = p * y, te = fma(p, y, -t);
    return t + fma(pe, y, te);
}

// The LM scalars into pinned, host-coherent memory, then the sequence number with system-scope
// release: the host polls the sequence number instead of a D2H copy + stream synchronisation
// (the interrupt-driven wake-up of hipStreamSynchronize costs ~50 us per LM step).
// It also clears the step's failure flag (already folded into the scalars by ba_finalize), so the
// next step starts without a separate memset.
__device__ __forceinline__ void publish_body(const double* __restrict__ src, int n, const double* __restrict__ src2,
                                             int n2, double* __restrict__ dst, unsigned* __restrict__ seq, unsigned v,
                                             int* __restrict__ fail) {
    for (int i = 0; i < n; ++i) dst[i] = src[i];
    for (int i = 0; i < n2; ++i) dst[n + i] = src2[i];
    *fail = 0;
    __threadfence_system();
    __hip_atomic_store(seq, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void ba_publish(const double* __restrict__ src, int n, double* __restrict__ dst, unsigned* __restrict__ seq,
                           unsigned v, int* __restrict__ fail) {
    if (threadIdx.x == 0) publish_body(src, n, nullptr, 0, dst, seq, v, fail);
}

// Speculative mode, the step's last kernel: Ceres 1.14 TrustRegionMinimizer +
// LevenbergMarquardtStrategy after one step (the host loop of run_lm_k, line for line): accept /
// reject / invalid, the radius update, then the next iteration's
// FinalizeIterationAndCheckIfMinimizerCanContinue; then the scalars + this state are published as
// ba_publish does and the gate for the next step is set.  scal holds the step's (all-reduced) scalars.
__global__ void ba_decide(const double* __restrict__ scal, double* __restrict__ lm, int* __restrict__ fail, LmOpt o,
                          double* __restrict__ dst, unsigned* __restrict__ seq, unsigned v) {
#pragma clang fp contract(off)   // the host loop's arithmetic, bit for bit
    if (threadIdx.x != 0 || step_gated(fail + 1)) return;
    double cost = lm[LM_COST], gmax = lm[LM_GMAX], xn = lm[LM_XNORM], radius = lm[LM_RADIUS], dec = lm[LM_DECREASE];
    int consec = (int)lm[LM_CONSEC];
    bool successful = lm[LM_SUCCESSFUL] != 0.0, accepted = false, trace = false;
    double term = LM_RUNNING;
    const double sn2 = scal[SC_STEPN] + scal[SC_STEPN_F], mcc = -scal[SC_MODEL], sn = sqrt(sn2);
    const bool valid = scal[SC_FAIL] == 0.0 && isfinite(sn2) && isfinite(scal[SC_MODEL]) && mcc > 0.0;
    if (scal[SC_FAIL] >= 2.0) {   // internal error (a dependency wait timed out)
        lm[LM_ERROR] = 1.0;
        term = o.term_fail;
    } else if (!valid) {          // HandleInvalidStep
        lm[LM_INVALID] += 1.0;
        if (++consec >= o.maxinv) term = o.term_fail;
        else { radius /= dec; dec *= 2.0; successful = false; }
    } else {
        consec = 0;
        const double ccost = isfinite(scal[SC_COST]) ? scal[SC_COST] : DBL_MAX;
        if (sn <= o.ptol * (xn + o.ptol)) term = o.term_conv;
        else if (fabs(cost - ccost) <= o.ftol * cost) term = o.term_conv;
        else {
            const double rel = (cost - ccost) / mcc;
            if (rel > o.minrel) {     // HandleSuccessfulStep
                accepted = true;
                cost = ccost;
                gmax = scal[SC_GMAX];
                xn = sqrt(scal[SC_XN] + scal[SC_XN_F]);
                radius = radius / fmax(1.0 / 3.0, 1.0 - lm_cube(2.0 * rel - 1.0));
                radius = fmin(o.maxr, radius);
                dec = 2.0;
                successful = true;
            } else {                  // HandleUnsuccessfulStep
                radius /= dec; dec *= 2.0;
                successful = false;
            }
        }
    }
    if (term == LM_RUNNING) {         // the next iteration's FinalizeIteration...
        lm[successful ? LM_SUCC : LM_UNSUCC] += 1.0;
        trace = true;
        if (lm[LM_ITER] >= o.maxit) term = o.term_noconv;
        else if (successful && gmax <= o.gtol) term = o.term_conv;
        else if (radius <= o.minr) term = o.term_conv;
        else lm[LM_ITER] += 1.0;
    }
    lm[LM_COST] = cost; lm[LM_GMAX] = gmax; lm[LM_XNORM] = xn; lm[LM_RADIUS] = radius; lm[LM_DECREASE] = dec;
    lm[LM_CONSEC] = consec; lm[LM_SUCCESSFUL] = successful ? 1.0 : 0.0; lm[LM_TERM] = term;
    lm[LM_ACCEPTED] = accepted ? 1.0 : 0.0; lm[LM_TRACE] = trace ? 1.0 : 0.0;
    fail[1] = (term == LM_RUNNING && accepted) ? 1 : 0;
    publish_body(scal, SC_N, lm, LM_N, dst, seq, v, fail);
}

// Re-opens the step gate (after a rejected step, before the host enqueues the step again).
__global__ void ba_open_gate(int* __restrict__ fail) { if (threadIdx.x == 0) fail[1] = 1; }

// problem setup: every observation's (internal) point from the point-major CSR
__global__ void ba_obs_point(int P, const int* __restrict__ pt_start, int* __restrict__ obs_point) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < P)
        for (int o = pt_start[p]; o < pt_start[p + 1]; ++o) obs_point[o] = p;
}
// sfmx_ba_update: an unchanged bucket's observation data moves to its offset in the new layout
// (pixels, camera, local camera, feature row: 24 B per observation), one workgroup per <= 4096.
struct ObsMove { long long src, dst; int n, pad; };
constexpr int RELAYOUT_CHUNK = 4096;
__global__ __launch_bounds__(256) void ba_relayout(const ObsMove* __restrict__ mv, const double2* __restrict__ xy,
                                                   const int* __restrict__ cam, const short* __restrict__ lc,
                                                   const short* __restrict__ row, double2* __restrict__ xy2,
                                                   int* __restrict__ cam2, short* __restrict__ lc2, short* __restrict__ row2) {
    const ObsMove m = mv[blockIdx.x];
    for (int k = threadIdx.x; k < m.n; k += blockDim.x) {
        xy2[m.dst + k] = xy[m.src + k];
        cam2[m.dst + k] = cam[m.src + k];
        lc2[m.dst + k] = lc[m.src + k];
        row2[m.dst + k] = row[m.src + k];
    }
}
__global__ void ba_fill(int64_t n, double v, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = v;
}
// scale = 1 / (1 + sqrt(colsq)) (iteration 0 only, Ceres jacobi_scaling)
__global__ void ba_scale(int n, const double* __restrict__ colsq, double* __restrict__ scale) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) scale[i] = 1.0 / (1.0 + sqrt(colsq[i]));
}

}  // namespace ba
}  // namespace sfmx
