// SPDX-License-Identifier: MIT
// sfmx bundle adjustment, point-group kernels (gfx950, fp64) — the r02 Schur pipeline.
//
// One Levenberg-Marquardt step of the reference's Ceres problem (BundleAdjustment.cpp:29-91,
// CeresUtils::solve with DENSE_SCHUR, CeresUtils.cpp:43-50) with every per-observation stream
// read or written ONCE per pass, organised around point groups:
//   a group = consecutive points of the locality order (points sorted by their camera lists,
//   observations point-major) whose observations number <= GOBS, whose points number <= GPTS and
//   whose cameras (the union, u <= UMAX) are few; it is cut into chunks of <= GCH observations
//   holding whole points.  A point with more observations / cameras than that, or with two
//   observations in one camera, is a "big" group of its own (slow, general path).
//
// Reduced camera system with E_p = Je^T Je + D_p^2 = L_c L_c^T (3x3) and M_p = L_c^-1:
//   S   = C + D_f^2 - sum_p H_p H_p^T,   H_p = (M_p W_p)^T,  W_p = sum_o Je_o^T [Jc_o | Ji_o]
//   rhs = g_f - sum_p H_p t_p,           t_p = M_p g_p
//   x_e = M_p^T (t_p - M_p sum_o Je_o^T ([Jc_o | Ji_o] x_f))                       (back substitution)
// C and g_f (camera-camera part of J^T J, J^T r) do not depend on the LM radius: they are summed
// once per linearization from per-(group, camera) partials.  Per group and LM step the kernel
// ba_gschur builds the dense (6u+K)^2 block -sum H H^T of its points on the fp64 matrix cores
// (SYRK in sub-batches of SBP points); ba_assemble sums the group blocks into S in group order
// (deterministic, no atomics).
//
// Kernels (all one workgroup per group unless noted):
//   ba_glin      residuals + Jacobian (dual numbers, = ceres::AutoDiffCostFunction on the reference
//                functors) at x or at the candidate; J records; cost; per-point column norms and
//                gradient; per-(group, camera) partials of J^T J and J^T r of the camera columns
//   ba_camred    per camera (one workgroup each, + one for the intrinsics): those partials in group order
//   ba_gschur    per-point E, M, t, H; the group's -sum H H^T block and -sum H t
//   ba_assemble  one workgroup per block of S: sum over the groups that hold it, in group order
//   ba_add_cam   + scaled C, D_f^2 and g_f (after any cross-rank all-reduce of S)
//   ba_gupdate   back substitution, step, candidate points, model cost change, step norm
//   ba_fstep     candidate cameras / intrinsics
//   ba_finalize  the LM scalars of one step (one workgroup)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cfloat>

#include "ba_kernels.hpp"

namespace sfmx {
namespace ba {

constexpr int GCH = 256;      // observations per chunk = threads per group workgroup
constexpr int GOBS = 1024;    // observations per (normal) group
constexpr int GPTS = 128;     // points per group (one thread per point)
constexpr int UMAX = 16;      // cameras per group: S block <= (6*16 + K)^2
constexpr int SBP = 16;       // points per SYRK sub-batch
constexpr int SBK = 3 * SBP;  // SYRK depth per sub-batch (3 per point)
constexpr int ALD = SBK + 1;  // LDS row stride of the SYRK operand (doubles)
constexpr int MAXT = 7;       // 16x16 upper tiles per wave: dp <= 112 -> 28 tiles / 4 waves

// per-(group, camera) partials of the unscaled camera columns:
//   Jc^T Jc upper (21) | Jc^T Ji (6K) | Jc^T r (6) | Ji^T Ji upper (K(K+1)/2) | Ji^T r (K)
__host__ __device__ constexpr int ncp(int K) { return 21 + 6 * K + 6 + K * (K + 1) / 2 + K; }
__host__ __device__ constexpr int cp_ci(int) { return 21; }
__host__ __device__ constexpr int cp_gc(int K) { return 21 + 6 * K; }
__host__ __device__ constexpr int cp_ii(int K) { return 27 + 6 * K; }
__host__ __device__ constexpr int cp_gi(int K) { return 27 + 6 * K + K * (K + 1) / 2; }
// per-group scalar partials
enum { GP_COST = 0, GP_MODEL = 1, GP_STEPN = 2, GP_XN = 3, GP_GMAX = 4, GP_N = 8 };
// LM scalars (scal[]): [0..3] rank-local sums, [4..5] maxima, [6..7] replicated camera parts
enum { SC_COST = 0, SC_MODEL = 1, SC_STEPN = 2, SC_XN = 3, SC_GMAX = 4, SC_FAIL = 5, SC_STEPN_F = 6, SC_XN_F = 7, SC_N = 8 };

struct Grp {
    int o0, o1, p0, p1;      // observation / point range (internal order)
    int u, cam_off;          // cameras: gcam[cam_off .. cam_off + u), sorted; partial rows gpart[cam_off + lc]
    int ch0, nch;            // chunks chk[ch0 .. ch0 + nch)
    long long sg_off;        // dense (6u+K)^2 block in sg (normal groups)
    long long h_off;         // H (dim x 3) in hbig (big groups)
    int rg_off, big;         // rhs block (dim) in rg; big-group flag
};
struct Chunk { int o0, o1, q0, q1; };   // observations [o0, o1), point slots [q0, q1) of the group
struct ATask { int type, a, b, l0, l1, pad0, pad1, pad2; };   // 0: pose (a <= b), 1: pose-intr a, 2: intr
struct AEnt { int g, la, lb, pad; };

__device__ __forceinline__ int gdim(const Grp& G, int K) { return 6 * G.u + K; }

// M = L^-1 of the Cholesky factor of the SPD 3x3 E (row-major full); false if not positive definite.
// Packed lower: M[0] = m00, M[1] = m10, M[2] = m11, M[3] = m20, M[4] = m21, M[5] = m22
// (the same operation order as inv3_spd).
__device__ __forceinline__ bool chol3_inv(const double* E, double* M) {
    double l00 = E[0];
    if (!(l00 > 0)) return false;
    l00 = sqrt(l00);
    const double l10 = E[3] / l00, l20 = E[6] / l00;
    double l11 = E[4] - l10 * l10;
    if (!(l11 > 0)) return false;
    l11 = sqrt(l11);
    const double l21 = (E[7] - l20 * l10) / l11;
    double l22 = E[8] - l20 * l20 - l21 * l21;
    if (!(l22 > 0)) return false;
    l22 = sqrt(l22);
    const double i00 = 1 / l00, i11 = 1 / l11, i22 = 1 / l22;
    const double i10 = -l10 * i00 * i11;
    const double i21 = -l21 * i11 * i22;
    const double i20 = -(l20 * i00 + l21 * i10) * i22;
    M[0] = i00; M[1] = i10; M[2] = i11; M[3] = i20; M[4] = i21; M[5] = i22;
    return true;
}
__device__ __forceinline__ double mlo(const double* M, int k, int j) {   // M[k][j], j <= k
    return k == 0 ? M[0] : (k == 1 ? (j == 0 ? M[1] : M[2]) : (j == 0 ? M[3] : (j == 1 ? M[4] : M[5])));
}

// LM diagonal entry: D^2 with D = sqrt(clamp(colsq * s^2, dmin, dmax) / radius) (Ceres: lm_diagonal_ =
// sqrt(diag / radius); the Schur eliminator adds D.^2)
__device__ __forceinline__ double dsq(double colsq, double s, double dmin, double dmax, double radius) {
    const double d = sqrt(fmin(fmax(colsq * s * s, dmin), dmax) / radius);
    return d * d;
}

template <int K>
struct JRec {            // one observation's Jacobian record, scaled
    double r[2], je[2][3], jc[2][6], ji[2][K];
};
template <int K>
__device__ __forceinline__ void load_rec(const double* __restrict__ jr, const double* sp, const double* sc,
                                         const double* si, JRec<K>& R) {
    R.r[0] = jr[0]; R.r[1] = jr[1];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int i = 0; i < 3; ++i) R.je[j][i] = jr[2 + 3 * j + i] * sp[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) R.jc[j][i] = jr[8 + 6 * j + i] * sc[i];
#pragma unroll
        for (int i = 0; i < K; ++i) R.ji[j][i] = jr[20 + K * j + i] * si[i];
    }
}
template <int K>
__device__ __forceinline__ void load_jrec(const double* __restrict__ J, int o, const double* sp, const double* sc,
                                          const double* si, JRec<K>& R) {
    load_rec<K>(J + (size_t)o * jst(K), sp, sc, si, R);
}

// ---------------------------------------------------------------------------------------------
// ba_gschur: per group, its block -sum_p H_p H_p^T (dense dim x dim into sg) and -sum_p H_p t_p
// (into rg); per point M_p and t_p (plt, 9 doubles) for the back substitution.
// Dynamic LDS: stage[max(GCH * jst(K), dp_max * ALD)] (the chunk's J records, coalesced; later the
// SYRK operand A[dp][ALD]) | pd[GPTS][9 + 3K].
template <int K>
__global__ __launch_bounds__(256, K == 7 ? 1 : 2)
void ba_gschur(const Grp* __restrict__ grp, const Chunk* __restrict__ chk, const int* __restrict__ gcam,
               const short* __restrict__ obs_lc, const int* __restrict__ obs_point, const int* __restrict__ obs_cam,
               const int* __restrict__ pt_start, const double* __restrict__ J, const double* __restrict__ scale,
               const double* __restrict__ colsq, double dmin, double dmax, double radius, int P, int C, int stage_n,
               double* __restrict__ plt, double* __restrict__ sg, double* __restrict__ rg, double* __restrict__ hbig,
               int* __restrict__ fail) {
    extern __shared__ __attribute__((aligned(16))) double gl[];
    constexpr int JS = jst(K);
    constexpr int PD = 9 + 3 * K;           // LDS per point: M (6) | t (3) | Hi (K x 3)
    double* stg = gl;                       // J records of the chunk, then the SYRK operand
    double* A = gl;
    double* pd = gl + stage_n;
    const Grp G = grp[blockIdx.x];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, m16 = l & 15, kq = l >> 4;
    const size_t ne = 3 * (size_t)P, ni = ne + 6 * (size_t)C;
    double si[K];
#pragma unroll
    for (int i = 0; i < K; ++i) si[i] = scale[ni + i];
    const int dim = gdim(G, K);

    if (G.big) {   // one point, any number of observations / cameras: serial per point, per camera
        const int p = G.p0;
        if (tid == 0) {
            const double sp[3] = {scale[3 * (size_t)p], scale[3 * (size_t)p + 1], scale[3 * (size_t)p + 2]};
            double E[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0}, Wi[3 * K];
#pragma unroll
            for (int i = 0; i < 3 * K; ++i) Wi[i] = 0.0;
            for (int o = G.o0; o < G.o1; ++o) {
                const int c = obs_cam[o];
                double sc[6];
#pragma unroll
                for (int d = 0; d < 6; ++d) sc[d] = scale[ne + 6 * (size_t)c + d];
                JRec<K> R;
                load_jrec<K>(J, o, sp, sc, si, R);
#pragma unroll
                for (int a = 0; a < 3; ++a) {
#pragma unroll
                    for (int b = 0; b < 3; ++b) E[a * 3 + b] += R.je[0][a] * R.je[0][b] + R.je[1][a] * R.je[1][b];
                    g[a] += R.je[0][a] * R.r[0] + R.je[1][a] * R.r[1];
#pragma unroll
                    for (int i = 0; i < K; ++i) Wi[a * K + i] += R.je[0][a] * R.ji[0][i] + R.je[1][a] * R.ji[1][i];
                }
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) E[4 * i] += dsq(colsq[3 * (size_t)p + i], sp[i], dmin, dmax, radius);
            double M[6];
            if (!chol3_inv(E, M)) {
                atomicOr(fail, 1);
#pragma unroll
                for (int i = 0; i < 6; ++i) M[i] = 0.0;
            }
            double t[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                t[k] = 0.0;
                for (int j = 0; j <= k; ++j) t[k] += mlo(M, k, j) * g[j];
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) { plt[9 * (size_t)p + i] = M[i]; pd[i] = M[i]; }
#pragma unroll
            for (int k = 0; k < 3; ++k) { plt[9 * (size_t)p + 6 + k] = t[k]; pd[6 + k] = t[k]; }
            double* H = hbig + G.h_off;
#pragma unroll
            for (int i = 0; i < K; ++i)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double h = 0.0;
                    for (int j = 0; j <= k; ++j) h += mlo(M, k, j) * Wi[j * K + i];
                    H[(6 * G.u + i) * 3 + k] = h;
                }
        }
        __syncthreads();
        double M[6], t[3];
#pragma unroll
        for (int i = 0; i < 6; ++i) M[i] = pd[i];
#pragma unroll
        for (int k = 0; k < 3; ++k) t[k] = pd[6 + k];
        const double sp[3] = {scale[3 * (size_t)p], scale[3 * (size_t)p + 1], scale[3 * (size_t)p + 2]};
        double* H = hbig + G.h_off;
        for (int lc = tid; lc < G.u; lc += blockDim.x) {   // W of camera lc over the point's observations, in order
            const int c = gcam[G.cam_off + lc];
            double sc[6];
#pragma unroll
            for (int d = 0; d < 6; ++d) sc[d] = scale[ne + 6 * (size_t)c + d];
            double W[3][6];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int d = 0; d < 6; ++d) W[a][d] = 0.0;
            for (int o = G.o0; o < G.o1; ++o) {
                if (obs_lc[o] != lc) continue;
                JRec<K> R;
                load_jrec<K>(J, o, sp, sc, si, R);
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int d = 0; d < 6; ++d) W[a][d] += R.je[0][a] * R.jc[0][d] + R.je[1][a] * R.jc[1][d];
            }
#pragma unroll
            for (int d = 0; d < 6; ++d)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double h = 0.0;
                    for (int j = 0; j <= k; ++j) h += mlo(M, k, j) * W[j][d];
                    H[(6 * lc + d) * 3 + k] = h;
                }
        }
        __syncthreads();
        for (int i = tid; i < dim; i += blockDim.x)
            rg[G.rg_off + i] = -(H[i * 3] * t[0] + H[i * 3 + 1] * t[1] + H[i * 3 + 2] * t[2]);
        return;
    }

    const int dp = (dim + 15) & ~15, nt = dp >> 4, ntiles = nt * (nt + 1) / 2;
    f64x4 acc[MAXT];
    int ti[MAXT], tj[MAXT];
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
        acc[i] = f64x4{0.0, 0.0, 0.0, 0.0};
        int tt = w + 4 * i, I = 0;
        while (tt >= nt - I && I < nt) { tt -= nt - I; ++I; }
        ti[i] = I; tj[i] = I + tt;                 // valid when w + 4i < ntiles
    }
    double racc = 0.0;                             // rhs row tid (< dim)
    const int np = G.p1 - G.p0;
    for (int c = 0; c < G.nch; ++c) {
        const Chunk ch = chk[G.ch0 + c];
        {   // the chunk's J records -> LDS (16-B coalesced loads)
            const double2* src = reinterpret_cast<const double2*>(J + (size_t)ch.o0 * JS);
            double2* dst = reinterpret_cast<double2*>(stg);
            const int n2 = (ch.o1 - ch.o0) * (JS / 2);
            for (int i = tid; i < n2; i += blockDim.x) dst[i] = src[i];
        }
        __syncthreads();
        const int a = tid, o = ch.o0 + a;
        const bool ov = o < ch.o1;
        // B2: one thread per point of the chunk: E, g, Wi; M, t, Hi
        if (tid >= ch.q0 && tid < ch.q1) {
            const int p = G.p0 + tid;
            const int a0 = pt_start[p] - ch.o0, a1 = pt_start[p + 1] - ch.o0;
            const double sp[3] = {scale[3 * (size_t)p], scale[3 * (size_t)p + 1], scale[3 * (size_t)p + 2]};
            double E[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0}, Wi[3 * K];
#pragma unroll
            for (int i = 0; i < 3 * K; ++i) Wi[i] = 0.0;
            for (int b = a0; b < a1; ++b) {
                const double* s_ = stg + b * JS;
                double je[2][3], ji[2][K];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
#pragma unroll
                    for (int i = 0; i < 3; ++i) je[j][i] = s_[2 + 3 * j + i] * sp[i];
#pragma unroll
                    for (int i = 0; i < K; ++i) ji[j][i] = s_[20 + K * j + i] * si[i];
                }
                const double r0 = s_[0], r1 = s_[1];
#pragma unroll
                for (int u = 0; u < 3; ++u) {
#pragma unroll
                    for (int v = 0; v < 3; ++v) E[u * 3 + v] += je[0][u] * je[0][v] + je[1][u] * je[1][v];
                    g[u] += je[0][u] * r0 + je[1][u] * r1;
#pragma unroll
                    for (int i = 0; i < K; ++i) Wi[u * K + i] += je[0][u] * ji[0][i] + je[1][u] * ji[1][i];
                }
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) E[4 * i] += dsq(colsq[3 * (size_t)p + i], sp[i], dmin, dmax, radius);
            double M[6];
            if (!chol3_inv(E, M)) {
                atomicOr(fail, 1);
#pragma unroll
                for (int i = 0; i < 6; ++i) M[i] = 0.0;
            }
            double* q_ = pd + tid * PD;
#pragma unroll
            for (int i = 0; i < 6; ++i) { q_[i] = M[i]; plt[9 * (size_t)p + i] = M[i]; }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                double t = 0.0;
#pragma unroll
                for (int j = 0; j <= k; ++j) t += mlo(M, k, j) * g[j];
                q_[6 + k] = t;
                plt[9 * (size_t)p + 6 + k] = t;
            }
#pragma unroll
            for (int i = 0; i < K; ++i)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double h = 0.0;
#pragma unroll
                    for (int j = 0; j <= k; ++j) h += mlo(M, k, j) * Wi[j * K + i];
                    q_[9 + 3 * i + k] = h;
                }
        }
        __syncthreads();   // pd complete
        // B3: one thread per observation: H_o = (M_p W_o)^T (6x3), W_o = Je_o^T Jc_o, from the staged record
        double H[6][3];
        int q = 0, lc = 0;
        if (ov) {
            const int p = obs_point[o], cm = obs_cam[o];
            q = p - G.p0;
            lc = obs_lc[o];
            const double* rr = stg + (size_t)a * JS;
            double je[2][3], jc[2][6];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int i = 0; i < 3; ++i) je[j][i] = rr[2 + 3 * j + i] * scale[3 * (size_t)p + i];
#pragma unroll
                for (int i = 0; i < 6; ++i) jc[j][i] = rr[8 + 6 * j + i] * scale[ne + 6 * (size_t)cm + i];
            }
            const double* M = pd + q * PD;
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                double Wd[3];
#pragma unroll
                for (int j = 0; j < 3; ++j) Wd[j] = je[0][j] * jc[0][d] + je[1][j] * jc[1][d];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double h = 0.0;
#pragma unroll
                    for (int j = 0; j <= k; ++j) h += mlo(M, k, j) * Wd[j];
                    H[d][k] = h;
                }
            }
        }
        __syncthreads();   // every staged record read: A reuses the buffer
        // SYRK over sub-batches of SBP points: A[row][3s + k] = H_p[row][k]
        for (int sb = ch.q0; sb < ch.q1; sb += SBP) {
            for (int e = tid; e < dp * ALD; e += blockDim.x) A[e] = 0.0;
            __syncthreads();
            if (ov && q >= sb && q < sb + SBP) {
#pragma unroll
                for (int d = 0; d < 6; ++d)
#pragma unroll
                    for (int k = 0; k < 3; ++k) A[(6 * lc + d) * ALD + 3 * (q - sb) + k] = H[d][k];
            }
            if (tid >= sb && tid < min(sb + SBP, ch.q1)) {
                const double* q_ = pd + tid * PD;
#pragma unroll
                for (int i = 0; i < K; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) A[(6 * G.u + i) * ALD + 3 * (tid - sb) + k] = q_[9 + 3 * i + k];
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < MAXT; ++i) {
                if (w + 4 * i >= ntiles) continue;
                const double* Ar = A + (16 * ti[i] + m16) * ALD;
                const double* Br = A + (16 * tj[i] + m16) * ALD;
#pragma unroll
                for (int st = 0; st < SBK / 4; ++st)
                    acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(Ar[4 * st + kq], Br[4 * st + kq], acc[i], 0, 0, 0);
            }
            if (tid < dim) {
                const int sn = min(SBP, ch.q1 - sb);
                for (int s = 0; s < sn; ++s) {
                    const double* q_ = pd + (sb + s) * PD;
                    racc += A[tid * ALD + 3 * s] * q_[6] + A[tid * ALD + 3 * s + 1] * q_[7] + A[tid * ALD + 3 * s + 2] * q_[8];
                }
            }
            __syncthreads();
        }
    }
    // -sum H H^T (full square) and -sum H t
    double* Sg = sg + G.sg_off;
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
        if (w + 4 * i >= ntiles) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * ti[i] + trow(r), col = 16 * tj[i] + tcol();
            if (row < dim && col < dim) {
                Sg[(size_t)row * dim + col] = -acc[i][r];
                Sg[(size_t)col * dim + row] = -acc[i][r];
            }
        }
    }
    if (tid < dim) rg[G.rg_off + tid] = -racc;
    (void)np;
}

// ---------------------------------------------------------------------------------------------
// ba_assemble: one 64-thread workgroup per block of S, summing the group contributions in group
// order (normal groups: their dense block; big groups: -H_a H_b^T from the stored H); writes S and
// its transpose, and the rhs rows (pose-intr task: camera rows; intr task: intrinsics rows and the
// padding).  S is zeroed before; C, D^2 and g_f are added by ba_add_cam.
__device__ __forceinline__ double gval(const Grp& G, const double* __restrict__ sg, const double* __restrict__ hbig,
                                       int K, int r, int c) {
    if (!G.big) return sg[G.sg_off + (size_t)r * gdim(G, K) + c];
    const double* H = hbig + G.h_off;
    return -(H[r * 3] * H[c * 3] + H[r * 3 + 1] * H[c * 3 + 1] + H[r * 3 + 2] * H[c * 3 + 2]);
}
__global__ __launch_bounds__(64)
void ba_assemble(const ATask* __restrict__ tasks, const AEnt* __restrict__ ents, const Grp* __restrict__ grp,
                 const double* __restrict__ sg, const double* __restrict__ hbig, const double* __restrict__ rg, int C,
                 int K, int nf, int npad, double* __restrict__ S, double* __restrict__ rhs) {
    const ATask T = tasks[blockIdx.x];
    const int t = threadIdx.x;
    if (T.type == 0) {
        if (t >= 36) return;
        const int u = t / 6, w = t % 6;
        double v = 0.0;
        for (int e = T.l0; e < T.l1; ++e) {
            const AEnt E = ents[e];
            v += gval(grp[E.g], sg, hbig, K, 6 * E.la + u, 6 * E.lb + w);
        }
        S[(size_t)(6 * T.a + u) * npad + 6 * T.b + w] = v;
        if (T.a != T.b) S[(size_t)(6 * T.b + w) * npad + 6 * T.a + u] = v;
    } else if (T.type == 1) {
        if (t < 6 * K) {
            const int u = t / K, i = t % K;
            double v = 0.0;
            for (int e = T.l0; e < T.l1; ++e) {
                const AEnt E = ents[e];
                const Grp G = grp[E.g];
                v += gval(G, sg, hbig, K, 6 * E.la + u, 6 * G.u + i);
            }
            S[(size_t)(6 * T.a + u) * npad + 6 * C + i] = v;
            S[(size_t)(6 * C + i) * npad + 6 * T.a + u] = v;
        } else if (t < 6 * K + 6) {
            const int d = t - 6 * K;
            double v = 0.0;
            for (int e = T.l0; e < T.l1; ++e) {
                const AEnt E = ents[e];
                v += rg[grp[E.g].rg_off + 6 * E.la + d];
            }
            rhs[6 * T.a + d] = v;
        }
    } else {
        for (int x = t; x < K * K + K; x += 64) {
            double v = 0.0;
            if (x < K * K) {
                const int i = x / K, j = x % K;
                for (int e = T.l0; e < T.l1; ++e) {
                    const Grp G = grp[ents[e].g];
                    v += gval(G, sg, hbig, K, 6 * G.u + i, 6 * G.u + j);
                }
                S[(size_t)(6 * C + i) * npad + 6 * C + j] = v;
            } else {
                const int i = x - K * K;
                for (int e = T.l0; e < T.l1; ++e) {
                    const Grp G = grp[ents[e].g];
                    v += rg[G.rg_off + 6 * G.u + i];
                }
                rhs[6 * C + i] = v;
            }
        }
        for (int i = nf + t; i < npad; i += 64) { S[(size_t)i * npad + i] = 1.0; rhs[i] = 0.0; }
    }
}

// + the camera-camera part C of the scaled J^T J, D_f^2 and g_f: one workgroup per camera
// (blockIdx.x < C) and one for the intrinsics.  camsum (per camera ncp(K) unscaled sums, then
// the intrinsics K(K+1)/2 + K) is already summed over ranks.
template <int K>
__global__ __launch_bounds__(64)
void ba_add_cam(int P, int C, int npad, const double* __restrict__ camsum, const double* __restrict__ scale,
                const double* __restrict__ colsq, double dmin, double dmax, double radius, double* __restrict__ S,
                double* __restrict__ rhs) {
    constexpr int NCP = ncp(K);
    const size_t ne = 3 * (size_t)P, nfc = 6 * (size_t)C;
    const int t = threadIdx.x;
    const double* si = scale + ne + nfc;
    if ((int)blockIdx.x < C) {
        const int c = blockIdx.x;
        const double* cs = camsum + (size_t)c * NCP;
        const double* sc = scale + ne + 6 * (size_t)c;
        if (t < 36) {
            const int u = t / 6, w = t % 6, a = u < w ? u : w, b = u < w ? w : u;
            int e = 0;
            for (int x = 0; x < a; ++x) e += 6 - x;
            e += b - a;
            double v = sc[u] * sc[w] * cs[e];
            if (u == w) v += dsq(colsq[ne + 6 * (size_t)c + u], sc[u], dmin, dmax, radius);
            S[(6 * (size_t)c + u) * npad + 6 * c + w] += v;
        } else if (t < 36 + 6 * K) {
            const int x = t - 36, u = x / K, i = x % K;
            const double v = sc[u] * si[i] * cs[cp_ci(K) + u * K + i];
            S[(6 * (size_t)c + u) * npad + 6 * C + i] += v;
            S[(nfc + i) * npad + 6 * c + u] += v;
        } else if (t < 42 + 6 * K) {
            const int u = t - 36 - 6 * K;
            rhs[6 * c + u] += sc[u] * cs[cp_gc(K) + u];
        }
    } else {
        const double* ii = camsum + (size_t)C * NCP;
        for (int x = t; x < K * K + K; x += 64) {
            if (x < K * K) {
                const int i = x / K, j = x % K, a = i < j ? i : j, b = i < j ? j : i;
                int e = 0;
                for (int y = 0; y < a; ++y) e += K - y;
                e += b - a;
                double v = si[i] * si[j] * ii[e];
                if (i == j) v += dsq(colsq[ne + nfc + i], si[i], dmin, dmax, radius);
                S[(nfc + i) * npad + nfc + j] += v;
            } else {
                const int i = x - K * K;
                rhs[nfc + i] += si[i] * ii[K * (K + 1) / 2 + i];
            }
        }
    }
}

// sum over the chunk's observations of camera lc (in order) of one field of the per-(group,
// camera) partials (see ncp); records in LDS (jst(K) doubles each), olc = local camera per obs.
template <int K>
__device__ __forceinline__ double cam_field_sum(const double* __restrict__ jl, const short* __restrict__ olc, int no,
                                                int lc, int f) {
    constexpr int JS = jst(K);
    // decode the field into two operand offsets within a record: v = x0[i] * y0[j] + x1[i] * y1[j]
    int oa, ob;   // offsets of row 0 operands; row 1 operands are at oa + da, ob + db
    int da, db;
    if (f < 21) {
        int u = 0, e = f;
        while (e >= 6 - u) { e -= 6 - u; ++u; }
        oa = 8 + u; ob = 8 + u + e; da = 6; db = 6;
    } else if (f < cp_gc(K)) {
        const int y = f - 21, u = y / K, ii = y % K;
        oa = 8 + u; ob = 20 + ii; da = 6; db = K;
    } else if (f < cp_ii(K)) {
        oa = 8 + (f - cp_gc(K)); ob = 0; da = 6; db = 1;
    } else if (f < cp_gi(K)) {
        int ii = 0, e = f - cp_ii(K);
        while (e >= K - ii) { e -= K - ii; ++ii; }
        oa = 20 + ii; ob = 20 + ii + e; da = K; db = K;
    } else {
        oa = 20 + (f - cp_gi(K)); ob = 0; da = K; db = 1;
    }
    double s = 0.0;
    for (int b = 0; b < no; ++b) {
        if (olc[b] != lc) continue;
        const double* r = jl + b * JS;
        s += r[oa] * r[ob] + r[oa + da] * r[ob + db];
    }
    return s;
}

// ---------------------------------------------------------------------------------------------
// ba_glin: residuals + Jacobian at xp (x or the candidate) for the group's observations.
// Writes the J records, per point colsq / grad (unscaled), per (group, camera) partials (gpart),
// and the group's cost, sum xp^2 (its points) and max |grad| partials.
// Dynamic LDS: jl[GCH][jst(K)] | olc[GCH] (short).
template <int K>
__global__ __launch_bounds__(256)
void ba_glin(const Grp* __restrict__ grp, const Chunk* __restrict__ chk, const short* __restrict__ obs_lc,
             const int* __restrict__ obs_point, const int* __restrict__ obs_cam, const double* __restrict__ obs_xy,
             const int* __restrict__ pt_start, double cx, double cy, int P, int C, const double* __restrict__ xp,
             double* __restrict__ J, double* __restrict__ colsq, double* __restrict__ grad, double* __restrict__ gpart,
             double* __restrict__ gpl) {
    extern __shared__ __attribute__((aligned(16))) double gl[];
    constexpr int JS = jst(K), NCP = ncp(K), N = 9 + K;
    constexpr int NOWN = (UMAX * NCP + 255) / 256;   // (camera, field) pairs per thread, normal groups
    __shared__ double sh[8];
    double* jl = gl;
    short* olc = reinterpret_cast<short*>(jl + GCH * JS);
    const Grp G = grp[blockIdx.x];
    const int tid = threadIdx.x;
    const double* pts = xp;
    const double* poses = xp + 3 * (size_t)P;
    const double* intr = poses + 6 * (size_t)C;
    double cost = 0.0, xn = 0.0, gmax = 0.0;
    double own[NOWN];
#pragma unroll
    for (int i = 0; i < NOWN; ++i) own[i] = 0.0;
    const int npart = G.u * NCP;
    double pcs[3] = {0, 0, 0}, pgr[3] = {0, 0, 0};   // big groups: the point's sums (thread 0)
    if (G.big)
        for (int i = tid; i < npart; i += blockDim.x) gpart[(size_t)G.cam_off * NCP + i] = 0.0;
    const int nchunks = G.big ? (G.o1 - G.o0 + GCH - 1) / GCH : G.nch;
    for (int c = 0; c < nchunks; ++c) {
        Chunk ch;
        if (G.big) { ch.o0 = G.o0 + c * GCH; ch.o1 = min(G.o1, ch.o0 + GCH); ch.q0 = 0; ch.q1 = 0; }
        else ch = chk[G.ch0 + c];
        const int a = tid, o = ch.o0 + a;
        if (o < ch.o1) {
            const int p = obs_point[o], cm = obs_cam[o];
            const double ox = obs_xy[2 * (size_t)o], oy = obs_xy[2 * (size_t)o + 1];
            DJet<N> X[3], ps[6], in[K], res[2];
#pragma unroll
            for (int i = 0; i < 3; ++i) X[i] = jvar<N>(pts[3 * (size_t)p + i], i);
#pragma unroll
            for (int i = 0; i < 6; ++i) ps[i] = jvar<N>(poses[6 * (size_t)cm + i], 3 + i);
#pragma unroll
            for (int i = 0; i < K; ++i) in[i] = jvar<N>(intr[i], 9 + i);
            project<K, N>(X, ps, in, ox, oy, cx, cy, res);
            double rec[JS];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                rec[j] = res[j].a;
#pragma unroll
                for (int i = 0; i < 3; ++i) rec[2 + 3 * j + i] = res[j].v[i];
#pragma unroll
                for (int i = 0; i < 6; ++i) rec[8 + 6 * j + i] = res[j].v[3 + i];
#pragma unroll
                for (int i = 0; i < K; ++i) rec[20 + K * j + i] = res[j].v[9 + i];
            }
#pragma unroll
            for (int i = 0; i < JS; ++i) jl[a * JS + i] = rec[i];
            olc[a] = obs_lc[o];
            cost += res[0].a * res[0].a + res[1].a * res[1].a;
        }
        __syncthreads();
        const int no = ch.o1 - ch.o0;
        {   // J records of the chunk -> HBM (16-B coalesced stores)
            const double2* src = reinterpret_cast<const double2*>(jl);
            double2* dst = reinterpret_cast<double2*>(J + (size_t)ch.o0 * JS);
            for (int i = tid; i < no * (JS / 2); i += blockDim.x) dst[i] = src[i];
        }
        // per point: column norms and gradient of its 3 columns (whole points in a normal chunk)
        if (!G.big) {
            if (tid >= ch.q0 && tid < ch.q1) {
                const int p = G.p0 + tid;
                const int a0 = pt_start[p] - ch.o0, a1 = pt_start[p + 1] - ch.o0;
                double cs[3] = {0, 0, 0}, gr[3] = {0, 0, 0};
                for (int b = a0; b < a1; ++b) {
                    const double* r = jl + b * JS;
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        const double j0 = r[2 + i], j1 = r[5 + i];
                        cs[i] += j0 * j0 + j1 * j1;
                        gr[i] += j0 * r[0] + j1 * r[1];
                    }
                }
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    colsq[3 * (size_t)p + i] = cs[i];
                    grad[3 * (size_t)p + i] = gr[i];
                    gmax = fmax(gmax, fabs(gr[i]));
                    xn += pts[3 * (size_t)p + i] * pts[3 * (size_t)p + i];
                }
            }
        } else if (tid == 0) {
            for (int b = 0; b < no; ++b) {
                const double* r = jl + b * JS;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const double j0 = r[2 + i], j1 = r[5 + i];
                    pcs[i] += j0 * j0 + j1 * j1;
                    pgr[i] += j0 * r[0] + j1 * r[1];
                }
            }
        }
        // per (camera, field): sum over this chunk's observations of that camera, in order
        if (!G.big) {
#pragma unroll
            for (int i = 0; i < NOWN; ++i) {
                const int x = tid + 256 * i;
                if (x < npart) own[i] += cam_field_sum<K>(jl, olc, no, x / NCP, x % NCP);
            }
        } else {
            for (int x = tid; x < npart; x += blockDim.x)
                gpart[(size_t)G.cam_off * NCP + x] += cam_field_sum<K>(jl, olc, no, x / NCP, x % NCP);
        }
        __syncthreads();
    }
    if (!G.big) {
#pragma unroll
        for (int i = 0; i < NOWN; ++i) {
            const int x = tid + 256 * i;
            if (x < npart) gpart[(size_t)G.cam_off * NCP + x] = own[i];
        }
    } else if (tid == 0) {
        const int p = G.p0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            colsq[3 * (size_t)p + i] = pcs[i];
            grad[3 * (size_t)p + i] = pgr[i];
            gmax = fmax(gmax, fabs(pgr[i]));
            xn += pts[3 * (size_t)p + i] * pts[3 * (size_t)p + i];
        }
    }
    const double sc = block_sum(cost, sh);
    const double sx = block_sum(xn, sh);
    for (int o_ = 32; o_ > 0; o_ >>= 1) gmax = fmax(gmax, __shfl_xor(gmax, o_));
    __syncthreads();
    if ((tid & 63) == 0) sh[tid >> 6] = gmax;
    __syncthreads();
    if (tid == 0) {
        double gm = 0.0;
        for (int i = 0; i < 4; ++i) gm = fmax(gm, sh[i]);
        double* q = gpl + (size_t)blockIdx.x * GP_N;
        q[GP_COST] = 0.5 * sc;
        q[GP_XN] = sx;
        q[GP_GMAX] = gm;
    }
}

// ba_camred: per camera (one workgroup) the partials of its (group, camera) slots in group
// order -> camsum[c]; one more workgroup: the intrinsics fields of every slot, in slot order.
template <int K>
__global__ __launch_bounds__(128)
void ba_camred(int C, int nslots, const int* __restrict__ cref_start, const int* __restrict__ cref,
               const double* __restrict__ gpart, double* __restrict__ camsum) {
    constexpr int NCP = ncp(K), NI = K * (K + 1) / 2 + K;
    const int t = threadIdx.x;
    if ((int)blockIdx.x < C) {
        const int c = blockIdx.x;
        for (int f = t; f < cp_ii(K); f += blockDim.x) {
            double s = 0.0;
            for (int e = cref_start[c]; e < cref_start[c + 1]; ++e) s += gpart[(size_t)cref[e] * NCP + f];
            camsum[(size_t)c * NCP + f] = s;
        }
    } else {
        for (int f = t; f < NI; f += blockDim.x) {
            double s = 0.0;
            for (int e = 0; e < nslots; ++e) s += gpart[(size_t)e * NCP + cp_ii(K) + f];
            camsum[(size_t)C * NCP + f] = s;
        }
    }
}

// ba_finalize (one workgroup of 256): camera column norms / gradient from camsum, and the LM
// scalars: sums over the groups' partials (fixed order), max |grad|, the camera part of the
// step and parameter norms (candidate mode: cand vs x).
template <int K>
__global__ __launch_bounds__(256)
void ba_finalize(int ngroups, int P, int C, const double* __restrict__ camsum, const double* __restrict__ gpl,
                 const double* __restrict__ xf_new, const double* __restrict__ xf_old, int cand_mode,
                 const int* __restrict__ fail, double* __restrict__ colsq, double* __restrict__ grad,
                 double* __restrict__ scal) {
    constexpr int NCP = ncp(K);
    __shared__ double sh[8];
    const int t = threadIdx.x;
    const size_t ne = 3 * (size_t)P;
    const int nf = 6 * C + K;
    double gmax = 0.0, xn = 0.0, sn = 0.0;
    for (int i = t; i < nf; i += blockDim.x) {
        double cs, gr;
        if (i < 6 * C) {
            const int c = i / 6, u = i % 6;
            int e = 0;
            for (int x = 0; x < u; ++x) e += 6 - x;
            cs = camsum[(size_t)c * NCP + e];
            gr = camsum[(size_t)c * NCP + cp_gc(K) + u];
        } else {
            const int ii = i - 6 * C;
            int e = 0;
            for (int x = 0; x < ii; ++x) e += K - x;
            cs = camsum[(size_t)C * NCP + e];
            gr = camsum[(size_t)C * NCP + K * (K + 1) / 2 + ii];
        }
        colsq[ne + i] = cs;
        grad[ne + i] = gr;
        gmax = fmax(gmax, fabs(gr));
        const double v = xf_new[i];
        xn += v * v;
        if (cand_mode) {
            const double d = xf_old[i] - v;
            sn += isfinite(d) ? d * d : INFINITY;
        }
    }
    double g[5] = {0, 0, 0, 0, 0};
    for (int b = t; b < ngroups; b += blockDim.x) {
        const double* q = gpl + (size_t)b * GP_N;
        g[0] += q[GP_COST]; g[1] += q[GP_MODEL]; g[2] += q[GP_STEPN]; g[3] += q[GP_XN];
        g[4] = fmax(g[4], q[GP_GMAX]);
    }
    const double s0 = block_sum(g[0], sh);
    const double s1 = block_sum(g[1], sh);
    const double s2 = block_sum(g[2], sh);
    const double s3 = block_sum(g[3], sh);
    const double sxn = block_sum(xn, sh);
    const double ssn = block_sum(sn, sh);
    double gm = fmax(gmax, g[4]);
    for (int o = 32; o > 0; o >>= 1) gm = fmax(gm, __shfl_xor(gm, o));
    __syncthreads();
    if ((t & 63) == 0) sh[t >> 6] = gm;
    __syncthreads();
    if (t == 0) {
        double m = 0.0;
        for (int i = 0; i < 4; ++i) m = fmax(m, sh[i]);
        scal[SC_COST] = s0;
        scal[SC_MODEL] = s1;
        scal[SC_STEPN] = s2;
        scal[SC_XN] = s3;
        scal[SC_GMAX] = m;
        scal[SC_FAIL] = *fail ? 1.0 : 0.0;
        scal[SC_STEPN_F] = ssn;
        scal[SC_XN_F] = sxn;
    }
}

// ba_gupdate: per group, from sol_f (scaled camera/intrinsics solution) and the stored M, t:
// sol_e = M^T (t - M y), y = sum_o Je_o^T ([Jc_o | Ji_o] sol_f); step = -sol; candidate points
// cand = x + step * scale; ||x - cand||^2 and the model cost change sum m (r + m / 2), m = J_s step_s.
// Dynamic LDS: yv[GCH][3] | pst[GPTS][3].
template <int K>
__global__ __launch_bounds__(256)
void ba_gupdate(const Grp* __restrict__ grp, const Chunk* __restrict__ chk, const int* __restrict__ obs_point,
                const int* __restrict__ obs_cam, const int* __restrict__ pt_start, const double* __restrict__ J,
                const double* __restrict__ scale, const double* __restrict__ plt, const double* __restrict__ sol_f,
                int P, int C, const double* __restrict__ x, double* __restrict__ cand, double* __restrict__ gpl) {
    extern __shared__ __attribute__((aligned(16))) double gl[];
    __shared__ double sh[8];
    constexpr int JS = jst(K);
    double* stg = gl;                 // the chunk's J records
    double* yv = stg + GCH * JS;
    double* pst = yv + GCH * 3;
    const Grp G = grp[blockIdx.x];
    const int tid = threadIdx.x;
    const size_t ne = 3 * (size_t)P, ni = ne + 6 * (size_t)C;
    double si[K], soli[K];
#pragma unroll
    for (int i = 0; i < K; ++i) { si[i] = scale[ni + i]; soli[i] = sol_f[6 * (size_t)C + i]; }
    double model = 0.0, sn = 0.0;
    double ybig[3] = {0, 0, 0};
    const int nchunks = G.big ? (G.o1 - G.o0 + GCH - 1) / GCH : G.nch;
    // big groups: pass 0 accumulates y over all chunks, pass 1 evaluates the model terms
    for (int pass = G.big ? 0 : 1; pass < 2; ++pass) {
        for (int c = 0; c < nchunks; ++c) {
            Chunk ch;
            if (G.big) { ch.o0 = G.o0 + c * GCH; ch.o1 = min(G.o1, ch.o0 + GCH); ch.q0 = 0; ch.q1 = 1; }
            else ch = chk[G.ch0 + c];
            {
                const double2* src = reinterpret_cast<const double2*>(J + (size_t)ch.o0 * JS);
                double2* dst = reinterpret_cast<double2*>(stg);
                for (int i = tid; i < (ch.o1 - ch.o0) * (JS / 2); i += blockDim.x) dst[i] = src[i];
            }
            __syncthreads();
            const int a = tid, o = ch.o0 + a;
            const bool ov = o < ch.o1;
            JRec<K> R;
            int q = 0, cm = 0;
            double f[2] = {0, 0};
            if (ov) {
                const int p = obs_point[o];
                cm = obs_cam[o];
                q = p - G.p0;
                const double sp[3] = {scale[3 * (size_t)p], scale[3 * (size_t)p + 1], scale[3 * (size_t)p + 2]};
                double sc[6];
#pragma unroll
                for (int d = 0; d < 6; ++d) sc[d] = scale[ne + 6 * (size_t)cm + d];
                load_rec<K>(stg + (size_t)a * JS, sp, sc, si, R);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
#pragma unroll
                    for (int d = 0; d < 6; ++d) f[j] += R.jc[j][d] * sol_f[6 * (size_t)cm + d];
#pragma unroll
                    for (int i = 0; i < K; ++i) f[j] += R.ji[j][i] * soli[i];
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) yv[a * 3 + k] = R.je[0][k] * f[0] + R.je[1][k] * f[1];
            }
            __syncthreads();
            if (G.big) {
                if (pass == 0 && tid == 0)
                    for (int b = 0; b < ch.o1 - ch.o0; ++b)
#pragma unroll
                        for (int k = 0; k < 3; ++k) ybig[k] += yv[b * 3 + k];
            } else if (tid >= ch.q0 && tid < ch.q1) {
                const int p = G.p0 + tid;
                const int a0 = pt_start[p] - ch.o0, a1 = pt_start[p + 1] - ch.o0;
                double y[3] = {0, 0, 0};
                for (int b = a0; b < a1; ++b)
#pragma unroll
                    for (int k = 0; k < 3; ++k) y[k] += yv[b * 3 + k];
                const double* Mt = plt + 9 * (size_t)p;
                double v[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double my = 0.0;
#pragma unroll
                    for (int j = 0; j <= k; ++j) my += mlo(Mt, k, j) * y[j];
                    v[k] = Mt[6 + k] - my;
                }
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    double s = 0.0;
#pragma unroll
                    for (int k = j; k < 3; ++k) s += mlo(Mt, k, j) * v[k];
                    const double st = -s;                       // step_s = -sol
                    pst[tid * 3 + j] = st;
                    const double xv = x[3 * (size_t)p + j], cv = xv + st * scale[3 * (size_t)p + j];
                    cand[3 * (size_t)p + j] = cv;
                    const double dd = xv - cv;
                    sn += isfinite(dd) ? dd * dd : INFINITY;
                }
            }
            if (G.big && pass == 1 && c == 0 && tid == 0) {   // the big point's step, once
                const int p = G.p0;
                const double* Mt = plt + 9 * (size_t)p;
                double v[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double my = 0.0;
#pragma unroll
                    for (int j = 0; j <= k; ++j) my += mlo(Mt, k, j) * ybig[j];
                    v[k] = Mt[6 + k] - my;
                }
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    double s = 0.0;
#pragma unroll
                    for (int k = j; k < 3; ++k) s += mlo(Mt, k, j) * v[k];
                    pst[j] = -s;
                    const double xv = x[3 * (size_t)p + j], cv = xv - s * scale[3 * (size_t)p + j];
                    cand[3 * (size_t)p + j] = cv;
                    const double dd = xv - cv;
                    sn += isfinite(dd) ? dd * dd : INFINITY;
                }
            }
            __syncthreads();
            if (pass == 1 && ov) {
                const double* ps = pst + (G.big ? 0 : q) * 3;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    double mm = R.je[j][0] * ps[0] + R.je[j][1] * ps[1] + R.je[j][2] * ps[2];
#pragma unroll
                    for (int d = 0; d < 6; ++d) mm -= R.jc[j][d] * sol_f[6 * (size_t)cm + d];
#pragma unroll
                    for (int i = 0; i < K; ++i) mm -= R.ji[j][i] * soli[i];
                    model += mm * (R.r[j] + mm / 2.0);
                }
            }
            __syncthreads();
        }
    }
    const double sm = block_sum(model, sh);
    const double ss = block_sum(sn, sh);
    if (tid == 0) {
        double* q = gpl + (size_t)blockIdx.x * GP_N;
        q[GP_MODEL] = sm;
        q[GP_STEPN] = ss;
    }
}

// candidate cameras / intrinsics: cand_f = x_f + (-sol_f) * scale_f (one or more workgroups)
__global__ void ba_fstep(int nf, const double* __restrict__ sol_f, const double* __restrict__ scale_f,
                         const double* __restrict__ x_f, double* __restrict__ cand_f) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nf) cand_f[i] = x_f[i] + (-sol_f[i]) * scale_f[i];
}

// Back substitution L~^T x = w over all panels in one workgroup (descending panels):
// x_k = rhs_k is final; rows < k0 get rhs_i -= U(i, k) x_k (upper tiles hold L~^T).
__global__ __launch_bounds__(256)
void chol_back_all(const double* __restrict__ S, int npad, int nf, int T, const double* __restrict__ rhs_in,
                   double* __restrict__ xout) {
    __shared__ double r[16 * 1024];   // npad <= 16384 doubles (128 KB)
    const int tid = threadIdx.x;
    for (int i = tid; i < npad; i += 256) r[i] = rhs_in[i];
    __syncthreads();
    for (int k = T - 1; k >= 0; --k) {
        const int k0 = k * NB;
        for (int i = tid; i < NB; i += 256)
            if (k0 + i < nf) xout[k0 + i] = r[k0 + i];
        // rows [0, k0): 4 threads per row, 16 terms each
        for (int rb = tid >> 2; rb < k0; rb += 64) {
            const int qq = tid & 3;
            const double* U = S + (size_t)rb * npad + k0;
            double t = 0.0;
#pragma unroll 4
            for (int m = 0; m < NB / 4; ++m) t = fma(U[4 * m + qq], r[k0 + 4 * m + qq], t);
            t += __shfl_xor(t, 1);
            t += __shfl_xor(t, 2);
            if (qq == 0) r[rb] -= t;
        }
        __syncthreads();
    }
}

}  // namespace ba
}  // namespace sfmx
