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
//   ba_camred    per camera (one workgroup each): those partials in group order (the intrinsics fields
//                per camera, folded over the cameras by ba_finalize)
//   ba_gschur    per-point E, M, t, H; the group's -sum H H^T block and -sum H t
//   ba_assemble  one workgroup per block of S: sum over the groups that hold it, in group order
//   ba_add_cam   + scaled C, D_f^2 and g_f (after any cross-rank all-reduce of S)
//   (the solve of S itself: ba_chol.hpp, planned by ba_plan.hpp)
//   ba_gupdate   back substitution, step, candidate points, model cost change, step norm
//                (its trailing workgroups: the candidate cameras / intrinsics)
//   ba_finalize  the LM scalars of one step (one workgroup)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cfloat>

#include "ba_kernels.hpp"

namespace sfmx {
namespace ba {

constexpr int GCH = 256;      // observations per chunk = threads per group workgroup (ba_glin, ba_gupdate)
constexpr int GOBS = 1024;    // observations per (normal) group
constexpr int GPTS = 128;     // points per group (one thread per point)
constexpr int UMAX = 16;      // cameras per group (ba_glin's per-camera Gram accumulators)
constexpr int GDPMAX = 64;    // ba_gschur: dp = round16(6u + K) <= 64 (the host cuts groups there)
constexpr int WB_OBS = 64;    // ba_gschur wave batch: observations (one lane each)
constexpr int WB_PTS = 16;    // ba_gschur wave batch: whole points

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

struct Grp {
    int o0, o1, p0, p1;      // observation / point range (internal order)
    int u, cam_off;          // cameras: gcam[cam_off .. cam_off + u), sorted; partial rows gpart[cam_off + lc]
    int ch0, nch;            // chunks chk[ch0 .. ch0 + nch)
    int b0, nb;              // ba_gschur wave batches bat[b0 .. b0 + nb)
    long long sg_off;        // dense (6u+K)^2 block in sg (normal groups)
    long long h_off;         // H (dim x 3) in hbig (big groups)
    int rg_off, big;         // rhs block (dim) in rg; big-group flag
};
// observations [o0, o1), point slots [q0, q1) of the group; the chunk's feature rows sorted by
// local camera: camera lc owns rows lcrow[lc0 + lc] .. lcrow[lc0 + lc + 1) (a multiple of 4, zero-padded)
struct Chunk { int o0, o1, q0, q1, lc0, nrows, pad0, pad1; };
// ba_gschur wave batch: whole points [p0, p1) with their observations [o0, o1) (<= WB_OBS, <= WB_PTS)
struct Batch { int o0, o1, p0, p1; };
struct ATask { int type, a, b, l0, l1, pad0, pad1, pad2; };   // 0: pose (a <= b), 1: pose-intr a, 2: intr
// one contribution to an S block: normal group: b0 = sg offset of its (6la, 6lb) element (row
// stride dim); big group: b0 / b1 = hbig offsets of the H rows 6la / 6lb (row stride 3)
struct AEnt { long long b0, b1; int dim, big, rg, pad; };

__device__ __forceinline__ int gdim(const Grp& G, int K) { return 6 * G.u + K; }

// A workgroup barrier for LDS only: s_waitcnt lgkmcnt(0) + s_barrier.  __syncthreads' workgroup
// release also waits vmcnt(0), i.e. for every outstanding global load AND store of the wave (gfx9
// counts both); a barrier whose other side reads only LDS does not need that.  Global data the waves
// exchange inside a launch still needs __syncthreads.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Diagnostic build only (make stamps -> lib/libsfmx_stamps.so, tools/ba_stamps.py): per-phase
// s_memtime cycle totals of thread 0 of every workgroup.  Compiled out of the product library.
#ifdef SFMX_BA_STAMPS
__device__ unsigned long long g_ba_stamps[64];
#define BA_T0() long long ba_t_ = __builtin_amdgcn_s_memtime(); long long ba_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define BA_STAMP(i)                                                                                \
    do {                                                                                           \
        const long long t_ = __builtin_amdgcn_s_memtime();                                         \
        ba_acc_[i] += t_ - ba_t_;                                                                  \
        ba_t_ = t_;                                                                                \
    } while (0)
#define BA_FLUSH(base)                                                                             \
    do {                                                                                           \
        if (threadIdx.x == 0)                                                                      \
            for (int i_ = 0; i_ < 8; ++i_)                                                         \
                if (ba_acc_[i_]) atomicAdd(&g_ba_stamps[(base) + i_], (unsigned long long)ba_acc_[i_]); \
    } while (0)
#else
#define BA_T0() do { } while (0)
#define BA_STAMP(i) do { } while (0)
#define BA_FLUSH(base) do { } while (0)
#endif

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

// The linearization is kept as what the step kernels consume, not as Jacobian rows (r03):
//   per observation  W_o = Je_o^T Jc_o          (3 x 6, row-major [a][d], WST = 18 doubles)
//   per point        PR_p = E_p 6 | g_p 3 | V_p 3K  with E_p = sum_o Je^T Je (upper: 00 01 02 11 12 22),
//                    g_p = sum_o Je^T r, V_p = sum_o Je^T Ji ([a][i]), sums in observation order
// ba_gschur forms M_p, t_p, H_p from them, ba_gupdate back-substitutes with W_o and V_p, and the
// model cost change is sum_p (s_p.g_p + s_p^T E_p s_p / 2 - s_p.y_p) + the camera part (ba_finalize),
// i.e. s^T J^T r + |J s|^2 / 2 by blocks: no step kernel reads a Jacobian row.  144 B per observation
// instead of the 208 B record (K = 3), and ba_gschur no longer sums per-observation partials.
// Both are stored Jacobi-scaled once the solve's scale is known (ba_glin at every candidate); the
// iteration-0 linearization, written before the scale exists, stays unscaled and the steps on it
// (ba_gschur / ba_gupdate <SCALEJ>) scale what they read, with the products rounded as stored (r05;
// r02-r04 scaled it in place in the first step: 144 B/obs + the records written once more per solve).
constexpr int WST = 18;
__host__ __device__ constexpr int npr(int K) { return 9 + 3 * K; }
// W_o <- diag(sp) W_o diag(sc)
__device__ __forceinline__ void scale_w(double* w, const double* sp, const double* sc) {
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int d = 0; d < 6; ++d) w[6 * a + d] = w[6 * a + d] * (sp[a] * sc[d]);
}
// element e of a point record -> its scale factor (sp: the point's 3, si: the intrinsics' K)
// (e may be lane-dependent: selects, no indexed register arrays)
__device__ __forceinline__ double pick3(const double* s, int u) { return u == 0 ? s[0] : (u == 1 ? s[1] : s[2]); }
template <int K>
__device__ __forceinline__ double pick_k(const double* s, int i) {
    double v = s[0];
#pragma unroll
    for (int j = 1; j < K; ++j) v = i == j ? s[j] : v;
    return v;
}
template <int K>
__device__ __forceinline__ double pr_scale(int e, const double* sp, const double* si) {
    if (e < 6) {
        const int u = e < 3 ? 0 : (e < 5 ? 1 : 2), v = e < 3 ? e : (e < 5 ? e - 2 : 2);
        return pick3(sp, u) * pick3(sp, v);
    }
    if (e < 9) return pick3(sp, e - 6);
    return pick3(sp, (e - 9) / K) * pick_k<K>(si, (e - 9) % K);
}

// Copy n2 16-B pieces global -> LDS with every load issued before the first store (a plain
// load / store loop waits for each load in turn).
template <int PER>
__device__ __forceinline__ void stage_copy(double2* __restrict__ dst, const double2* __restrict__ src, int n2) {
    if (n2 <= 0) return;
    double2 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = src[min((int)threadIdx.x + 256 * i, n2 - 1)];   // clamped: always valid
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int e = threadIdx.x + 256 * i;
        if (e < n2) dst[e] = v[i];
    }
}

// ---------------------------------------------------------------------------------------------
// ba_gschur: per group, its block -sum_p H_p H_p^T (dense dim x dim into sg) and -sum_p H_p t_p
// (into rg); per point M_p and t_p (plt, 9 doubles) for the back substitution.
// Normal groups: no workgroup barrier until the end.  Each wave takes every 4th batch of the
// group (<= 64 observations, <= 16 whole points, host-built) and keeps its own accumulators:
//   lane = observation: its W_o = Je_s^T Jc_s (9 x 16-B loads, prefetched a batch ahead) -> its
//     row of the wave's LDS W table, its lane -> the (point, local camera) map;
//   4 lanes = point: its record (E, g, V; a quarter each) -> the point's wave LDS slot; lane 0 of
//     the 4: + D_p^2, M = chol(E)^-1, t = M g, Hi = M V -> wave LDS + plt;
//   rounds of 4 points: the SYRK on v_mfma_f64_16x16x4f64 takes the 4 points as its k slots:
//     lane m + 16kk forms H_{p_kk}[16I + m][c] itself from LDS (a camera row (lc, d): Z_o[d][c] =
//     (M W_o)[c][d] of the point's observation o in camera lc, zero without one; an intrinsics
//     row: Hi), so tile (I, J) += 3 MFMAs (c = 0..2), the same register both as the A operand
//     (H[16I + m][kk]) and, for tile row J, the B operand; no LDS round trip of H, no barrier
//     inside a round;
//   rhs: lane rows 16I + m accumulate H t of its point.
// Then the 4 waves' tiles and rhs are summed in wave order (fixed, deterministic) through LDS.
// Groups are cut on the host so that dp = round16(6u + K) <= GDPMAX; the launch is specialised on
// NT = dp_max / 16 (NT (NT + 1) / 2 upper 16x16 tiles per wave).
// Big groups (one point with > 64 observations, too many cameras or two observations in one
// camera): the serial path, one thread per point / camera.
// SCALEJ (a step on the iteration-0 linearization, whose records are unscaled): every W_o and point
// record is scaled by the solve's Jacobi scale as it is read (r05: no longer written back -- that was a
// 144 B/obs + record write per solve; ba_gupdate<SCALEJ> scales its reads the same way).
// Dynamic LDS: per wave the W table, WB_PTS x PD point data and the lane map; the final combine
// reuses it as [dp][dp + 1] + rhs.
__host__ __device__ constexpr int gs_pd(int K) { return 9 + 3 * K; }                  // E | g | V, then M 6 | t 3 | Hi 3K
__host__ __device__ constexpr int gs_wreg(int K, int) {                               // doubles per wave
    return WB_OBS * WST + WB_PTS * gs_pd(K) + WB_PTS * UMAX / 8;                      // W rows | point data | lane map
}
__host__ __device__ constexpr int gs_comb(int NT) {   // doubles of the NT <= 3 combine's wave partials (tiles | rhs)
    return NT <= 3 ? 4 * (NT * (NT + 1) / 2 * 256 + 16 * NT) : 0;
}
#ifndef GSCHUR_WAVES
#define GSCHUR_WAVES 2   // waves per SIMD the register budget targets (A/B: -DGSCHUR_WAVES=3)
#endif
template <int K, int NT, bool SCALEJ>
__global__ __launch_bounds__(256, GSCHUR_WAVES)
void ba_gschur(const Grp* __restrict__ grp, const Batch* __restrict__ bat, const int* __restrict__ gcam,
               const short* __restrict__ obs_lc, const int* __restrict__ obs_point, const int* __restrict__ obs_cam,
               const int* __restrict__ pt_start, const double* __restrict__ Wr, const double* __restrict__ PRr,
               const double* __restrict__ scale, const double* __restrict__ colsq, double dmin, double dmax,
               double radius, int P, int C, double* __restrict__ plt, double* __restrict__ sg, double* __restrict__ rg,
               double* __restrict__ hbig, int* __restrict__ fail, const double* __restrict__ lm, int ngroups,
               double* __restrict__ zS, int npad, const int2* __restrict__ nzt, int nnz, long long tail,
               const int* __restrict__ rowmap) {
    if (step_gated(fail + 1)) return;
    if ((int)blockIdx.x >= ngroups) {
        // r06: the workgroups past the groups zero what ba_assemble accumulates into (instead of a 17 MB
        // memset of the dense S at C5): the structurally nonzero lower tiles of S_cc (the diagonal ones
        // whole) and the tail R | D | r_i.  Nothing reads another part of S_cc before the factorization
        // has written it (its upper tiles G^T; ba_plan.cpp row_masks).
        const int b = (int)blockIdx.x - ngroups;
        const double2 z = make_double2(0.0, 0.0);
        if (b < nnz) {
            const int2 tl = nzt[b];
            double* t0 = zS + (size_t)tl.x * 64 * npad + (size_t)tl.y * 64;
            for (int e = threadIdx.x; e < 64 * 32; e += blockDim.x)
                reinterpret_cast<double2*>(t0 + (size_t)(e >> 5) * npad)[e & 31] = z;
            if (tl.x == tl.y) {   // the identity padding rows of a diagonal tile (ba_add_cam's, r05)
                __syncthreads();
                if (threadIdx.x < 64 && rowmap[tl.x * 64 + threadIdx.x] < 0)
                    t0[(size_t)threadIdx.x * npad + threadIdx.x] = 1.0;
            }
        } else {
            double* t0 = zS + (size_t)npad * npad;
            for (long long e = threadIdx.x; e < tail; e += blockDim.x) t0[e] = 0.0;
        }
        return;
    }
    if (lm) radius = lm[LM_RADIUS];
    extern __shared__ __attribute__((aligned(16))) double gl[];
    constexpr int PD = gs_pd(K), NPR = npr(K);
    const Grp G = grp[blockIdx.x];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, m16 = l & 15, kk = l >> 4;
    const int dim = gdim(G, K);
    const size_t ne = 3 * (size_t)P;
    const double* si = scale + ne + 6 * (size_t)C;
    double* pd = gl;   // big groups: the point's M, t

    if (G.big) {   // one point, any number of observations / cameras: serial per point, per camera
        const int p = G.p0;
        const double* sp = scale + 3 * (size_t)p;
        if (tid == 0) {
            double pr[NPR];   // the point's record (SCALEJ: scaled as it is read, the products rounded as stored)
#pragma unroll
            for (int e = 0; e < NPR; ++e) {
                const double v = PRr[(size_t)p * NPR + e];
                pr[e] = SCALEJ ? __dmul_rn(v, pr_scale<K>(e, sp, si)) : v;
            }
            double E[9] = {pr[0], pr[1], pr[2], pr[1], pr[3], pr[4], pr[2], pr[4], pr[5]}, g[3], Wi[3 * K];
#pragma unroll
            for (int i = 0; i < 3; ++i) g[i] = pr[6 + i];
#pragma unroll
            for (int i = 0; i < 3 * K; ++i) Wi[i] = pr[9 + i];
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
        double* H = hbig + G.h_off;
        for (int lc = tid; lc < G.u; lc += blockDim.x) {   // W of camera lc over the point's observations, in order
            double W[3][6];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int d = 0; d < 6; ++d) W[a][d] = 0.0;
            for (int o = G.o0; o < G.o1; ++o) {
                if (obs_lc[o] != lc) continue;
                const double* wo = Wr + (size_t)o * WST;
                const double* sc = scale + ne + 6 * (size_t)obs_cam[o];
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int d = 0; d < 6; ++d)
                        W[a][d] += SCALEJ ? __dmul_rn(wo[6 * a + d], __dmul_rn(sp[a], sc[d])) : wo[6 * a + d];
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

    BA_T0();
    const int dp = (dim + 15) & ~15, nt = dp >> 4;
    const int wreg = gs_wreg(K, dp);
    double* Wl = gl + (size_t)w * wreg;               // [WB_OBS][WST] the batch's W_o, one row per lane
    double* pw = Wl + WB_OBS * WST;                   // [WB_PTS][PD] point data
    signed char* omap = reinterpret_cast<signed char*>(pw + WB_PTS * PD);   // [WB_PTS][UMAX] lane of (point, camera)
    constexpr int NTT = NT * (NT + 1) / 2;            // upper tiles (NT = dp_max / 16 of the launch)
    f64x4 acc[NTT];
#pragma unroll
    for (int t = 0; t < NTT; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    double racc[NT] = {};
    // The group's batch descriptors go to LDS once, so the batch loop issues no dependent loads.
    // Software pipeline: every global load of batch bi + 4 (this lane's observation: its W_o, point
    // and camera slot; this lane's point: a quarter of its record, colsq and scale) is issued right
    // after batch bi has consumed its own, before the plt stores; the SYRK rounds in between touch
    // only LDS and registers, so nothing waits for those loads until the next batch.
    Batch* bl = reinterpret_cast<Batch*>(gl + 4 * (size_t)wreg);
    for (int i = tid; i < G.nb; i += 256) bl[i] = bat[G.b0 + i];
    __syncthreads();
    constexpr int QS = (NPR + 3) / 4;                 // record elements per lane of a point
    const int qp = l >> 2, qk = l & 3;
    double2 pre[WST / 2];
    double pre_pr[QS];
    int pre_q = 0, pre_lc = 0, pre_p = 0, pre_c = 0;
    double pre_cs[3] = {0, 0, 0}, pre_sp[3] = {0, 0, 0};
    auto prefetch = [&](int bi) {
        if (bi >= G.nb) return;
        const Batch Bn = bl[bi];
        const int on = Bn.o0 + l;
        if (on < Bn.o1) {
            pre_p = obs_point[on];
            pre_q = pre_p - Bn.p0;
            pre_lc = obs_lc[on];
            if (SCALEJ) pre_c = obs_cam[on];
            const double2* s2 = reinterpret_cast<const double2*>(Wr + (size_t)on * WST);
#pragma unroll
            for (int i = 0; i < WST / 2; ++i) pre[i] = s2[i];
        }
        if (qp < Bn.p1 - Bn.p0) {
            const int p = Bn.p0 + qp;
            const double* pr = PRr + (size_t)p * NPR + qk * QS;
#pragma unroll
            for (int j = 0; j < QS; ++j)
                if (qk * QS + j < NPR) pre_pr[j] = pr[j];
            if (SCALEJ || qk == 0)
#pragma unroll
                for (int i = 0; i < 3; ++i) pre_sp[i] = scale[3 * (size_t)p + i];
            if (qk == 0)
#pragma unroll
                for (int i = 0; i < 3; ++i) pre_cs[i] = colsq[3 * (size_t)p + i];
        }
    };
    prefetch(w);
    for (int bi = w; bi < G.nb; bi += 4) {
        const Batch B = bl[bi];
        const int o = B.o0 + l, np = B.p1 - B.p0;
        // (point, local camera) -> lane map of this batch; cleared first (the wave's LDS operations
        // run in order, the fences keep the compiler's order)
        reinterpret_cast<int*>(omap)[l] = -1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (o < B.o1) {   // lane = observation: W_o -> its LDS row, its lane into the map
            double v[WST];
#pragma unroll
            for (int i = 0; i < WST / 2; ++i) { v[2 * i] = pre[i].x; v[2 * i + 1] = pre[i].y; }
            if (SCALEJ) scale_w(v, scale + 3 * (size_t)pre_p, scale + ne + 6 * (size_t)pre_c);   // W_s = diag(sp) W diag(sc)
            double2* wl = reinterpret_cast<double2*>(Wl + l * WST);
#pragma unroll
            for (int i = 0; i < WST / 2; ++i) wl[i] = make_double2(v[2 * i], v[2 * i + 1]);
            omap[pre_q * UMAX + pre_lc] = (signed char)l;
        }
        // point phase: the 4 lanes of a point put its record into the point's pw slot; after a wave
        // barrier lane k = 0 reads it back and does the rest
        if (qp < np) {
            double* ps = pw + qp * PD + qk * QS;
#pragma unroll
            for (int j = 0; j < QS; ++j)
                if (qk * QS + j < NPR) {
                    double vv = pre_pr[j];
                    if (SCALEJ) vv = vv * pr_scale<K>(qk * QS + j, pre_sp, si);
                    ps[j] = vv;
                }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        BA_STAMP(3);
        double Mq[6] = {0, 0, 0, 0, 0, 0}, tq[3] = {0, 0, 0};
        if (qp < np && qk == 0) {
            double* pq = pw + qp * PD;
            double E6[6], g[3], V[3 * K];
#pragma unroll
            for (int i = 0; i < 6; ++i) E6[i] = pq[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) g[i] = pq[6 + i];
#pragma unroll
            for (int i = 0; i < 3 * K; ++i) V[i] = pq[9 + i];
            double E[9] = {E6[0], E6[1], E6[2], E6[1], E6[3], E6[4], E6[2], E6[4], E6[5]};
#pragma unroll
            for (int i = 0; i < 3; ++i) E[4 * i] += dsq(pre_cs[i], pre_sp[i], dmin, dmax, radius);
            if (!chol3_inv(E, Mq)) {
                atomicOr(fail, 1);
#pragma unroll
                for (int i = 0; i < 6; ++i) Mq[i] = 0.0;
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                tq[k] = 0.0;
#pragma unroll
                for (int j = 0; j <= k; ++j) tq[k] += mlo(Mq, k, j) * g[j];
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) pq[i] = Mq[i];
#pragma unroll
            for (int k = 0; k < 3; ++k) pq[6 + k] = tq[k];
#pragma unroll
            for (int i = 0; i < K; ++i)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double h = 0.0;
#pragma unroll
                    for (int j = 0; j <= k; ++j) h += mlo(Mq, k, j) * V[j * K + i];
                    pq[9 + 3 * i + k] = h;
                }
        }
        prefetch(bi + 4);
        if (qp < np && qk == 0) {   // after the prefetch: a later wait for its loads does not wait for these stores
            const int p = B.p0 + qp;
#pragma unroll
            for (int i = 0; i < 6; ++i) plt[9 * (size_t)p + i] = Mq[i];
#pragma unroll
            for (int k = 0; k < 3; ++k) plt[9 * (size_t)p + 6 + k] = tq[k];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        BA_STAMP(4);
        // rounds of 4 points: lane (m16, kk) forms its own SYRK operands straight from LDS, rows
        // 16I + m16 of H of the round's point kk: a camera row (lc, d) is Z_o[d] = (M W_o[:, d])
        // of the point's observation o in camera lc (zero without one), an intrinsics row Hi
        for (int r0 = 0; r0 < np; r0 += 4) {
            double hv[NT][3];
            double tk[3] = {0, 0, 0};
            const int q = r0 + kk;
            if (q < np) {
                const double* pq = pw + q * PD;
                double Mr[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) Mr[i] = pq[i];
                tk[0] = pq[6]; tk[1] = pq[7]; tk[2] = pq[8];
#pragma unroll
                for (int I = 0; I < NT; ++I) {
                    const int r = 16 * I + m16;
                    hv[I][0] = hv[I][1] = hv[I][2] = 0.0;
                    if (r < 6 * G.u) {
                        const int lc = r / 6, d = r - 6 * lc, lo = omap[q * UMAX + lc];
                        if (lo >= 0) {
                            const double* wo = Wl + lo * WST + d;
                            const double w0 = wo[0], w1 = wo[6], w2 = wo[12];
                            hv[I][0] = Mr[0] * w0;
                            hv[I][1] = Mr[1] * w0 + Mr[2] * w1;
                            hv[I][2] = Mr[3] * w0 + Mr[4] * w1 + Mr[5] * w2;
                        }
                    } else if (r < dim) {
                        const double* hi = pq + 9 + 3 * (r - 6 * G.u);
                        hv[I][0] = hi[0]; hv[I][1] = hi[1]; hv[I][2] = hi[2];
                    }
                }
            } else {
#pragma unroll
                for (int I = 0; I < NT; ++I) hv[I][0] = hv[I][1] = hv[I][2] = 0.0;
            }
            BA_STAMP(5);
#pragma unroll
            for (int I = 0, t = 0; I < NT; ++I)
#pragma unroll
                for (int Jt = I; Jt < NT; ++Jt, ++t) {
                    if (Jt >= nt) continue;
#pragma unroll
                    for (int c = 0; c < 3; ++c) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(hv[I][c], hv[Jt][c], acc[t], 0, 0, 0);
                }
#pragma unroll
            for (int I = 0; I < NT; ++I) racc[I] += hv[I][0] * tk[0] + hv[I][1] * tk[1] + hv[I][2] * tk[2];
        }
        // the next batch rewrites Wl / pw / omap only after every lane's reads of this one
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        BA_STAMP(0);
    }
    // rhs: the 4 points of a round sit in the 4 lane groups: sum them (fixed order)
#pragma unroll
    for (int I = 0; I < NT; ++I) {
        const double a = racc[I] + __shfl_xor(racc[I], 16);   // lanes m, m+16 | m+32, m+48
        racc[I] = a + __shfl_xor(a, 32);
    }
    if constexpr (NT <= 3) {
        lds_barrier();   // (the last batch's plt stores stay in flight: nothing here reads them)
        // r06: every wave stores its tiles and rhs into its own LDS partial at once, one barrier, then all
        // 256 threads form each output element as ((p0 + p1) + p2) + p3 -- the association of the
        // wave-by-wave combine below, so the same bits -- with no chain of four store / barrier rounds
        // (the combine was ≈ 12 k cycles of a workgroup's ≈ 83 k, profiles/r06o_ba_stamps.txt).
        // gs_comb(NT) doubles: 4 x [NTT][256] | 4 x [16 NT]; NT = 4 would not fit two workgroups per CU.
        double* Pt = gl;                               // [4][NTT][256]
        double* Pr = gl + 4 * NTT * 256;               // [4][16 NT]
#pragma unroll
        for (int I = 0, t = 0; I < NT; ++I)
#pragma unroll
            for (int Jt = I; Jt < NT; ++Jt, ++t) {
                if (Jt >= nt) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) Pt[(w * NTT + t) * 256 + (kk + 4 * r) * 16 + m16] = acc[t][r];
            }
        if (l < 16)
#pragma unroll
            for (int I = 0; I < NT; ++I)
                if (I < nt) Pr[w * 16 * NT + 16 * I + l] = racc[I];
        lds_barrier();
        BA_STAMP(1);
        double* Sg = sg + G.sg_off;
        for (int e = tid; e < dim * dim; e += 256) {
            const int r0 = e / dim, c0 = e % dim, r = r0 <= c0 ? r0 : c0, c = r0 <= c0 ? c0 : r0;
            const int I = r >> 4, Jt = c >> 4, t = I * NT - I * (I - 1) / 2 + (Jt - I);
            const int at = t * 256 + (r & 15) * 16 + (c & 15);
            Sg[e] = -(((Pt[at] + Pt[NTT * 256 + at]) + Pt[2 * NTT * 256 + at]) + Pt[3 * NTT * 256 + at]);
        }
        if (tid < dim)
            rg[G.rg_off + tid] = -(((Pr[tid] + Pr[16 * NT + tid]) + Pr[32 * NT + tid]) + Pr[48 * NT + tid]);
        BA_STAMP(2);
        BA_FLUSH(0);
        return;
    }
    // NT = 4: combine the 4 waves' tiles and rhs in wave order: [dp][dp + 1] | rhs[dp]
    __syncthreads();
    double* Sb = gl;
    double* Rb = gl + dp * (dp + 1);
    for (int ww = 0; ww < 4; ++ww) {
        if (w == ww) {
            double prev[NTT][4];   // all reads first: the stores may alias them for the compiler
#pragma unroll
            for (int I = 0, t = 0; I < NT; ++I)
#pragma unroll
                for (int Jt = I; Jt < NT; ++Jt, ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        prev[t][r] = (ww == 0 || Jt >= nt) ? 0.0 : Sb[(16 * I + kk + 4 * r) * (dp + 1) + 16 * Jt + m16];
#pragma unroll
            for (int I = 0, t = 0; I < NT; ++I)
#pragma unroll
                for (int Jt = I; Jt < NT; ++Jt, ++t) {
                    if (Jt >= nt) continue;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = 16 * I + kk + 4 * r, col = 16 * Jt + m16;
                        Sb[row * (dp + 1) + col] = ww == 0 ? acc[t][r] : prev[t][r] + acc[t][r];
                    }
                }
            if (l < 16)
#pragma unroll
                for (int I = 0; I < NT; ++I)
                    if (I < nt) Rb[16 * I + l] = ww == 0 ? racc[I] : Rb[16 * I + l] + racc[I];
        }
        __syncthreads();
    }
    BA_STAMP(1);
    // -sum H H^T (full square from the upper tiles) and -sum H t
    double* Sg = sg + G.sg_off;
    for (int e = tid; e < dim * dim; e += 256) {
        const int r = e / dim, c = e % dim;
        Sg[e] = -(r <= c ? Sb[r * (dp + 1) + c] : Sb[c * (dp + 1) + r]);
    }
    if (tid < dim) rg[G.rg_off + tid] = -Rb[tid];
    BA_STAMP(2);
    BA_FLUSH(0);
}

// ---------------------------------------------------------------------------------------------
// ba_assemble: one 256-thread workgroup per block of the reduced system, summing the group
// contributions (normal groups: their dense block; big groups: -H_a H_b^T from the stored H).
// Bordered layout (ba_chol.hpp): pose blocks into S_cc at the plan's camera rows (and the
// transpose), pose-intrinsics blocks and the camera rhs into R = [B | r_c], the intrinsics block and
// rhs into D / r_i.  Everything is zeroed before; C, D^2 and g_f are added by ba_add_cam (after any
// cross-rank all-reduce).  A block's entry list (a pose pair of C5 is held by ~80 groups, the
// intrinsics by every group) is split over the workgroup: thread (part, output) sums the entries
// part, part + NP, ... (NP = 256 / outputs), the parts are then added in part order (fixed,
// deterministic); the intrinsics outputs (one per workgroup) reduce their 256 strided partials by
// waves.  r02 ran one thread per output over the whole list, a chain of dependent loads per entry.
__device__ __forceinline__ double aval(const AEnt& E, const double* __restrict__ sg, const double* __restrict__ hbig,
                                       int r, int c) {
    if (!E.big) return sg[E.b0 + (long long)r * E.dim + c];
    const double* Ha = hbig + E.b0 + 3 * r;
    const double* Hb = hbig + E.b1 + 3 * c;
    return -(Ha[0] * Hb[0] + Ha[1] * Hb[1] + Ha[2] * Hb[2]);
}
// ba_add_cam's terms, one rounding per operation (no contraction), shared by ba_add_cam (point-sharded
// ranks: added after the all-reduce) and ba_assemble's fused form (one rank, r06), so both give the
// same bits: the camera-camera block entry (u, w) (+ D^2 on the diagonal), camera-intrinsics B entry,
// camera gradient, intrinsics block entry, intrinsics gradient
// (HIP's __dadd_rn / __dmul_rn are plain + / * here, which the compiler may contract into an FMA with
// a neighbouring multiply depending on the surrounding code: these two never contract, so a term gives
// the same bits whichever kernel forms it)
__device__ __forceinline__ double add_nc(double a, double b) {
#pragma clang fp contract(off)
    return a + b;
}
__device__ __forceinline__ double mul_nc(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ int sym_idx(int a, int b, int n) {   // packed upper-triangle index of (a, b), a <= b
    int e = 0;
    for (int x = 0; x < a; ++x) e += n - x;
    return e + b - a;
}
__device__ __forceinline__ double cam_cc_term(const double* cs, const double* sc, const double* colsq_c, int u, int w,
                                              double dmin, double dmax, double radius) {
    double v = mul_nc(mul_nc(sc[u], sc[w]), cs[sym_idx(u < w ? u : w, u < w ? w : u, 6)]);
    if (u == w) v = add_nc(v, dsq(colsq_c[u], sc[u], dmin, dmax, radius));
    return v;
}
__device__ __forceinline__ double cam_ci_term(const double* cs, const double* sc, const double* si, int K, int u, int i) {
    return mul_nc(mul_nc(sc[u], si[i]), cs[cp_ci(K) + u * K + i]);
}
__device__ __forceinline__ double cam_g_term(const double* cs, const double* sc, int K, int u) {
    return mul_nc(sc[u], cs[cp_gc(K) + u]);
}
__device__ __forceinline__ double intr_ii_term(const double* ii, const double* si, const double* colsq_i, int K, int i, int j,
                                               double dmin, double dmax, double radius) {
    double v = mul_nc(mul_nc(si[i], si[j]), ii[sym_idx(i < j ? i : j, i < j ? j : i, K)]);
    if (i == j) v = add_nc(v, dsq(colsq_i[i], si[i], dmin, dmax, radius));
    return v;
}
__device__ __forceinline__ double intr_g_term(const double* ii, const double* si, int K, int i) {
    return mul_nc(si[i], ii[K * (K + 1) / 2 + i]);
}
__device__ __forceinline__ double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
constexpr int ASM_THREADS = 256, ASM_BATCH = 8;
// ASM_BATCH entries e0, e0 + step, ... (< l1) of a block's list: every entry record loaded, then every
// value (the normal groups' sg element, a big group's H rows, or the rhs rg element), so one batch costs
// two memory round trips instead of two per entry (r06: the lists are 80-2000 entries long, and a
// thread walked its share one dependent pair of loads at a time)
template <int NB_>
__device__ __forceinline__ void asm_batch(const AEnt* __restrict__ ents, const double* __restrict__ sg,
                                          const double* __restrict__ hbig, const double* __restrict__ rg, int e0,
                                          int step, int l1, bool rhs, int r, int c, double (&xv)[NB_]) {
    AEnt E[NB_];
#pragma unroll
    for (int k = 0; k < NB_; ++k)
        if (e0 + k * step < l1) E[k] = ents[e0 + k * step];
#pragma unroll
    for (int k = 0; k < NB_; ++k) {
        xv[k] = 0.0;
        if (e0 + k * step < l1) xv[k] = rhs ? rg[E[k].rg + r] : aval(E[k], sg, hbig, r, c);
    }
}
// stamps (diagnostic stamp build): per task type the longest workgroup's load phase, slots 32 + 2 type
#ifdef SFMX_BA_STAMPS
#define ASM_STAMP_END(type)                                                                        \
    do {                                                                                           \
        if (threadIdx.x == 0) {                                                                    \
            const long long d_ = (long long)__builtin_amdgcn_s_memtime() - ba_t_;                  \
            atomicAdd(&g_ba_stamps[32 + 2 * (type)], 1ull);                                        \
            atomicMax(&g_ba_stamps[33 + 2 * (type)], (unsigned long long)d_);                      \
        }                                                                                          \
    } while (0)
#else
#define ASM_STAMP_END(type) do { } while (0)
#endif
__global__ __launch_bounds__(ASM_THREADS)
void ba_assemble(const ATask* __restrict__ tasks, const AEnt* __restrict__ ents, const double* __restrict__ sg,
                 const double* __restrict__ hbig, const double* __restrict__ rg, int K, const int* __restrict__ camrow,
                 int npad, double* __restrict__ S, double* __restrict__ R, double* __restrict__ Dm,
                 double* __restrict__ ri, const int* __restrict__ gate, int fuse, int P, int C,
                 const double* __restrict__ camsum, const double* __restrict__ scale, const double* __restrict__ colsq,
                 double dmin, double dmax, double radius, const double* __restrict__ lm) {
    if (step_gated(gate)) return;
    BA_T0();
    if (fuse && lm) radius = lm[LM_RADIUS];
    __shared__ double part[ASM_THREADS];
    const ATask T = tasks[blockIdx.x];
    const int t = threadIdx.x, RW = K + 1;
    // fuse (one rank, r06): each output takes ba_add_cam's term as it is written, s + v in that order
    // (ba_add_cam added v to the stored s): the camera-camera C block + D^2, the camera-intrinsics part of
    // B and the camera gradient, the intrinsics block + D^2 and gradient (camsum unscaled, all-reduced)
    const int NCP = ncp(K);
    const size_t ne = 3 * (size_t)P, nfc = 6 * (size_t)C;
    const double* si = scale + ne + nfc;
    if (T.type == 2) {          // one intrinsics output x = T.b over every group; entries at the intrinsics rows
        const int x = T.b;
        double v0 = 0.0, v1 = 0.0;   // the thread's entries k = 0, 1, 2, ... alternate between two chains
        const bool blk = x < K * K;
        const int i = blk ? x / K : x - K * K, j = blk ? x % K : 0;   // (rhs: rg row i)
        for (int e0 = T.l0 + t; e0 < T.l1; e0 += ASM_BATCH * ASM_THREADS) {
            double xv[ASM_BATCH];
            asm_batch<ASM_BATCH>(ents, sg, hbig, rg, e0, ASM_THREADS, T.l1, !blk, i, j, xv);
#pragma unroll
            for (int k = 0; k < ASM_BATCH; k += 2) {   // (ASM_BATCH even: k keeps its parity across batches)
                if (e0 + k * ASM_THREADS < T.l1) v0 += xv[k];
                if (e0 + (k + 1) * ASM_THREADS < T.l1) v1 += xv[k + 1];
            }
        }
        ASM_STAMP_END(2);
        const double v = wave_sum(v0 + v1);
        if ((t & 63) == 0) part[t >> 6] = v;
        __syncthreads();
        if (t == 0) {
            double s = ((part[0] + part[1]) + part[2]) + part[3];
            if (fuse & 4) {
                const double* ii = camsum + (size_t)C * NCP;
                s = add_nc(s, x < K * K ? intr_ii_term(ii, si, colsq + ne + nfc, K, x / K, x % K, dmin, dmax, radius)
                                           : intr_g_term(ii, si, K, x - K * K));
            }
            if (x < K * K) Dm[x] = s;
            else ri[x - K * K] = s;
        }
        return;
    }
    // type 0: the 6 x 6 pose block (a, b); type 1: camera a's 6 x K block of B and its 6 rhs entries
    const int nout = T.type == 0 ? 36 : 6 * K + 6;
    const int np = ASM_THREADS / nout, o = t % nout, pt = t / nout;
    double v = 0.0;
    if (pt < np) {
        const bool rhs = T.type == 1 && o >= 6 * K;
        const int r = T.type == 0 ? o / 6 : (rhs ? o - 6 * K : o / K), c = T.type == 0 ? o % 6 : o % K;
        for (int e0 = T.l0 + pt; e0 < T.l1; e0 += ASM_BATCH * np) {
            double xv[ASM_BATCH];
            asm_batch<ASM_BATCH>(ents, sg, hbig, rg, e0, np, T.l1, rhs, r, c, xv);
#pragma unroll
            for (int k = 0; k < ASM_BATCH; ++k)
                if (e0 + k * np < T.l1) v += xv[k];
        }
        part[t] = v;
    }
    ASM_STAMP_END(T.type);
    __syncthreads();
    if (t < nout) {
        double s = part[t];
        for (int q = 1; q < np; ++q) s += part[q * nout + t];
        if (T.type == 0) {
            const int u = t / 6, w = t % 6, ra = camrow[T.a], rb = camrow[T.b];
            if ((fuse & 1) && T.a == T.b)   // camera T.a's diagonal block
                s = add_nc(s, cam_cc_term(camsum + (size_t)T.a * NCP, scale + ne + 6 * (size_t)T.a,
                                             colsq + ne + 6 * (size_t)T.a, u, w, dmin, dmax, radius));
            S[(size_t)(ra + u) * npad + rb + w] = s;
            if (T.a != T.b) S[(size_t)(rb + w) * npad + ra + u] = s;
        } else {
            const int ra = camrow[T.a];
            if (fuse & 2) {
                const double* cs = camsum + (size_t)T.a * NCP;
                const double* sc = scale + ne + 6 * (size_t)T.a;
                s = add_nc(s, t < 6 * K ? cam_ci_term(cs, sc, si, K, t / K, t % K) : cam_g_term(cs, sc, K, t - 6 * K));
            }
            if (t < 6 * K) R[(size_t)(ra + t / K) * RW + t % K] = s;
            else R[(size_t)(ra + t - 6 * K) * RW + K] = s;
        }
    }
}

// + the camera-camera part C of the scaled J^T J, D_f^2 and g_f: one workgroup per camera
// (blockIdx.x < C) and one for the intrinsics and the identity padding rows of S_cc.  camsum (per
// camera ncp(K) unscaled sums, then the intrinsics K(K+1)/2 + K) is already summed over ranks.
template <int K>
__global__ __launch_bounds__(64)
void ba_add_cam(int P, int C, int npad, const int* __restrict__ camrow, const int* __restrict__ padrows,
                int npadrows, const double* __restrict__ camsum,
                const double* __restrict__ scale, const double* __restrict__ colsq, double dmin, double dmax,
                double radius, double* __restrict__ S, double* __restrict__ R, double* __restrict__ Dm,
                double* __restrict__ ri, const int* __restrict__ gate, const double* __restrict__ lm, int fused = 0) {
    if (step_gated(gate)) return;
    if (lm) radius = lm[LM_RADIUS];
    constexpr int NCP = ncp(K), RW = K + 1;
    const size_t ne = 3 * (size_t)P, nfc = 6 * (size_t)C;
    const double* si = scale + ne + nfc;
    if ((int)blockIdx.x < C) {
        const int c = blockIdx.x, rc = camrow[c];
        const double* cs = camsum + (size_t)c * NCP;
        const double* sc = scale + ne + 6 * (size_t)c;
        for (int t = threadIdx.x; t < 42 + 6 * K; t += 64)
        if (t < 36 ? (fused & 1) : (fused & 2)) {
            continue;   // (ba_assemble added this term)
        } else if (t < 36) {
            const int u = t / 6, w = t % 6;
            double* d = &S[(size_t)(rc + u) * npad + rc + w];
            *d = add_nc(*d, cam_cc_term(cs, sc, colsq + ne + 6 * (size_t)c, u, w, dmin, dmax, radius));
        } else if (t < 36 + 6 * K) {
            const int x = t - 36, u = x / K, i = x % K;
            double* d = &R[(size_t)(rc + u) * RW + i];
            *d = add_nc(*d, cam_ci_term(cs, sc, si, K, u, i));
        } else if (t < 42 + 6 * K) {
            const int u = t - 36 - 6 * K;
            double* d = &R[(size_t)(rc + u) * RW + K];
            *d = add_nc(*d, cam_g_term(cs, sc, K, u));
        }
    } else {
        const double* ii = camsum + (size_t)C * NCP;
        for (int x = threadIdx.x; x < K * K + K && !(fused & 4); x += 64) {
            if (x < K * K) Dm[x] = add_nc(Dm[x], intr_ii_term(ii, si, colsq + ne + nfc, K, x / K, x % K, dmin, dmax, radius));
            else ri[x - K * K] = add_nc(ri[x - K * K], intr_g_term(ii, si, K, x - K * K));
        }
        for (int i = threadIdx.x; i < npadrows; i += 64) S[(size_t)padrows[i] * npad + padrows[i]] = 1.0;
    }
}

// Feature rows of the per-(group, camera) partials: each observation gives two rows (residual
// rows j = 0, 1) of NF(K) features [Jc (6) | Ji (K) | r], unscaled.  Their Gram matrix per camera
// holds every partial field (see ncp): D[u][w] = Jc^T Jc, D[u][6 + i] = Jc^T Ji, D[u][6 + K] =
// Jc^T r, D[6 + i][6 + l] = Ji^T Ji, D[6 + i][6 + K] = Ji^T r.
__host__ __device__ constexpr int nfeat(int K) { return 7 + K; }
// jer's row stride: 80 B keeps the 16-B alignment of the b128 reads and writes and moves a row 20
// banks on (64 B put every lane of a 16-lane read group on 4 bank sets: 12M conflict cycles, r04 PMC);
// K = 7 keeps 64 B: its 14 feature columns leave no room for two padded workgroups in 160 KiB
__host__ __device__ constexpr int jers(int K) { return K < 7 ? 10 : 8; }
template <int K>
__device__ __forceinline__ int field_of(int r, int c) {   // Gram entry (r <= c) -> partial field, -1: none
    if (r < 6) {
        if (c < 6) return 21 - (6 - r) * (7 - r) / 2 + (c - r);
        if (c < 6 + K) return 21 + r * K + (c - 6);
        return cp_gc(K) + r;
    }
    if (r < 6 + K) {
        const int i = r - 6;
        if (c < 6 + K) return cp_ii(K) + (K * (K + 1) / 2 - (K - i) * (K - i + 1) / 2) + (c - 6 - i);
        return cp_gi(K) + i;
    }
    return -1;   // r^T r (not a partial field)
}

// The same sums of a normal chunk's point in two halves on different waves (threads 0..127: E | g,
// colsq, grad; threads 128..255: V), each half in observation order as point_sums, with the scale
// products of pr_scale.
template <int K>
__device__ __forceinline__ void point_eg(const double* __restrict__ jer, int a0, int a1, int p,
                                         const double* __restrict__ jscale, double* __restrict__ colsq,
                                         double* __restrict__ grad, double* __restrict__ PRo, double& gmax) {
    constexpr int NPR = npr(K);
    double sv[3] = {1.0, 1.0, 1.0};   // loaded before any store of this thread (vmcnt order)
    if (jscale)
#pragma unroll
        for (int i = 0; i < 3; ++i) sv[i] = jscale[3 * (size_t)p + i];
    double pr[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) pr[i] = 0.0;
    for (int b = a0; b < a1; ++b) {
        const double* r = jer + b * jers(K);
        int e = 0;
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int v = u; v < 3; ++v) pr[e++] += r[u] * r[v] + r[3 + u] * r[3 + v];
#pragma unroll
        for (int u = 0; u < 3; ++u) pr[6 + u] += r[u] * r[6] + r[3 + u] * r[7];
    }
    constexpr int dg[3] = {0, 3, 5};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        colsq[3 * (size_t)p + i] = pr[dg[i]];
        grad[3 * (size_t)p + i] = pr[6 + i];
        gmax = fmax(gmax, fabs(pr[6 + i]));
    }
    if (jscale)
#pragma unroll
        for (int e = 0; e < 9; ++e) pr[e] = pr[e] * pr_scale<K>(e, sv, sv);
#pragma unroll
    for (int e = 0; e < 9; ++e) PRo[(size_t)p * NPR + e] = pr[e];
}
template <int K>
__device__ __forceinline__ void point_v(const double* __restrict__ jer, const double* __restrict__ G,
                                        const short* __restrict__ orw, int a0, int a1, int p, int P, int C,
                                        const double* __restrict__ jscale, double* __restrict__ PRo) {
    constexpr int NPR = npr(K), NF = nfeat(K);
    double sv[3] = {1.0, 1.0, 1.0}, sk[K];   // loaded before any store of this thread (vmcnt order)
#pragma unroll
    for (int i = 0; i < K; ++i) sk[i] = 1.0;
    if (jscale) {
        const double* si = jscale + 3 * (size_t)P + 6 * (size_t)C;
#pragma unroll
        for (int i = 0; i < 3; ++i) sv[i] = jscale[3 * (size_t)p + i];
#pragma unroll
        for (int i = 0; i < K; ++i) sk[i] = si[i];
    }
    double v[3 * K];
#pragma unroll
    for (int i = 0; i < 3 * K; ++i) v[i] = 0.0;
    for (int b = a0; b < a1; ++b) {
        const double* r = jer + b * jers(K);
        const double* g0 = G + orw[b] * NF;
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int i = 0; i < K; ++i) v[u * K + i] += r[u] * g0[6 + i] + r[3 + u] * g0[NF + 6 + i];
    }
    if (jscale)
#pragma unroll
        for (int e = 0; e < 3 * K; ++e) v[e] = v[e] * pr_scale<K>(9 + e, sv, sk);
#pragma unroll
    for (int e = 0; e < 3 * K; ++e) PRo[(size_t)p * NPR + 9 + e] = v[e];
}
// The LM step's point update (ba_gupdate): from sol_f (scaled
// camera/intrinsics solution), the stored M, t and the records: y_p = sum_o W_o sol_c(o) + V_p
// sol_i (= W_p sol_f), sol_e = M^T (t - M y), step = -sol; candidate points cand = x + step * scale;
// ||x - cand||^2; and the points' part of the model cost change, s.g + s^T E s / 2 - s.y with s the
// point's step: the sum of m (r + m / 2), m = J_s step, over the point's residuals, by blocks
// (s^T J^T r + |J s|^2 / 2 with J^T J's point rows E_p and W_p; the camera rows' part, s_f.g_f +
// s_f^T C s_f / 2, is ba_finalize's).
// y_o = W_o sol_c of the observation's camera (the back substitution's per-observation term)
// (jsp / jsc: the point's and the camera's Jacobi scales when the records are unscaled, else null:
// W_o scaled as it is read, each product rounded as scale_w stores it)
__device__ __forceinline__ void obs_y(const double* __restrict__ Wr, int o, const double* __restrict__ solc, double* __restrict__ y3,
                                      const double* __restrict__ jsp = nullptr, const double* __restrict__ jsc = nullptr) {
    const double2* s2 = reinterpret_cast<const double2*>(Wr + (size_t)o * WST);
    double wv[WST], sc[6];
#pragma unroll
    for (int i = 0; i < WST / 2; ++i) { const double2 t = s2[i]; wv[2 * i] = t.x; wv[2 * i + 1] = t.y; }
    if (jsp)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int d = 0; d < 6; ++d) wv[6 * a + d] = __dmul_rn(wv[6 * a + d], __dmul_rn(jsp[a], jsc[d]));
#pragma unroll
    for (int d = 0; d < 6; ++d) sc[d] = solc[d];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double yk = 0.0;
#pragma unroll
        for (int d = 0; d < 6; ++d) yk += wv[6 * k + d] * sc[d];
        y3[k] = yk;
    }
}
template <int K, bool SCALEJ = false>
__device__ __forceinline__ void point_step(int p, double (&y)[3], const double* __restrict__ PRr,
                                           const double* __restrict__ plt, const double (&soli)[K],
                                           const double* __restrict__ x, const double* __restrict__ scale,
                                           double* __restrict__ cand, double& model, double& sn, double (&cvo)[3],
                                           const double* __restrict__ si = nullptr) {
    constexpr int NPR = npr(K);
    double pr[NPR];   // (SCALEJ: the unscaled record scaled as it is read, the products rounded as stored)
#pragma unroll
    for (int e = 0; e < NPR; ++e) {
        const double v = PRr[(size_t)p * NPR + e];
        pr[e] = SCALEJ ? __dmul_rn(v, pr_scale<K>(e, scale + 3 * (size_t)p, si)) : v;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int i = 0; i < K; ++i) y[k] += pr[9 + k * K + i] * soli[i];
    const double* Mt = plt + 9 * (size_t)p;
    double v[3], st[3];
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
        st[j] = -s;                                 // step_s = -sol
        const double xv = x[3 * (size_t)p + j], cv = xv + st[j] * scale[3 * (size_t)p + j];
        cand[3 * (size_t)p + j] = cv;
        cvo[j] = cv;
        const double dd = xv - cv;
        sn += isfinite(dd) ? dd * dd : INFINITY;
    }
    const double q = pr[0] * st[0] * st[0] + pr[3] * st[1] * st[1] + pr[5] * st[2] * st[2] +
                     2.0 * (pr[1] * st[0] * st[1] + pr[2] * st[0] * st[2] + pr[4] * st[1] * st[2]);
    model += (st[0] * pr[6] + st[1] * pr[7] + st[2] * pr[8]) + 0.5 * q - (st[0] * y[0] + st[1] * y[1] + st[2] * y[2]);
}
// ba_glin: residuals + Jacobian at xp (x or the candidate) for the group's observations.
// Writes the step kernels' records (scaled by jscale when given: the solve's Jacobi scale): W_o per
// observation and E | g | V per point (see WST / npr); per point colsq / grad (unscaled: the diagonal
// of E and g before scaling); per (group, camera) partials (gpart: the per-camera Gram matrices of
// the feature rows on the fp64 matrix cores, rows of one camera contiguous and zero-padded by the
// host-built layout); and the group's cost, sum xp^2 (its points) and max |grad| partials.  Big
// groups: feature rows in observation order, a scalar per-(camera, field) loop, the point sums by
// thread 0 across the chunks.
// Dynamic LDS: G[max rows][NF] | jer[GCH][jers(K)] (je | r, padded) | olc[GCH] | orw[GCH]
// (short: camera slot, feature row of the observation).
constexpr int GROWS = 2 * GCH + 3 * UMAX;   // feature rows of a chunk incl. per-camera padding
// ba_glin's dynamic LDS (bytes) and the two workgroups per CU its launch bounds and group sizing assume
__host__ __device__ constexpr size_t glin_lds(int K) {
    return sizeof(double) * ((size_t)GROWS * nfeat(K) + (size_t)GCH * jers(K)) + sizeof(short) * 2 * GCH;
}
static_assert(2 * glin_lds(1) <= 160 * 1024 && 2 * glin_lds(3) <= 160 * 1024 && 2 * glin_lds(7) <= 160 * 1024,
              "two ba_glin workgroups per CU");
// the point sums of E | g | V over observations b in [a0, a1) of a chunk: Je and r from jer, Ji from
// the observation's feature rows (unscaled)
template <int K>
__device__ __forceinline__ void point_sums(const double* __restrict__ jer, const double* __restrict__ G,
                                           const short* __restrict__ orw, int a0, int a1, double (&pr)[npr(K)]) {
    constexpr int NF = nfeat(K);
    for (int b = a0; b < a1; ++b) {
        const double* r = jer + b * jers(K);
        const double* g0 = G + orw[b] * NF;
        int e = 0;
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int v = u; v < 3; ++v) pr[e++] += r[u] * r[v] + r[3 + u] * r[3 + v];
#pragma unroll
        for (int u = 0; u < 3; ++u) pr[6 + u] += r[u] * r[6] + r[3 + u] * r[7];
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int i = 0; i < K; ++i) pr[9 + u * K + i] += r[u] * g0[6 + i] + r[3 + u] * g0[NF + 6 + i];
    }
}
// colsq / grad of the point (unscaled), then its record (scaled) -> PRo
template <int K>
__device__ __forceinline__ void point_store(int p, int P, int C, double (&pr)[npr(K)], const double* __restrict__ jscale,
                                            double* __restrict__ colsq, double* __restrict__ grad,
                                            double* __restrict__ PRo, double& gmax) {
    constexpr int NPR = npr(K);
    constexpr int dg[3] = {0, 3, 5};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        colsq[3 * (size_t)p + i] = pr[dg[i]];
        grad[3 * (size_t)p + i] = pr[6 + i];
        gmax = fmax(gmax, fabs(pr[6 + i]));
    }
    if (jscale) {
        const double* sp = jscale + 3 * (size_t)p;
        const double* si = jscale + 3 * (size_t)P + 6 * (size_t)C;
        const double sv[3] = {sp[0], sp[1], sp[2]};
        double sk[K];
#pragma unroll
        for (int i = 0; i < K; ++i) sk[i] = si[i];
#pragma unroll
        for (int e = 0; e < NPR; ++e) pr[e] = pr[e] * pr_scale<K>(e, sv, sk);
    }
    double2* d2 = reinterpret_cast<double2*>(PRo + (size_t)p * NPR);
#pragma unroll
    for (int i = 0; i < NPR / 2; ++i) d2[i] = make_double2(pr[2 * i], pr[2 * i + 1]);
}
// MULTI: several cameras, each pose's block and principal point from (pim, pcc) (project_blk).
template <int K, bool MULTI = false>
__global__ __launch_bounds__(256, 2)
void ba_glin(const Grp* __restrict__ grp, const Chunk* __restrict__ chk, const int* __restrict__ lcrow,
             const short* __restrict__ obs_lc, const short* __restrict__ obs_row, const int* __restrict__ obs_point,
             const int* __restrict__ obs_cam, const double* __restrict__ obs_xy, const int* __restrict__ pt_start,
             double cx, double cy, int P, int C, const double* __restrict__ xp, const double* __restrict__ jscale,
             double* __restrict__ Wo, double* __restrict__ PRo, double* __restrict__ colsq, double* __restrict__ grad,
             double* __restrict__ gpart, double* __restrict__ gpl, const int* __restrict__ gate,
             const int* __restrict__ pim, const double2* __restrict__ pcc) {
    if (step_gated(gate)) return;
    extern __shared__ __attribute__((aligned(16))) double gl[];
    constexpr int JS = jst(K), NCP = ncp(K), N = 9 + K, NF = nfeat(K), NPR = npr(K);
    __shared__ double sh[8];
    double* G = gl;                                    // [GROWS][NF]
    double* jer = G + GROWS * NF;                      // [GCH][jers(K)]
    short* olc = reinterpret_cast<short*>(jer + GCH * jers(K));
    short* orw = olc + GCH;
    const Grp Gp = grp[blockIdx.x];
    // w through readfirstlane: the per-camera row ranges (lcrow of camera w + 4i) become scalar, so
    // the Gram loop's bounds and its tail conditions are scalar branches, not exec-masked lanes
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63, m16 = l & 15, kq = l >> 4;
    const double* pts = xp;
    const double* poses = xp + 3 * (size_t)P;
    const double* intr = poses + 6 * (size_t)C;
    double cost = 0.0, xn = 0.0, gmax = 0.0;
    f64x4 acc[UMAX / 4];
#pragma unroll
    for (int i = 0; i < UMAX / 4; ++i) acc[i] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int npart = Gp.u * NCP;
    __shared__ double bpr[npr(7)];   // big groups: the point's sums across the chunks (thread 0)
    if (tid < NPR) bpr[tid] = 0.0;
    if (Gp.big)
        for (int i = tid; i < npart; i += blockDim.x) gpart[(size_t)Gp.cam_off * NCP + i] = 0.0;
    const int nchunks = Gp.big ? (Gp.o1 - Gp.o0 + GCH - 1) / GCH : Gp.nch;
    BA_T0();
    for (int c = 0; c < nchunks; ++c) {
        Chunk ch;
        if (Gp.big) { ch.o0 = Gp.o0 + c * GCH; ch.o1 = min(Gp.o1, ch.o0 + GCH); ch.q0 = 0; ch.q1 = 0; ch.lc0 = 0; ch.nrows = 2 * (ch.o1 - ch.o0); }
        else ch = chk[Gp.ch0 + c];
        // every global load of the chunk goes out before its record stores: a wait for a load issued
        // after the stores would wait for the stores too (vmcnt counts both, in order)
        const int a = tid, o = ch.o0 + a;
        // point threads: tid and tid + 128 hold point q0 + (tid & 127) (its E | g and V halves); the
        // point's norm is the first half's
        const int qv = tid & 127;
        const bool pth = !Gp.big && qv >= ch.q0 && qv < ch.q1;
        const bool ptl = pth && tid < 128;
        int pa0 = 0, pa1 = 0, orow = 0, olcv = 0;
        if (pth) {
            const int p = Gp.p0 + qv;
            pa0 = pt_start[p] - ch.o0;
            pa1 = pt_start[p + 1] - ch.o0;
            if (ptl)
#pragma unroll
                for (int i = 0; i < 3; ++i) xn += pts[3 * (size_t)p + i] * pts[3 * (size_t)p + i];
        }
        int cr0[UMAX / 4], cr1[UMAX / 4];
#pragma unroll
        for (int i = 0; i < UMAX / 4; ++i) {
            const int lc = w + 4 * i;
            cr0[i] = cr1[i] = 0;
            if (!Gp.big && lc < Gp.u) { cr0[i] = lcrow[ch.lc0 + lc]; cr1[i] = lcrow[ch.lc0 + lc + 1]; }
        }
        // a camera's rows are padded to a multiple of 4: 2 zero rows at its end when it has an odd
        // number of observations in the chunk.  Its last 2 rows are zeroed before the barrier; real
        // rows there are written after it.  Every other row the Gram and point sums read is written
        // by an observation (big groups: 2 rows per observation, no padding).
#pragma unroll
        for (int i = 0; i < UMAX / 4; ++i)
            if (cr1[i] > cr0[i] && l < 2 * NF) G[(cr1[i] - 2) * NF + l] = 0.0;
        if (o < ch.o1) {
            orow = Gp.big ? 2 * a : obs_row[o];
            olcv = obs_lc[o];
        }
        // r06: LDS-only barriers in the chunk loop of a normal group (the W_o / point record stores and
        // the next loads stay in flight); a big group exchanges its gpart sums through global memory
        if (Gp.big) __syncthreads(); else lds_barrier();
        BA_STAMP(0);
        if (o < ch.o1) {
            const int p = obs_point[o], cm = obs_cam[o];
            const double ox = obs_xy[2 * (size_t)o], oy = obs_xy[2 * (size_t)o + 1];
            DJet<N> X[3], ps[6], in[K], res[2];
#pragma unroll
            for (int i = 0; i < 3; ++i) X[i] = jvar<N>(pts[3 * (size_t)p + i], i);
#pragma unroll
            for (int i = 0; i < 6; ++i) ps[i] = jvar<N>(poses[6 * (size_t)cm + i], 3 + i);
            if constexpr (MULTI) {
                project_blk<K, N>(X, ps, intr, pim[cm], pcc[cm], ox, oy, res);
            } else {
#pragma unroll
                for (int i = 0; i < K; ++i) in[i] = jvar<N>(intr[i], 9 + i);
                project<K, N>(X, ps, in, ox, oy, cx, cy, res);
            }
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
            // the scales go out before any store (a load issued after a store waits for it: vmcnt
            // counts both, in order); the LDS stores below cover their latency
            double sv[9];
            if (jscale) {
                const double* sp = jscale + 3 * (size_t)p;
                const double* sc = jscale + 3 * (size_t)P + 6 * (size_t)cm;
#pragma unroll
                for (int i = 0; i < 3; ++i) sv[i] = sp[i];
#pragma unroll
                for (int i = 0; i < 6; ++i) sv[3 + i] = sc[i];
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) jer[a * jers(K) + i] = rec[2 + i];
            jer[a * jers(K) + 6] = rec[0];
            jer[a * jers(K) + 7] = rec[1];
            const int row = orow;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                double* gr = G + (row + j) * NF;
#pragma unroll
                for (int i = 0; i < 6; ++i) gr[i] = rec[8 + 6 * j + i];
#pragma unroll
                for (int i = 0; i < K; ++i) gr[6 + i] = rec[20 + K * j + i];
                gr[6 + K] = rec[j];
            }
            olc[a] = (short)olcv;
            orw[a] = (short)row;
            cost += res[0].a * res[0].a + res[1].a * res[1].a;
            {   // W_o = Je^T Jc (unscaled products, then the scale: the same values ba_gschur<SCALEJ> makes)
                double wv[WST];
#pragma unroll
                for (int u = 0; u < 3; ++u)
#pragma unroll
                    for (int d = 0; d < 6; ++d) {
                        wv[6 * u + d] = rec[2 + u] * rec[8 + d] + rec[5 + u] * rec[14 + d];
                        if (jscale) wv[6 * u + d] = wv[6 * u + d] * (sv[u] * sv[3 + d]);
                    }
                double2* dst = reinterpret_cast<double2*>(Wo + (size_t)o * WST);
#pragma unroll
                for (int i = 0; i < WST / 2; ++i) dst[i] = make_double2(wv[2 * i], wv[2 * i + 1]);
            }
        }
        BA_STAMP(1);
        if (Gp.big) __syncthreads(); else lds_barrier();
        BA_STAMP(2);
        const int no = ch.o1 - ch.o0;
        // per point: E | g | V of its observations (whole points in a normal chunk)
        if (!Gp.big) {
            if (pth) {   // wave-uniform halves
                if (tid < 128) point_eg<K>(jer, pa0, pa1, Gp.p0 + qv, jscale, colsq, grad, PRo, gmax);
                else point_v<K>(jer, G, orw, pa0, pa1, Gp.p0 + qv, P, C, jscale, PRo);
            }
            // per camera: Gram of its feature rows, accumulated over the group's chunks; the
            // operand reads go out 8 MFMA steps at a time, ahead of their MFMAs
#pragma unroll
            for (int i = 0; i < UMAX / 4; ++i) {
                const int lc = w + 4 * i;
                if (lc >= Gp.u) continue;
                const int r0 = cr0[i], r1 = cr1[i];
                for (int row = r0; row < r1; row += 32) {
                    double v[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int rr = row + 4 * u;
                        v[u] = (m16 < NF && rr < r1) ? G[(rr + kq) * NF + m16] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (row + 4 * u < r1) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[u], v[u], acc[i], 0, 0, 0);
                }
            }
        } else {
            if (tid == 0) {
                double pr[NPR];
#pragma unroll
                for (int i = 0; i < NPR; ++i) pr[i] = bpr[i];
                point_sums<K>(jer, G, orw, 0, no, pr);
#pragma unroll
                for (int i = 0; i < NPR; ++i) bpr[i] = pr[i];
            }
            for (int x = tid; x < npart; x += blockDim.x) {   // per (camera, field), in observation order
                const int lc = x / NCP, f = x % NCP;
                int fr = -1, fc = -1;
                for (int rr = 0; rr < NF && fr < 0; ++rr)
                    for (int cc = rr; cc < NF; ++cc)
                        if (field_of<K>(rr, cc) == f) { fr = rr; fc = cc; break; }
                double sum = 0.0;
                for (int b = 0; b < no; ++b) {
                    if (olc[b] != lc) continue;
                    const double* g0 = G + (2 * b) * NF;
                    sum += g0[fr] * g0[fc] + g0[NF + fr] * g0[NF + fc];
                }
                gpart[(size_t)Gp.cam_off * NCP + x] += sum;
            }
        }
        if (Gp.big) __syncthreads(); else lds_barrier();
        BA_STAMP(3);
    }
    if (!Gp.big) {
#pragma unroll
        for (int i = 0; i < UMAX / 4; ++i) {
            const int lc = w + 4 * i;
            if (lc >= Gp.u) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rr = trow(r), cc = tcol();
                if (rr <= cc && cc < NF) {
                    const int f = field_of<K>(rr, cc);
                    if (f >= 0) gpart[(size_t)(Gp.cam_off + lc) * NCP + f] = acc[i][r];
                }
            }
        }
    } else if (tid == 0) {
        const int p = Gp.p0;
        double pr[NPR];
#pragma unroll
        for (int i = 0; i < NPR; ++i) pr[i] = bpr[i];
        point_store<K>(p, P, C, pr, jscale, colsq, grad, PRo, gmax);
#pragma unroll
        for (int i = 0; i < 3; ++i) xn += pts[3 * (size_t)p + i] * pts[3 * (size_t)p + i];
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
    BA_STAMP(4);
    BA_FLUSH(8);
}

// ---------------------------------------------------------------------------------------------
// stamps of ba_camred (slots 24..31): phase totals, then per kind (camera / intrinsics workgroups) the
// workgroup count and the longest workgroup
#ifdef SFMX_BA_STAMPS
#define CAMRED_FLUSH(kind)                                                                         \
    do {                                                                                           \
        BA_FLUSH(24);                                                                              \
        if (threadIdx.x == 0) {                                                                    \
            const long long d_ = ba_acc_[0] + ba_acc_[1] + ba_acc_[2] + ba_acc_[3];                 \
            atomicAdd(&g_ba_stamps[28 + 2 * (kind)], 1ull);                                        \
            atomicMax(&g_ba_stamps[29 + 2 * (kind)], (unsigned long long)d_);                      \
        }                                                                                          \
    } while (0)
#else
#define CAMRED_FLUSH(kind) do { } while (0)
#endif
// ba_camred: per camera (one workgroup of 512) the partials of its (group, camera) slots ->
// camsum[c]: thread (part, field) sums the slots part, part + NP, ... (NP = 512 / NCP), the parts are
// added in part order (fixed).  Every field of the slot record is summed, the intrinsics ones too:
// camsum[c]'s intrinsics fields hold camera c's share of the intrinsics block and gradient, which
// ba_finalize folds over the cameras (fixed order) after the all-reduce.  (r06: until then one
// workgroup per intrinsics field gathered that field from every slot, 113 dependent rounds per
// thread at C5: 40-47 k cycles per workgroup against 7.6 k for a camera, profiles/r06o_ba_stamps.txt.)
constexpr int CRED_THREADS = 512;
template <int K>
__global__ __launch_bounds__(CRED_THREADS)
void ba_camred(int C, int nslots, const int* __restrict__ cref_start, const int* __restrict__ cref,
               const double* __restrict__ gpart, double* __restrict__ camsum, const int* __restrict__ gate) {
    if (step_gated(gate)) return;
    BA_T0();
    constexpr int NCP = ncp(K), NP = CRED_THREADS / NCP;
    __shared__ double part[CRED_THREADS];
    const int t = threadIdx.x;
    const int c = blockIdx.x, e0 = cref_start[c], e1 = cref_start[c + 1], f = t % NCP, pt = t / NCP;
    if (pt < NP) {
        double sacc = 0.0;
        int e = e0 + pt;
#pragma unroll 4
        for (; e < e1; e += NP) sacc += gpart[(size_t)cref[e] * NCP + f];
        part[t] = sacc;
    }
    __syncthreads();
    BA_STAMP(0);
    if (t < NCP) {
        double sm = part[t];
        for (int q = 1; q < NP; ++q) sm += part[q * NCP + t];
        camsum[(size_t)c * NCP + t] = sm;
    }
    BA_STAMP(1);
    CAMRED_FLUSH(0);
    (void)nslots;
}

// The intrinsics block and gradient: camsum[c]'s intrinsics fields summed over the cameras, one wave
// per field (lane l adds cameras l, l + 64, ... in order, then the wave's xor tree: a fixed order).
// Every thread of the workgroup calls it; tot[NI] in LDS, valid after the caller's next barrier.
// The loads go out 4 cameras at a time (one memory round trip per 256 cameras, not per 64).
template <int K>
__device__ __forceinline__ void fold_intrinsics(int C, const double* __restrict__ camsum, double* tot) {
    constexpr int NCP = ncp(K), NFC = cp_ii(K), NI = NCP - NFC;
    const int lane = threadIdx.x & 63, nw = (int)(blockDim.x >> 6);
    for (int f = (int)(threadIdx.x >> 6); f < NI; f += nw) {
        double s = 0.0;
        for (int c0 = lane; c0 < C; c0 += 256) {
            double v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int c = c0 + 64 * k;
                v[k] = c < C ? camsum[(size_t)c * NCP + NFC + f] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (c0 + 64 * k < C) s += v[k];
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) tot[f] = s;
    }
}

// NS sums and one maximum over a workgroup of up to 1024 threads in one pass: every value reduced
// within its wave (xor shuffles), then thread 0 adds the waves in wave order (the order of
// block_sum, value by value).  sh: 16 (NS + 1) doubles.  Results valid in thread 0.
template <int NS>
__device__ __forceinline__ void block_reduce(double (&v)[NS], double& mx, double* sh) {
#pragma unroll
    for (int i = 0; i < NS; ++i)
        for (int o = 32; o > 0; o >>= 1) v[i] += __shfl_xor(v[i], o);
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NS; ++i) sh[wid * (NS + 1) + i] = v[i];
        sh[wid * (NS + 1) + NS] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            double t = 0.0;
            for (int w = 0; w < nw; ++w) t += sh[w * (NS + 1) + i];
            v[i] = t;
        }
        double m = 0.0;
        for (int w = 0; w < nw; ++w) m = fmax(m, sh[w * (NS + 1) + NS]);
        mx = m;
    }
}

// ba_finalize (one workgroup of 1024): camera column norms / gradient from camsum, and the LM
// scalars: sums over the groups' partials (fixed order), max |grad|, the camera part of the
// step and parameter norms (candidate mode: cand vs x).
template <int K>
__global__ __launch_bounds__(1024)
void ba_finalize(int ngroups, int P, int C, const double* __restrict__ camsum, const double* __restrict__ gpl,
                 const double* __restrict__ xf_new, const double* __restrict__ xf_old, int cand_mode,
                 int* __restrict__ fail, double* __restrict__ colsq, double* __restrict__ grad,
                 double* __restrict__ scal, double* __restrict__ camsum_out, int ncs,
                 const double* __restrict__ pre, double* __restrict__ pub_dst, unsigned* __restrict__ pub_seq,
                 unsigned pub_v, const double* __restrict__ camsum_cur, const double* __restrict__ sol_f,
                 const double* __restrict__ scale_f) {
    if (step_gated(fail + 1)) return;
    constexpr int NCP = ncp(K), NI = K * (K + 1) / 2 + K;
    __shared__ double sh[16 * 8];
    __shared__ double itot[NI];
    const int t = threadIdx.x;
    BA_T0();
    fold_intrinsics<K>(C, camsum, itot);   // (ba_camred leaves the intrinsics per camera; barrier below)
    BA_STAMP(0);
    // the camera sums were all-reduced in a scratch buffer (a skipped speculative step reduces only
    // scratch): the linearization's own copy is written here, behind the gate
    // r06: every load-only loop first (group partials, the camera model part), the loops with stores
    // last: a load issued after a store waits for it (vmcnt counts both, in order), which serialised
    // the loops' memory round trips.  Each quantity keeps its per-thread order and the block reduction.
    const size_t ne = 3 * (size_t)P;
    const int nf = 6 * C + K;
    double gmax = 0.0, xn = 0.0, sn = 0.0;
    double g[5] = {0, 0, 0, 0, 0};
    if (!pre)
#pragma unroll 2
        for (int b = t; b < ngroups; b += blockDim.x) {
            const double* q = gpl + (size_t)b * GP_N;
            g[0] += q[GP_COST]; g[1] += q[GP_MODEL]; g[2] += q[GP_STEPN]; g[3] += q[GP_XN];
            g[4] = fmax(g[4], q[GP_GMAX]);
        }
    // candidate mode: the camera rows' part of the model cost change, d.g_f + d^T C d / 2 with the
    // step d = -sol_f * scale_f and C, g_f the current linearization's (all-reduced, unscaled) camera
    // sums: per camera its 6 x 6 block, its coupling to the intrinsics and its gradient, then the
    // intrinsics block (one more slot); fixed order (thread stride, then the block sum)
    double mf = 0.0;
    BA_STAMP(1);
    if (cand_mode) {
        const double* sif = scale_f + 6 * (size_t)C;
        double di[K];
#pragma unroll
        for (int i = 0; i < K; ++i) di[i] = -sol_f[6 * (size_t)C + i] * sif[i];
        for (int c = t; c <= C; c += blockDim.x) {
            double q = 0.0;
            if (c < C) {
                const double* cs = camsum_cur + (size_t)c * NCP;
                double dc[6];
#pragma unroll
                for (int u = 0; u < 6; ++u) dc[u] = -sol_f[6 * (size_t)c + u] * scale_f[6 * (size_t)c + u];
                int e = 0;
#pragma unroll
                for (int u = 0; u < 6; ++u)
#pragma unroll
                    for (int v = u; v < 6; ++v, ++e) {
                        const double m = dc[u] * cs[e] * dc[v];
                        q += u == v ? 0.5 * m : m;
                    }
#pragma unroll
                for (int u = 0; u < 6; ++u)
#pragma unroll
                    for (int i = 0; i < K; ++i) q += dc[u] * cs[cp_ci(K) + u * K + i] * di[i];
#pragma unroll
                for (int u = 0; u < 6; ++u) q += dc[u] * cs[cp_gc(K) + u];
            } else {
                const double* ii = camsum_cur + (size_t)C * NCP;
                int e = 0;
#pragma unroll
                for (int i = 0; i < K; ++i)
#pragma unroll
                    for (int j = i; j < K; ++j, ++e) {
                        const double m = di[i] * ii[e] * di[j];
                        q += i == j ? 0.5 * m : m;
                    }
#pragma unroll
                for (int i = 0; i < K; ++i) q += di[i] * ii[K * (K + 1) / 2 + i];
            }
            mf += q;
        }
    }
    BA_STAMP(2);
    __syncthreads();   // itot
    BA_STAMP(3);
    // two rows per thread per pass, both rows' loads ahead of both rows' stores
    const int bd = (int)blockDim.x;
    for (int i0 = t; i0 < nf; i0 += 2 * bd) {
        double cs[2], gr[2], xv[2], xo[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int i = i0 + r * bd;
            cs[r] = gr[r] = xv[r] = xo[r] = 0.0;
            if (i >= nf) continue;
            if (i < 6 * C) {
                const int c = i / 6, u = i % 6;
                int e = 0;
                for (int x = 0; x < u; ++x) e += 6 - x;
                cs[r] = camsum[(size_t)c * NCP + e];
                gr[r] = camsum[(size_t)c * NCP + cp_gc(K) + u];
            } else {
                const int ii = i - 6 * C;
                int e = 0;
                for (int x = 0; x < ii; ++x) e += K - x;
                cs[r] = itot[e];
                gr[r] = itot[K * (K + 1) / 2 + ii];
            }
            xv[r] = xf_new[i];
            if (cand_mode) xo[r] = xf_old[i];
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int i = i0 + r * bd;
            if (i >= nf) continue;
            colsq[ne + i] = cs[r];
            grad[ne + i] = gr[r];
            gmax = fmax(gmax, fabs(gr[r]));
            const double v = xv[r];
            xn += v * v;
            if (cand_mode) {
                const double d = xo[r] - v;
                sn += isfinite(d) ? d * d : INFINITY;
            }
        }
    }
    BA_STAMP(4);
    for (int i = t; i < ncs; i += blockDim.x)
        if ((unsigned)(i - C * NCP) >= (unsigned)NI) camsum_out[i] = camsum[i];
    if (t < NI) camsum_out[(size_t)C * NCP + t] = itot[t];   // (camsum_out may be camsum: other bytes)
    // one pass: the group sums (unless the all-reduced ones are given), the camera model part, the
    // camera parts of the parameter and step norms, and max |grad|
    double v[7] = {g[0], g[1], g[2], g[3], mf, xn, sn};
    double gm = fmax(gmax, g[4]);
    block_reduce<7>(v, gm, sh);
    BA_STAMP(5);
    if (t == 0) {
        const double s0 = pre ? pre[0] : v[0], s1 = pre ? pre[1] : v[1], s2 = pre ? pre[2] : v[2], s3 = pre ? pre[3] : v[3];
        const double m = pre ? fmax(gm, pre[4]) : gm;
        scal[SC_COST] = s0;
        scal[SC_MODEL] = cand_mode ? s1 + v[4] : s1;
        scal[SC_STEPN] = s2;
        scal[SC_XN] = s3;
        scal[SC_GMAX] = m;
        scal[SC_FAIL] = (double)*fail;   // bit 0: non-positive pivot / invalid step, bit 1: solve wait timed out
        scal[SC_STEPN_F] = v[6];
        scal[SC_XN_F] = v[5];
        // one rank: nothing is reduced after this kernel, so it publishes the scalars itself (ba_publish)
        if (pub_dst) publish_body(scal, SC_N, nullptr, 0, pub_dst, pub_seq, pub_v, fail);
    }
    BA_STAMP(6);
#ifdef SFMX_BA_STAMPS
    ba_acc_[7] = 1;   // calls
#endif
    BA_FLUSH(cand_mode ? 48 : 40);
}

// Point-sharded ranks: the rank's group sums (cost, model change, step and parameter norms: the
// loop of ba_finalize) and its max |grad| of the points, written behind the camera sums so the
// four sums travel in the camera-sum all-reduce (one collective per linearization fewer);
// out[4] (the max) stays outside the reduced range.  One workgroup of 1024.
__global__ __launch_bounds__(1024)
void ba_group_sums(int ngroups, const double* __restrict__ gpl, double* __restrict__ out, const int* __restrict__ gate) {
    if (step_gated(gate)) return;
    __shared__ double sh[16 * 5];
    const int t = threadIdx.x;
    double g[4] = {0, 0, 0, 0}, gm = 0.0;
    for (int b = t; b < ngroups; b += blockDim.x) {
        const double* q = gpl + (size_t)b * GP_N;
        g[0] += q[GP_COST]; g[1] += q[GP_MODEL]; g[2] += q[GP_STEPN]; g[3] += q[GP_XN];
        gm = fmax(gm, q[GP_GMAX]);
    }
    block_reduce<4>(g, gm, sh);
    if (t == 0) { out[0] = g[0]; out[1] = g[1]; out[2] = g[2]; out[3] = g[3]; out[4] = gm; }
}

// ba_gupdate: the LM step's point update (above).  One thread per observation of a chunk (its W_o:
// 9 independent 16-B loads) and one per point.  Workgroups past the groups do ba_fstep's work
// (the candidate cameras / intrinsics), so the step needs no launch of its own for it.  (Fusing it into the candidate's ba_glin, per chunk
// before the linearization, was measured slower: DESIGN.md §5.)
template <int K, bool SCALEJ>
__global__ __launch_bounds__(256)
void ba_gupdate(const Grp* __restrict__ grp, const Chunk* __restrict__ chk, const int* __restrict__ obs_cam,
                const int* __restrict__ obs_point,
                const int* __restrict__ pt_start, const double* __restrict__ Wr, const double* __restrict__ PRr,
                const double* __restrict__ scale, const double* __restrict__ plt, const double* __restrict__ sol_f,
                int P, int C, const double* __restrict__ x, double* __restrict__ cand, double* __restrict__ gpl,
                const int* __restrict__ gate, int ngroups, int nf) {
    if (step_gated(gate)) return;
    if ((int)blockIdx.x >= ngroups) {   // cand_f = x_f + (-sol_f) * scale_f (as ba_fstep)
        const int i = ((int)blockIdx.x - ngroups) * blockDim.x + threadIdx.x;
        const size_t ne = 3 * (size_t)P;
        if (i < nf) cand[ne + i] = x[ne + i] + (-sol_f[i]) * scale[ne + i];
        return;
    }
    __shared__ double yv[GCH * 3];
    __shared__ double sh[8];
    const Grp G = grp[blockIdx.x];
    const int tid = threadIdx.x;
    double soli[K];
#pragma unroll
    for (int i = 0; i < K; ++i) soli[i] = sol_f[6 * (size_t)C + i];
    double model = 0.0, sn = 0.0;
    double ybig[3] = {0, 0, 0};
    const int nchunks = G.big ? (G.o1 - G.o0 + GCH - 1) / GCH : G.nch;
    for (int c = 0; c < nchunks; ++c) {
        Chunk ch;
        if (G.big) { ch.o0 = G.o0 + c * GCH; ch.o1 = min(G.o1, ch.o0 + GCH); ch.q0 = 0; ch.q1 = 0; }
        else ch = chk[G.ch0 + c];
        const int o = ch.o0 + tid;
        int pa0 = 0, pa1 = 0;
        const bool ptl = tid >= ch.q0 && tid < ch.q1;
        if (ptl) {
            pa0 = pt_start[G.p0 + tid] - ch.o0;
            pa1 = pt_start[G.p0 + tid + 1] - ch.o0;
        }
        if (o < ch.o1) {
            const int cam = obs_cam[o];
            if (SCALEJ) obs_y(Wr, o, sol_f + 6 * (size_t)cam, yv + tid * 3, scale + 3 * (size_t)obs_point[o],
                              scale + 3 * (size_t)P + 6 * (size_t)cam);
            else obs_y(Wr, o, sol_f + 6 * (size_t)cam, yv + tid * 3);
        }
        if (G.big) __syncthreads(); else lds_barrier();   // (r06: the point stores of the last chunk stay in flight)
        if (G.big) {
            if (tid == 0)
                for (int b = 0; b < ch.o1 - ch.o0; ++b)
#pragma unroll
                    for (int k = 0; k < 3; ++k) ybig[k] += yv[b * 3 + k];
        } else if (ptl) {
            double y[3] = {0, 0, 0};
            for (int b = pa0; b < pa1; ++b)
#pragma unroll
                for (int k = 0; k < 3; ++k) y[k] += yv[b * 3 + k];
            double cv[3];
            point_step<K, SCALEJ>(G.p0 + tid, y, PRr, plt, soli, x, scale, cand, model, sn, cv, scale + 3 * (size_t)P + 6 * (size_t)C);
        }
        if (G.big) __syncthreads(); else lds_barrier();   // yv is rewritten by the next chunk
    }
    if (G.big && tid == 0) {
        double cv[3];
        point_step<K, SCALEJ>(G.p0, ybig, PRr, plt, soli, x, scale, cand, model, sn, cv, scale + 3 * (size_t)P + 6 * (size_t)C);
    }
    const double sm = block_sum(model, sh);
    const double ss = block_sum(sn, sh);
    if (tid == 0) {
        double* q = gpl + (size_t)blockIdx.x * GP_N;
        q[GP_MODEL] = sm;
        q[GP_STEPN] = ss;
    }
}

}  // namespace ba
}  // namespace sfmx
