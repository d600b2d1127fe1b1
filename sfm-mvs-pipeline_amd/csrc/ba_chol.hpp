// SPDX-License-Identifier: MIT
// sfmx bundle adjustment — solve of the reduced camera system on gfx950 (fp64 matrix cores).
//
// Ceres DENSE_SCHUR (CeresUtils.cpp:43-50) solves  [S_cc B; B^T D] [x_c; x_i] = [r_c; r_i]  with
// one dense LLT, the shared intrinsics block (k unknowns) last.  Here the same system is solved as
// a bordered one, in the order the factorization plan (ba_plan.hpp) gives:
//   * S_cc (6C camera rows, nested-dissection order, identity padding rows) by block LDL^T on 64x64
//     tiles, S_cc = L~ D~ L~^T, L~_ak = A_ak W_k, W_k = D~_k^-1, level by level (one launch per
//     level of the tile elimination tree, one workgroup per destination tile);
//   * the forward solve rides along with k + 1 right-hand sides R = [B | r_c]: y_a = R_a - sum
//     A_ak w_k, w_a = W_a y_a (RW = k + 1 columns);
//   * the intrinsics Schur complement D' = D - B^T S_cc^-1 B = D - sum_a y_a(B)^T w_a(B) and
//     r' = r_i - sum_a y_a(B)^T w_a(r_c) are summed per panel (fixed panel order), D' is factored
//     (k x k Cholesky) and x_i = D'^-1 r';
//   * back solve L~^T x_c = w(r_c) - w(B) x_i, level by level from the root.
// A non-positive pivot of any D~_k (scalar Cholesky pivots of the symmetric sweeps) or of D' is
// where Eigen's LLT on the whole matrix fails (in exact arithmetic the same condition: S is
// positive definite iff S_cc and D' are); LM treats it as an invalid step.
//
// Storage (SR buffer, row-major): S_cc npad x npad | R npad x RW | D k x k | r_i k.
//   lower tiles (a, b), a > b : A, updated in place until consumed
//   upper tile (k, a), a > k  : L~_ak^T (for the back solve)
//   W[k] (one 64x64 tile per panel), contrib[k] (k x RW per panel)
#pragma once
#include <hip/hip_runtime.h>

#include "ba_kernels.hpp"

namespace sfmx {
namespace ba {

constexpr int LDT = NB + 2;   // LDS row stride (doubles): 16-B aligned rows
// Bound of every in-launch wait without progress: 20 ms of the 100 MHz wall clock (the kernels take
// it as an argument; the diagnostic build can shorten it, SFMX_BA_DAG_TIMEOUT).  A wait that sees
// the polled version / flag move restarts its clock, so a preempted queue (ranks sharing a GPU, a
// profiler) only trips it when nothing at all advances.  Fail bits: 2 = chol_factor, 4 =
// chol_backsolve; the host then re-runs the step with the per-level launches.
constexpr long long DAG_TIMEOUT = 2000000;
enum { FAIL_PIVOT = 1, FAIL_FACTOR_WAIT = 2, FAIL_BACK_WAIT = 4 };
// global-address-space words for in-launch hand-offs (agent-scope atomics / sc1 accesses)
typedef __attribute__((address_space(1))) int g_i32;
typedef __attribute__((address_space(1))) unsigned long long g_u64;
__device__ __forceinline__ double ld_wt(const double* p) {   // sc1 load (bypasses this CU's L1)
    return __longlong_as_double((long long)__hip_atomic_load((g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_wt(double* p, double v) {   // sc1 (write-through) store
    __hip_atomic_store((g_u64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-B sc1 loads through a buffer resource (aux 16 = sc1 on gfx950; word 3 as for every gfx9 raw buffer)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const double* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ double2 ld_wt2(__amdgpu_buffer_rsrc_t rs, size_t elem) {
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(elem * 8), 0, 16));
}
// NB x NB fp64 tiles on the matrix cores (layout: f64x4 / trow / tcol in ba_kernels.hpp).  Wave w of an
// NTH = 4 NB thread block owns the row strip 16w..16w+15 and NW = NB / 16 16x16 column tiles.

__device__ __forceinline__ void tile_load(double (*dst)[LDT], const double* __restrict__ src, int ld) {
#pragma unroll
    for (int q = 0; q < NB * NB / (2 * NTH); ++q) {
        const int e = q * (2 * NTH) + 2 * threadIdx.x;
        *reinterpret_cast<double2*>(&dst[e / NB][e % NB]) = *reinterpret_cast<const double2*>(src + (size_t)(e / NB) * ld + e % NB);
    }
}
// the same from bytes another workgroup of this launch stored write-through (sc1 loads; elements of rs)
__device__ __forceinline__ void tile_load_wt(double (*dst)[LDT], __amdgpu_buffer_rsrc_t rs, size_t src, int ld) {
#pragma unroll
    for (int q = 0; q < NB * NB / (2 * NTH); ++q) {
        const int e = q * (2 * NTH) + 2 * threadIdx.x;
        *reinterpret_cast<double2*>(&dst[e / NB][e % NB]) = ld_wt2(rs, src + (size_t)(e / NB) * ld + e % NB);
    }
}
// tile_load_wt of the rows in 4-row chunks `chunks` only (the other rows of dst are not written)
__device__ __forceinline__ void tile_load_wt_rows(double (*dst)[LDT], __amdgpu_buffer_rsrc_t rs, size_t src, int ld, int chunks) {
#pragma unroll
    for (int q = 0; q < NB * NB / (2 * NTH); ++q) {
        const int e = q * (2 * NTH) + 2 * threadIdx.x;
        if ((chunks >> ((e / NB) >> 2)) & 1)
            *reinterpret_cast<double2*>(&dst[e / NB][e % NB]) = ld_wt2(rs, src + (size_t)(e / NB) * ld + e % NB);
    }
}
__device__ __forceinline__ void tile_regs_wt(f64x4 (&t)[NW], const double* __restrict__ src, int ld) {
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < NW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) t[c][r] = ld_wt(&src[(size_t)(16 * w + trow(r)) * ld + 16 * c + tcol()]);
}
__device__ __forceinline__ void tile_store_wt(const f64x4 (&t)[NW], double* __restrict__ dst, int ld) {
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < NW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) st_wt(&dst[(size_t)(16 * w + trow(r)) * ld + 16 * c + tcol()], t[c][r]);
}
__device__ __forceinline__ void tile_regs(f64x4 (&t)[NW], const double* __restrict__ src, int ld) {
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < NW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) t[c][r] = src[(size_t)(16 * w + trow(r)) * ld + 16 * c + tcol()];
}
__device__ __forceinline__ void tile_store(const f64x4 (&t)[NW], double* __restrict__ dst, int ld) {
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < NW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(size_t)(16 * w + trow(r)) * ld + 16 * c + tcol()] = t[c][r];
}

// acc[c] = A[strip] * B          (A, B row-major 64x64 in LDS)
__device__ __forceinline__ void mfma_nn(const double (*A)[LDT], const double (*B)[LDT], f64x4 acc[NW]) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, m = l & 15, kq = l >> 4;
#pragma unroll
    for (int c = 0; c < NW; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int st = 0; st < NB / 4; ++st) {
        const double av = A[16 * w + m][4 * st + kq];
#pragma unroll
        for (int c = 0; c < NW; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, B[4 * st + kq][16 * c + m], acc[c], 0, 0, 0);
    }
}
// acc[c] = A[strip] * X^T        (A, X row-major 64x64 in LDS)
__device__ __forceinline__ void mfma_nt(const double (*A)[LDT], const double (*X)[LDT], f64x4 acc[NW]) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, m = l & 15, kq = l >> 4;
#pragma unroll
    for (int c = 0; c < NW; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int st = 0; st < NB / 4; ++st) {
        const double av = A[16 * w + m][4 * st + kq];
#pragma unroll
        for (int c = 0; c < NW; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, X[16 * c + m][4 * st + kq], acc[c], 0, 0, 0);
    }
}

// The same products restricted to the structurally nonzero operands (r06, ba_plan.cpp row_masks):
// only the waves whose row strip is in `rows`, the output column tiles in `cols` and the 4-wide
// k-steps of the hull of `ks`; the skipped steps would add exact zeros, so every computed tile has
// the bits of the full product (up to the sign of a zero).  Masks are wave-uniform; the column set
// is a template argument (a switch over the 15 sets) so the k loop keeps the branch-free form whose
// LDS operand loads the compiler pipelines (a per-MFMA mask test made the r06 first form slower
// than the full product: 4.1 us for 36 MFMA steps per wave against 2.9 us for 64).
template <int CM, bool NT>
__device__ __forceinline__ void mfma_cm(const double (*A)[LDT], const double (*B)[LDT], f64x4 acc[NW], int w, int klo,
                                        int khi) {
    const int l = threadIdx.x & 63, m = l & 15, kq = l >> 4;
#pragma unroll 4
    for (int st = klo; st < khi; ++st) {
        const double av = A[16 * w + m][4 * st + kq];
#pragma unroll
        for (int c = 0; c < NW; ++c)
            if ((CM >> c) & 1)
                acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, NT ? B[16 * c + m][4 * st + kq] : B[4 * st + kq][16 * c + m],
                                                              acc[c], 0, 0, 0);
    }
}
template <bool NT>
__device__ __forceinline__ void mfma_masked(const double (*A)[LDT], const double (*B)[LDT], f64x4 acc[NW], int rows,
                                            int cols, int ks) {
    static_assert(NW == 4, "column-set dispatch over 4 column tiles");
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int c = 0; c < NW; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
    if (!((rows >> w) & 1) || !ks || !cols) return;
    const int klo = __builtin_ctz((unsigned)ks), khi = 32 - __builtin_clz((unsigned)ks);
    switch (cols & 15) {
#define SFMX_CM(v) case v: mfma_cm<v, NT>(A, B, acc, w, klo, khi); break;
        SFMX_CM(1) SFMX_CM(2) SFMX_CM(3) SFMX_CM(4) SFMX_CM(5) SFMX_CM(6) SFMX_CM(7) SFMX_CM(8) SFMX_CM(9)
        SFMX_CM(10) SFMX_CM(11) SFMX_CM(12) SFMX_CM(13) SFMX_CM(14) SFMX_CM(15)
#undef SFMX_CM
        default: break;
    }
}
// acc[c] = A[strip] * B restricted (A, B row-major 64x64 in LDS)
__device__ __forceinline__ void mfma_nn_m(const double (*A)[LDT], const double (*B)[LDT], f64x4 acc[NW], int rows,
                                          int cols, int ks) {
    mfma_masked<false>(A, B, acc, rows, cols, ks);
}
// acc[c] = A[strip] * X^T restricted
__device__ __forceinline__ void mfma_nt_m(const double (*A)[LDT], const double (*X)[LDT], f64x4 acc[NW], int rows,
                                          int cols, int ks) {
    mfma_masked<true>(A, X, acc, rows, cols, ks);
}

// r06: the masked products with their output tiles spread over the waves.  The tiles (strip of
// `rows`) x (column tile of `cols`) are listed row by row; tile q goes to wave q % NW, which keeps up
// to 4 of them (acc[i]: strip ts[i], column tile tc[i]).  Each tile is accumulated over the same
// k-steps in the same order as in mfma_masked, so its bits are those of the full product; only the
// waves share the work (mfma_masked leaves the waves of zero strips idle: 2 of 4 on the C5 chain).
__device__ __forceinline__ int nth_bit(int m, int i) {   // the i-th set bit of m (scalar)
    for (int b = 0; b < 4; ++b)
        if ((m >> b) & 1) { if (i == 0) return b; --i; }
    return 0;
}
template <int NTI, bool NT>
__device__ __forceinline__ void mfma_tiles(const double (*A)[LDT], const double (*B)[LDT], f64x4 acc[4], const int (&ts)[4],
                                           const int (&tc)[4], int klo, int khi) {
    const int l = threadIdx.x & 63, m = l & 15, kq = l >> 4;
#pragma unroll 4
    for (int st = klo; st < khi; ++st) {
#pragma unroll
        for (int i = 0; i < NTI; ++i)
            acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[16 * ts[i] + m][4 * st + kq],
                                                          NT ? B[16 * tc[i] + m][4 * st + kq] : B[4 * st + kq][16 * tc[i] + m],
                                                          acc[i], 0, 0, 0);
    }
}
template <bool NT>
__device__ __forceinline__ int mfma_spread(const double (*A)[LDT], const double (*B)[LDT], f64x4 acc[4], int rows, int cols,
                                           int ks, int (&ts)[4], int (&tc)[4]) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nr = __builtin_popcount(rows & 15), nc = __builtin_popcount(cols & 15);
    int nt = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        acc[i] = f64x4{0.0, 0.0, 0.0, 0.0};
        const int q = w + NW * i;
        ts[i] = tc[i] = 0;
        if (q < nr * nc) {
            ts[i] = nth_bit(rows, q / nc);
            tc[i] = nth_bit(cols, q % nc);
            nt = i + 1;
        }
    }
    if (!ks || !nt) return nt;
    const int klo = __builtin_ctz((unsigned)ks), khi = 32 - __builtin_clz((unsigned)ks);
    switch (nt) {
        case 1: mfma_tiles<1, NT>(A, B, acc, ts, tc, klo, khi); break;
        case 2: mfma_tiles<2, NT>(A, B, acc, ts, tc, klo, khi); break;
        case 3: mfma_tiles<3, NT>(A, B, acc, ts, tc, klo, khi); break;
        default: mfma_tiles<4, NT>(A, B, acc, ts, tc, klo, khi); break;
    }
    return nt;
}
// the spread tiles into an LDS tile buffer (row-major 64 x 64); the tiles outside rows x cols as zeros
__device__ __forceinline__ void spread_store(double (*dst)[LDT], const f64x4 (&acc)[4], const int (&ts)[4], const int (&tc)[4],
                                             int nt, int rows, int cols) {
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[16 * ts[i] + trow(r)][16 * tc[i] + tcol()] = acc[i][r];
#pragma unroll
    for (int c = 0; c < NW; ++c)   // wave w: the zero tiles of strip w
        if (!((rows >> w) & 1) || !((cols >> c) & 1))
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[16 * w + trow(r)][16 * c + tcol()] = 0.0;
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
//   inner: Qn = -A_BB^-1 (16x16) by wave 0 alone (no barriers, no LDS): 8 sweeps
//          of 2x2 pivot blocks, each lane holding a 2x2 block; the 2x2 pivot
//          inverse is closed-form and its two scalar pivots (a, det/a) are the
//          scalar Cholesky pivots, i.e. exactly where LLT would fail.
// diagnostic build only (r06): a timeline of the last chol_factor launch, per ticket 16 wall-clock stamps
// (0 start, 1 operands ready, 2 W_k ready, 3 W_k loaded, 4 G done, 5 update done, 6 task finisher known,
// 7 inverse start, 8-11 its sweeps, 12 W_k published, 13 end, 15 hw id),
// read by sfmx_ba_debug_chol_trace (tools/chol_trace.py)
constexpr int CHOL_TRACE_MAX = 512;
#ifdef SFMX_DIAG
__device__ long long g_chol_trace[CHOL_TRACE_MAX][16];
#define CHOL_TRACE(tk, i) do { if (threadIdx.x == 0 && (tk) < CHOL_TRACE_MAX) g_chol_trace[tk][i] = wall_clock64(); } while (0)
#else
#define CHOL_TRACE(tk, i) do { } while (0)
#endif
constexpr int LDP = 18;   // LDS row stride of the 16-wide panels (16-B aligned rows)
// chol_diag_tile's workspace: column panel [NB][LDP] | -A_BB^-1 [16][LDP] | inner panel [32] | one
// -M strip [16][LDP] per wave; it fits a tile buffer at NB = 64, not at NB = 32
constexpr int DIAG_WS = NB * LDP + 16 * LDP + 32 + NW * 16 * LDP;
constexpr bool DIAG_WS_IN_BUF = DIAG_WS <= NB * LDT;
#ifdef SFMX_CHOL_STAMPS   // tools/micro/chol_tile.hip: phase timestamps of block 0 (never in the product build)
__device__ long long g_chol_stamps[64];
#define CHOL_STAMP(i) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_chol_stamps[i] = wall_clock64(); } while (0)
#else
#define CHOL_STAMP(i) do { } while (0)
#endif

// (r04: a form passing the pivot, row and column blocks between lanes by v_readlane / ds_swizzle /
// ds_bpermute instead of this LDS panel -- 16 LDS-path ops per step instead of 1 store + 6 reads --
// measured slower: chol_factor 144 -> 165 us per LM step, profiles/r04a_ba_kernel_stats.txt; reverted.)
__device__ __forceinline__ void inner_inverse16(const double* __restrict__ Pc, int s, double* __restrict__ Qn,
                                                double* __restrict__ ipan, bool& bad) {
    // wave 0 only: Qn = -(Pc[16s + i][j])^-1, i, j < 16
    const int lane = threadIdx.x & 63, r = lane >> 3, c = lane & 7;
    double p[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int w = 0; w < 2; ++w) p[u][w] = Pc[(16 * s + 2 * r + u) * LDP + 2 * c + w];
#pragma unroll
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
        // q = -[a b; b d]^-1 = -adj / det.  The row panel's m = -A_iB q = (A_iB adj) / det: the
        // adjugate products run beside the reciprocal, so only one multiply follows it.
        const double a = b0.x, bb = b0.y, d = b1.y;
        double det = fma(a, d, -bb * bb);
        const bool badj = !(a > 0.0) || !isfinite(a) || !(det > 0.0) || !isfinite(det);   // branch-free
        bad |= badj;
        det = badj ? 1.0 : det;
        const double ai[2][2] = {{i0.x, i0.y}, {i1.x, i1.y}};
        double pre[2][2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            pre[u][0] = fma(ai[u][0], d, -ai[u][1] * bb);
            pre[u][1] = fma(ai[u][1], a, -ai[u][0] * bb);
        }
        const double rd = rcp_nr(det);
        const double q00 = -d * rd, q01 = bb * rd, q11 = -a * rd;   // q10 = q01
        const bool rowB = (r == j), colB = (c == j);
        double m[2][2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            m[u][0] = rowB ? (u == 0 ? q00 : q01) : pre[u][0] * rd;
            m[u][1] = rowB ? (u == 0 ? q01 : q11) : pre[u][1] * rd;
        }
        const double al[2][2] = {{l0.x, l0.y}, {l1.x, l1.y}};   // al[w][b] = A_(2c+w),(2j+b) = A_Bl[b][w]
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                const double base = rowB ? 0.0 : p[u][w];
                const double upd = fma(-m[u][1], al[w][1], fma(-m[u][0], al[w][0], base));
                p[u][w] = colB ? m[u][w] : upd;
            }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int w = 0; w < 2; ++w) Qn[(2 * r + u) * LDP + 2 * c + w] = p[u][w];
}

// The inverse of the (final) diagonal tile k held in registers t (MFMA layout) -> W_k (global)
// and buf (LDS); then w_k = W_k y_k for the RW right-hand sides (y: LDS [NB][RW] -> R rows of
// tile k) and the panel's intrinsics Schur terms contrib_k[i][j] = sum_r y[r][i] w[r][j] (i < RW-1).
// buf: 64 x LDT doubles of LDS workspace; wv: NB x RW doubles of LDS.  WT: W_k and the R rows are
// stored write-through (sc1), for readers in the same launch (chol_factor).
// The symmetric sweeps of chol_diag_tile over the 16-row panels in `sweep` (ascending); the panels in
// `pad` are identity padding (r06: not swept, set to their result directly); the others are left
// alone (already swept: r06's pre-sweep of the panels an update does not touch, see chol_factor).
// A non-positive pivot sets fail bit 1.
__device__ __forceinline__ void diag_sweeps(f64x4 (&t)[NW], int sweep, int skip_panels, int* __restrict__ fail,
                                            double (*buf)[LDT], double* dws, int trk = CHOL_TRACE_MAX) {
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, m = l & 15, kq = l >> 4;
    double* ws = DIAG_WS_IN_BUF ? &buf[0][0] : dws;   // the sweeps' workspace
    double* Pc = ws;                       // [64][LDP]  column panel A_:B
    double* Qn = ws + NB * LDP;            // [16][LDP]  -A_BB^-1
    double* ipan = Qn + 16 * LDP;          // [16][2]    inner column panel
    double* Mw = ipan + 32 + 16 * LDP * w; // [16][LDP]  this wave's -M strip
    bool bad = false;
#pragma unroll
    for (int s = 0; s < NB / 16; ++s) {
        const bool rowB = (w == s);
        if (!(((sweep | skip_panels) >> s) & 1)) continue;   // swept before (pre-sweep)
        if ((skip_panels >> s) & 1) {
            // r06: a panel of identity padding rows (no coupling, diagonal exactly 1: ba_add_cam) sweeps
            // to A_BB <- -1 on its diagonal and M = 0; the other column tiles are unchanged
#pragma unroll
            for (int r = 0; r < 4; ++r) t[s][r] = (rowB && trow(r) == tcol()) ? -1.0 : 0.0;
            continue;
        }
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
        for (int c = 0; c < NW; ++c) {
            if (c == s) continue;
            f64x4 acc = rowB ? f64x4{0.0, 0.0, 0.0, 0.0} : t[c];
#pragma unroll
            for (int st = 0; st < 4; ++st)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Mw[m * LDP + 4 * st + kq], Pc[(16 * c + m) * LDP + 4 * st + kq], acc, 0, 0, 0);
            t[c] = acc;
        }
        __syncthreads();   // Pc is rewritten by the next sweep
        CHOL_STAMP(5 + 4 * s);
        CHOL_TRACE(trk, 8 + s);
    }
    if (bad) atomicOr(fail, 1);
}

struct NoDefer { __device__ void operator()() const {} };

template <int RW, bool WT = false, class Defer = NoDefer>
__device__ __forceinline__ void chol_diag_tile(f64x4 (&t)[NW], int k, double* __restrict__ Wk,
                                               double* __restrict__ R, const double* __restrict__ y,
                                               double* __restrict__ wv, double* __restrict__ contrib,
                                               int* __restrict__ fail, double (*buf)[LDT], double* dws,
                                               int* wver = nullptr, int skip_panels = 0, int trk = CHOL_TRACE_MAX,
                                               int done_panels = 0, Defer defer = Defer{}) {
    const int tid = threadIdx.x, w = tid >> 6, k0 = k * NB;
    CHOL_STAMP(0);
    CHOL_STAMP(1);
    diag_sweeps(t, ((1 << (NB / 16)) - 1) & ~skip_panels & ~done_panels, skip_panels, fail, buf, dws, trk);
#pragma unroll
    for (int c = 0; c < NW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * w + trow(r), j = 16 * c + tcol();
            buf[i][j] = -t[c][r];
            if (WT) st_wt(&Wk[i * NB + j], -t[c][r]);
            else Wk[i * NB + j] = -t[c][r];
        }
    if (WT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // W_k drained before its version add
    __syncthreads();
    if (wver && tid == 0) __hip_atomic_fetch_add((g_i32*)wver, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // W_k ready
    CHOL_TRACE(trk, 12);
    CHOL_STAMP(20);
    defer();   // (r06: an inverting one-source task's y terms, once W_k is out; they only feed y below)
    {   // w = W y: 4 threads per row i, each over 16 columns c for all RW right-hand sides (16-B LDS
        // reads), the 4 partial sums combined by two shuffles in a fixed order
        static_assert(RW % 2 == 0, "RW is k + 1 with k odd");
        const int i = tid >> 2, cp = tid & 3;
        double acc[RW];
#pragma unroll
        for (int q = 0; q < RW; ++q) acc[q] = 0.0;
#pragma unroll
        for (int cc = 0; cc < NB / 4; cc += 2) {
            const int c = cp * (NB / 4) + cc;
            const double2 wi = *reinterpret_cast<const double2*>(&buf[i][c]);
#pragma unroll
            for (int q = 0; q < RW; q += 2) {
                const double2 y0 = *reinterpret_cast<const double2*>(&y[c * RW + q]);
                const double2 y1 = *reinterpret_cast<const double2*>(&y[(c + 1) * RW + q]);
                acc[q] = fma(wi.x, y0.x, acc[q]);
                acc[q + 1] = fma(wi.x, y0.y, acc[q + 1]);
                acc[q] = fma(wi.y, y1.x, acc[q]);
                acc[q + 1] = fma(wi.y, y1.y, acc[q + 1]);
            }
        }
#pragma unroll
        for (int q = 0; q < RW; ++q) {
            acc[q] += __shfl_xor(acc[q], 1);
            acc[q] += __shfl_xor(acc[q], 2);
        }
        if (cp == 0) {
#pragma unroll
            for (int q = 0; q < RW; ++q) {
                wv[i * RW + q] = acc[q];
                if (WT) st_wt(&R[(size_t)(k0 + i) * RW + q], acc[q]);
                else R[(size_t)(k0 + i) * RW + q] = acc[q];
            }
        }
    }
    CHOL_STAMP(22);
    __syncthreads();
    CHOL_STAMP(23);
    // contrib_k[i][j] = sum_r y[r][i] w[r][j]: 16 lanes per output, 4 rows each, then 4 shuffles
    for (int o = tid >> 4; o < (RW - 1) * RW; o += NTH / 16) {
        const int i = o / RW, j = o % RW, rp = tid & 15;
        double sacc = 0.0;
#pragma unroll
        for (int h = 0; h < NB / 16; ++h) sacc = fma(y[(rp + 16 * h) * RW + i], wv[(rp + 16 * h) * RW + j], sacc);
        sacc += __shfl_xor(sacc, 1);
        sacc += __shfl_xor(sacc, 2);
        sacc += __shfl_xor(sacc, 4);
        sacc += __shfl_xor(sacc, 8);
        if (rp == 0) contrib[(size_t)k * (RW - 1) * RW + o] = sacc;
    }
    CHOL_STAMP(21);
}

template <int RW>
struct alignas(16) CholLds {
    double a[NB][LDT], m[NB][LDT], n[NB][LDT];
    double rk[NB * RW], ra[NB * RW], wv[NB * RW];   // w_k of a source panel; y_a; w_a
    double dws[DIAG_WS_IN_BUF ? 2 : DIAG_WS];        // chol_diag_tile's workspace when a tile buffer is too small
};

// launch 0: the diagonal tiles of the level-0 panels (untouched by any update) -> W_k, w_k, contrib_k
template <int RW>
__global__ __launch_bounds__(NTH)
void chol_leaves(double* __restrict__ S, int npad, double* __restrict__ R, const int* __restrict__ leaves,
                 double* __restrict__ W, double* __restrict__ contrib, int* __restrict__ fail) {
    if (step_gated(fail + 1)) return;
    __shared__ CholLds<RW> sm;
    const int k = leaves[blockIdx.x], k0 = k * NB;
    f64x4 t[NW];
    tile_regs(t, S + (size_t)k0 * npad + k0, npad);
    for (int e = threadIdx.x; e < NB * RW; e += NTH) sm.ra[e] = R[(size_t)k0 * RW + e];
    __syncthreads();
    chol_diag_tile<RW>(t, k, W + (size_t)k * NB * NB, R, sm.ra, sm.wv, contrib, fail, sm.a, sm.dws);
}

// launch l + 1: one workgroup per destination tile (a, b) of level l's updates, its source panels
// k = src[s0 .. s1) in ascending order:
//   G = A_ak W_k;  A_ab -= G A_bk^T  (b == a: A_aa -= G A_ak^T, G^T -> upper tile (k, a), y_a -= A_ak w_k)
// The first ninv workgroups hold diagonal tiles whose last update this is: they invert it.
template <int RW>
__global__ __launch_bounds__(NTH)
void chol_level(double* __restrict__ S, int npad, double* __restrict__ R, const int4* __restrict__ tasks,
                const int* __restrict__ src, int ninv, double* __restrict__ W, double* __restrict__ contrib,
                int* __restrict__ fail, const int* __restrict__ tpre) {
    if (step_gated(fail + 1)) return;
    __shared__ CholLds<RW> sm;
    const int tid = threadIdx.x, w = tid >> 6;
    const int4 task = tasks[blockIdx.x];
    const int a = task.x, b = task.y, a0 = a * NB, b0 = b * NB;
    const bool diag = (a == b);
    CHOL_STAMP(30);
    f64x4 t[NW];
    double* dst = S + (size_t)a0 * npad + b0;
    tile_regs(t, dst, npad);                                                   // A_ab (prefetch)
    if (diag)
        for (int e = tid; e < NB * RW; e += NTH) sm.ra[e] = R[(size_t)a0 * RW + e];
    // r06: an inverting one-source task sweeps the panels its update does not touch first (tpre,
    // ba_plan.cpp row_masks), as chol_factor does while it waits for W_k: the same bits in every form
    const int pre = (diag && (int)blockIdx.x < ninv && task.w - task.z == 1) ? tpre[blockIdx.x] : 0;
    if (pre) diag_sweeps(t, pre, 0, fail, sm.n, sm.dws);
    for (int s = task.z; s < task.w; ++s) {
        const int k = src[s], k0 = k * NB;
        tile_load(sm.a, S + (size_t)a0 * npad + k0, npad);                     // A_ak
        tile_load(sm.m, W + (size_t)k * NB * NB, NB);                          // W_k
        if (!diag) tile_load(sm.n, S + (size_t)b0 * npad + k0, npad);          // A_bk
        else
            for (int e = tid; e < NB * RW; e += NTH) sm.rk[e] = R[(size_t)k0 * RW + e];   // w_k
        __syncthreads();
        CHOL_STAMP(31);
        f64x4 g[NW];
        mfma_nn(sm.a, sm.m, g);   // G = A_ak W_k
        __syncthreads();
        CHOL_STAMP(32);
#pragma unroll
        for (int c = 0; c < NW; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) sm.m[16 * w + trow(r)][16 * c + tcol()] = g[c][r];
        __syncthreads();
        f64x4 upd[NW];
        mfma_nt(sm.m, diag ? sm.a : sm.n, upd);   // G X^T
#pragma unroll
        for (int c = 0; c < NW; ++c) t[c] -= upd[c];
        CHOL_STAMP(33);
        if (diag) {
            // y_a -= A_ak w_k: NB x RW outputs, 256 / RW ... threads; 4 lanes per output for RW <= 4
            constexpr int TPO = (NTH / (NB * RW)) > 0 ? NTH / (NB * RW) : 1;
            constexpr int OPT = (NB * RW) / (NTH / TPO);
            const int part = tid % TPO;
#pragma unroll
            for (int u = 0; u < OPT; ++u) {
                const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                double sum = 0.0;
                for (int c = part; c < NB; c += TPO) sum = fma(sm.a[i][c], sm.rk[c * RW + q], sum);
                if (TPO >= 2) sum += __shfl_xor(sum, 1);
                if (TPO >= 4) sum += __shfl_xor(sum, 2);
                if (part == 0) sm.ra[i * RW + q] -= sum;
            }
            // upper tile (k, a): row k0 + j, column a0 + i holds G[i][j]
#pragma unroll
            for (int c = 0; c < NW; ++c)
#pragma unroll
                for (int r = 0; r < 4; ++r) S[(size_t)(k0 + 16 * c + tcol()) * npad + a0 + 16 * w + trow(r)] = g[c][r];
        }
        __syncthreads();   // the next source panel overwrites sm
    }
    if (diag && (int)blockIdx.x < ninv) {
        chol_diag_tile<RW>(t, a, W + (size_t)a * NB * NB, R, sm.ra, sm.wv, contrib, fail, sm.n, sm.dws, nullptr, 0,
                           CHOL_TRACE_MAX, pre);
    } else {
        tile_store(t, dst, npad);
        if (diag)
            for (int e = tid; e < NB * RW; e += NTH) R[(size_t)a0 * RW + e] = sm.ra[e];
    }
    CHOL_STAMP(34);
}

// chol_level with the sources of a destination tile split over workgroups (SFMX_BA_SPLIT, default
// on): one workgroup per (task, source) "part".  A task with one source runs as in chol_level.  A
// task with n > 1 sources: every part computes its product U_k = G A_bk^T (diag: also its y term
// A_ak w_k and the upper tile G^T) from zero, exactly as chol_level's loop body does, writes U_k
// (+ y term) write-through (sc1) into its slot of pbuf, drains, and adds to the task's arrival
// counter; the part whose add returns n - 1 (the last) loads A_ab and subtracts the n products in
// source order (its own from registers, the others by sc1 loads behind its add: no acquire needed,
// MI355X_MICROARCH.md inter-workgroup visibility, valid sc1-load form row 1), then inverts or
// stores as chol_level does.  Same operations in the same order as chol_level: bit-identical.
// The critical path of a level falls from n source steps + inverse to one source step + the
// hand-off + inverse.  part = {task (global index), source index, slot, n | inverting << 16};
// ctr[task] is zero at launch and the last part zeroes it again.
// r06: only the product tiles a part's row masks allow (strip w in ra, column tile c in rb; the rest
// are exact zeros): a quarter of the stores on the C5 ring, and the finisher loads the same subset
template <int RW>
__device__ __forceinline__ void part_store_m(double* __restrict__ slot, const f64x4 (&u)[NW], const double* ys, int nys,
                                             int ra, int rb) {
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((ra >> w) & 1)
#pragma unroll
        for (int c = 0; c < NW; ++c)
            if ((rb >> c) & 1)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    __hip_atomic_store((g_u64*)&slot[(4 * c + r) * NTH + tid], (unsigned long long)__double_as_longlong(u[c][r]),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int u2 = 0; u2 < nys; ++u2)
        __hip_atomic_store((g_u64*)&slot[(4 * NW + u2) * NTH + tid], (unsigned long long)__double_as_longlong(ys[u2]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int RW>
__device__ __forceinline__ void part_store(double* __restrict__ slot, const f64x4 (&u)[NW], const double* ys, int nys) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int c = 0; c < NW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            __hip_atomic_store((g_u64*)&slot[(4 * c + r) * NTH + tid], (unsigned long long)__double_as_longlong(u[c][r]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int u2 = 0; u2 < nys; ++u2)
        __hip_atomic_store((g_u64*)&slot[(4 * NW + u2) * NTH + tid], (unsigned long long)__double_as_longlong(ys[u2]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int RW>
__global__ __launch_bounds__(NTH)
void chol_level_split(double* __restrict__ S, int npad, double* __restrict__ R, const int4* __restrict__ tasks,
                      const int4* __restrict__ parts, const int* __restrict__ src, double* __restrict__ W,
                      double* __restrict__ contrib, int* __restrict__ fail, double* pbuf, int* ctr,
                      const int* __restrict__ tpre) {
    if (step_gated(fail + 1)) return;
    __shared__ CholLds<RW> sm;
    __shared__ int last_sh;
    constexpr int TPO = (NTH / (NB * RW)) > 0 ? NTH / (NB * RW) : 1;
    constexpr int OPT = (NB * RW) / (NTH / TPO);
    constexpr int SLOT = (4 * NW + OPT) * NTH;   // doubles per part slot
    const int tid = threadIdx.x, w = tid >> 6;
    const int4 part = parts[blockIdx.x];
    const int4 task = tasks[part.x];
    const int a = task.x, b = task.y, a0 = a * NB, b0 = b * NB, n = part.w & 0xffff, j = part.y - task.z;
    const bool diag = (a == b), inv = (part.w >> 16) != 0;
    const int k = src[part.y], k0 = k * NB;
    double* dst = S + (size_t)a0 * npad + b0;
    f64x4 t[NW];
    const int pre = (n == 1 && diag && inv) ? tpre[part.x] : 0;   // (r06, as chol_level)
    if (n == 1) {
        tile_regs(t, dst, npad);                                                   // A_ab (prefetch)
        if (diag)
            for (int e = tid; e < NB * RW; e += NTH) sm.ra[e] = R[(size_t)a0 * RW + e];
        if (pre) diag_sweeps(t, pre, 0, fail, sm.n, sm.dws);
    }
    tile_load(sm.a, S + (size_t)a0 * npad + k0, npad);                         // A_ak
    tile_load(sm.m, W + (size_t)k * NB * NB, NB);                              // W_k
    if (!diag) tile_load(sm.n, S + (size_t)b0 * npad + k0, npad);              // A_bk
    else
        for (int e = tid; e < NB * RW; e += NTH) sm.rk[e] = R[(size_t)k0 * RW + e];   // w_k
    __syncthreads();
    f64x4 g[NW];
    mfma_nn(sm.a, sm.m, g);   // G = A_ak W_k
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.m[16 * w + trow(r)][16 * c + tcol()] = g[c][r];
    __syncthreads();
    f64x4 upd[NW];
    mfma_nt(sm.m, diag ? sm.a : sm.n, upd);   // G X^T
    double ys[OPT];
    if (diag) {
        const int pp = tid % TPO;
#pragma unroll
        for (int u = 0; u < OPT; ++u) {
            const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
            double sum = 0.0;
            for (int c = pp; c < NB; c += TPO) sum = fma(sm.a[i][c], sm.rk[c * RW + q], sum);
            if (TPO >= 2) sum += __shfl_xor(sum, 1);
            if (TPO >= 4) sum += __shfl_xor(sum, 2);
            ys[u] = sum;
        }
#pragma unroll
        for (int c = 0; c < NW; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) S[(size_t)(k0 + 16 * c + tcol()) * npad + a0 + 16 * w + trow(r)] = g[c][r];
    }
    if (n > 1) {   // publish this part; the last arriver finishes the task
        part_store<RW>(pbuf + (size_t)part.z * SLOT, upd, ys, diag ? OPT : 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
            last_sh = __hip_atomic_fetch_add((g_i32*)&ctr[part.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1;
        __syncthreads();
        if (!last_sh) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the slot loads below
        if (tid == 0) ctr[part.x] = 0;                              // nobody else touches it in this launch
        tile_regs(t, dst, npad);
        if (diag)
            for (int e = tid; e < NB * RW; e += NTH) sm.ra[e] = R[(size_t)a0 * RW + e];
        __syncthreads();
        const double* base = pbuf + (size_t)(part.z - j) * SLOT;   // slot of source 0 of this task
        for (int jj = 0; jj < n; ++jj) {
            const double* sl = base + (size_t)jj * SLOT;
#pragma unroll
            for (int c = 0; c < NW; ++c)
#pragma unroll
                for (int r = 0; r < 4; ++r) t[c][r] -= (jj == j) ? upd[c][r] : ld_wt(&sl[(4 * c + r) * NTH + tid]);
            if (diag) {
#pragma unroll
                for (int u = 0; u < OPT; ++u) {
                    const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                    const double y = (jj == j) ? ys[u] : ld_wt(&sl[(4 * NW + u) * NTH + tid]);
                    if (tid % TPO == 0) sm.ra[i * RW + q] -= y;
                }
            }
        }
    } else {
#pragma unroll
        for (int c = 0; c < NW; ++c) t[c] -= upd[c];
        if (diag) {
#pragma unroll
            for (int u = 0; u < OPT; ++u) {
                const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                if (tid % TPO == 0) sm.ra[i * RW + q] -= ys[u];
            }
        }
    }
    __syncthreads();
    if (diag && inv) {
        chol_diag_tile<RW>(t, a, W + (size_t)a * NB * NB, R, sm.ra, sm.wv, contrib, fail, sm.n, sm.dws, nullptr, 0,
                           CHOL_TRACE_MAX, pre);
    } else {
        tile_store(t, dst, npad);
        if (diag)
            for (int e = tid; e < NB * RW; e += NTH) R[(size_t)a0 * RW + e] = sm.ra[e];
    }
}

// The whole factorization in ONE launch (SFMX_BA_DAG, default on): the leaves and every level's
// parts of chol_level_split, with in-launch hand-offs instead of launch boundaries.  A workgroup
// takes a ticket (atomic counter) and the item at that ticket; items are listed leaves first, then
// level by level, so everything an item waits for holds an earlier ticket and is running or done
// (no residency or dispatch-order assumption).  Every lower tile (a, b) has a version word
// tver[a (a + 1) / 2 + b] = the number of its tasks (leaf inverse included) that have finished.
// An inverse adds 2 to its diagonal tile's version: once W_k is stored, and at its end (the R rows
// of k, contrib).  A part waits (one lane, sc1 polls, bounded) until A_ak and A_bk carry their final
// versions (and, for a one-source task, A_ab the version before this task) and loads them, then
// until W_k is stored, and -- a diagonal part, after its tile product -- until the R rows of k are;
// the last arriver of a multi-source task waits for A_ab's version before this task.  The arithmetic
// is chol_level_split's body.  Every
// byte another item reads in this launch (lower tiles, W_k, R rows) is stored write-through (sc1)
// and loaded only with sc1 loads; the storing workgroup drains (vmcnt(0)), meets at a barrier and
// one lane adds to the tile's version (MI355X_MICROARCH.md, inter-workgroup visibility, sc1 form
// row 1).  The upper tiles (k, a) and contrib are read only by chol_backsolve (the next launch).
// items[i] = {task | leaf panel, source index (-1: leaf), slot, n | inverting << 16};
// need[i] = {version of A_ak, of A_bk, of (k, k) (final; W_k stored at one less), of A_ab before this task}.
// ctr = [ticket, finished, tver[T (T + 1) / 2]], zero at launch; the last workgroup re-zeroes it.
// Same operations in the same order as the level launches: bit-identical.
__device__ __forceinline__ int tver_id(int a, int b) { return a * (a + 1) / 2 + b; }



template <int RW>
__global__ __launch_bounds__(NTH)
void chol_factor(double* __restrict__ S, int npad, double* __restrict__ R, const int4* __restrict__ tasks,
                 const int4* __restrict__ items, const int4* __restrict__ need, const int* __restrict__ src,
                 double* __restrict__ W, double* __restrict__ contrib, int* __restrict__ fail, double* pbuf,
                 int* tctr, int* ctr, int nitems, int nver, long long tmo, const int4* __restrict__ imask) {
    if (step_gated(fail + 1)) return;
    __shared__ CholLds<RW> sm;
    __shared__ int sh[2];
    constexpr int TPO = (NTH / (NB * RW)) > 0 ? NTH / (NB * RW) : 1;
    constexpr int OPT = (NB * RW) / (NTH / TPO);
    constexpr int SLOT = (4 * NW + OPT) * NTH;
    const int tid = threadIdx.x, w = tid >> 6;
    int* tver = ctr + 2;
    if (tid == 0) sh[0] = __hip_atomic_fetch_add((g_i32*)ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int tk = sh[0];
    const int4 it = items[tk], nd = need[tk];
    // r06 row masks (ba_plan.cpp row_masks): x = ra | rb << 4 | G's column tiles << 8 | the inverted
    // tile's padding panels << 12, y = ka, z = kb (wave-uniform)
    const int4 mk0 = imask[tk];
    const int mx = __builtin_amdgcn_readfirstlane(mk0.x), mka = __builtin_amdgcn_readfirstlane(mk0.y),
              mkb = __builtin_amdgcn_readfirstlane(mk0.z);
    const int m_ra = mx & 15, m_rb = (mx >> 4) & 15, m_gc = (mx >> 8) & 15, m_pad = (mx >> 12) & 15,
              m_pre = (mx >> 16) & 15;   // pre: an inverting one-source task's panels its update leaves alone
    CHOL_TRACE(tk, 0);
#ifdef SFMX_DIAG
    if (tid == 0 && tk < CHOL_TRACE_MAX) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_chol_trace[tk][15] = ((long long)xcc << 32) | hw;
        for (int q = 1; q < 15; ++q) g_chol_trace[tk][q] = 0;
    }
#endif
    // one lane waits until tile `id` carries version `v` (bounded: `tmo` ticks without the version
    // moving set fail bit 2 and the item runs on, so every counter still advances and the launch drains)
    auto wait_at = [&](int* word, int v) {
        long long t0 = wall_clock64();
        int last = -1;
        for (;;) {
            const int cur = __hip_atomic_load((g_i32*)word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur >= v) return;
            if (cur != last) { last = cur; t0 = wall_clock64(); }   // progress restarts the clock
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > tmo) { atomicOr(fail, FAIL_FACTOR_WAIT); return; }
        }
    };
    auto wait_ver = [&](int id, int v) { wait_at(&tver[id], v); };
    const __amdgpu_buffer_rsrc_t rS = wt_rsrc(S), rW = wt_rsrc(W);
    int done_id = -1;   // the tile whose version this item advances (-1: none)
    int upper_k0 = -1, upper_a0 = 0;   // a diagonal part's upper tile G^T, stored after the version add
    if (it.y < 0) {     // leaf: diagonal tile k, untouched by any update
        const int k = it.x, k0 = k * NB;
        f64x4 t[NW];
        tile_regs(t, S + (size_t)k0 * npad + k0, npad);
        for (int e = tid; e < NB * RW; e += NTH) sm.ra[e] = R[(size_t)k0 * RW + e];
        __syncthreads();
        CHOL_TRACE(tk, 7);
        chol_diag_tile<RW, true>(t, k, W + (size_t)k * NB * NB, R, sm.ra, sm.wv, contrib, fail, sm.a, sm.dws, &tver[tver_id(k, k)],
                                 m_pad, tk);
        done_id = tver_id(k, k);
    } else {
        const int4 task = tasks[it.x];
        const int a = task.x, b = task.y, a0 = a * NB, b0 = b * NB, n = it.w & 0xffff, j = it.y - task.z;
        const bool diag = (a == b), inv = (it.w >> 16) != 0;
        const int k = src[it.y], k0 = k * NB;
        double* dst = S + (size_t)a0 * npad + b0;
        // A_ak, A_bk (and A_ab of a one-source task) are final before W_k is (the inverse of (k, k) ends
        // the previous level's chain): they load while that inverse still runs
        if (tid == 0) {
            wait_ver(tver_id(a, k), nd.x);
            if (!diag) wait_ver(tver_id(b, k), nd.y);
            if (n == 1) wait_ver(tver_id(a, b), nd.w);
        }
        __syncthreads();
        CHOL_TRACE(tk, 1);
        f64x4 t[NW];
        // the destination (final but for this task) loads now in a one-source task and, r06, in every
        // part of an inverting multi-source task (the finisher then starts its subtraction at once)
        const bool early_dst = n == 1 || (diag && inv);
        if (n > 1 && early_dst && tid == 0) wait_ver(tver_id(a, b), nd.w);
        if (n > 1 && early_dst) __syncthreads();
        if (early_dst) {
            tile_regs_wt(t, dst, npad);
            if (diag)
                for (int e = tid; e < NB * RW; e += NTH) sm.ra[e] = ld_wt(&R[(size_t)a0 * RW + e]);
        }
        tile_load_wt(sm.a, rS, (size_t)a0 * npad + k0, npad);                   // A_ak
        if (!diag) tile_load_wt(sm.n, rS, (size_t)b0 * npad + k0, npad);        // A_bk
        // r06: the update A_aa -= G A_ak^T touches only A_ak's row strips; the other panels of the
        // (final-but-this-update) diagonal tile are swept now, while W_k is still being computed
        // (sweeping commutes with adding to the unswept block: the same inverse, other rounding)
        if (m_pre) diag_sweeps(t, m_pre, 0, fail, sm.n, sm.dws, tk);
        if (tid == 0) wait_ver(tver_id(k, k), nd.z - 1);   // W_k stored (its R rows may still be in flight)
        __syncthreads();
        CHOL_TRACE(tk, 2);
        tile_load_wt_rows(sm.m, rW, (size_t)k * NB * NB, NB, mka);             // W_k (the rows G reads)
        __syncthreads();
        CHOL_TRACE(tk, 3);
        f64x4 upd[NW];
        {   // r06: G = A_ak W_k and U = G X^T on their structurally nonzero tiles, spread over the waves
            f64x4 sp[4];
            int ts[4], tc[4];
            const int n1 = mfma_spread<false>(sm.a, sm.m, sp, m_ra, m_gc, mka, ts, tc);   // G
            __syncthreads();
            CHOL_TRACE(tk, 4);
            spread_store(sm.m, sp, ts, tc, n1, m_ra, m_gc);   // G (zero strips included: G^T is stored whole)
            __syncthreads();
            const int n2 = mfma_spread<true>(sm.m, diag ? sm.a : sm.n, sp, m_ra, m_rb, mkb, ts, tc);   // G X^T
            __syncthreads();   // (X = A_bk in sm.n is read; sm.n takes U)
            spread_store(sm.n, sp, ts, tc, n2, m_ra, m_rb);
            __syncthreads();
#pragma unroll
            for (int c = 0; c < NW; ++c)   // back to the strip-owned layout of t
#pragma unroll
                for (int r = 0; r < 4; ++r) upd[c][r] = sm.n[16 * w + trow(r)][16 * c + tcol()];
        }
        CHOL_TRACE(tk, 5);
        double ys[OPT];
        // y_a terms of a diagonal part: ys = A_ak w_k (w_k = the R rows of k, stored after W_k)
        auto y_terms = [&]() {
            if (tid == 0) wait_ver(tver_id(k, k), nd.z);   // w_k (the R rows of k) stored
            __syncthreads();
            for (int e = tid; e < NB * RW; e += NTH) sm.rk[e] = ld_wt(&R[(size_t)k0 * RW + e]);   // w_k
            __syncthreads();
            const int pp = tid % TPO;
#pragma unroll
            for (int u = 0; u < OPT; ++u) {
                const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                double sum = 0.0;
                for (int c = pp; c < NB; c += TPO) sum = fma(sm.a[i][c], sm.rk[c * RW + q], sum);
                if (TPO >= 2) sum += __shfl_xor(sum, 1);
                if (TPO >= 4) sum += __shfl_xor(sum, 2);
                ys[u] = sum;
            }
        };
        // r06: an inverting diagonal task takes its y terms after W_a is out (they feed only the inverse's
        // right-hand-side phase), its parts publish their products first and their y terms second, and
        // every diagonal part stores the upper tile G^T (read by the next launch only) after its version
        // add: none of it is on the level chain any more
        const bool defer_y = diag && inv;
        if (diag && !defer_y) y_terms();
        bool fin = true;
        int* const stored1 = tctr + nitems;       // per task: non-finishing parts whose product is stored
        int* const stored2 = tctr + 2 * nitems;   // ... and whose y terms are (inverting diagonal tasks)
        if (n > 1) {
            // arrive first, publish only if not last: the arrival add picks the finisher, whose own
            // product never leaves its registers (r05 stored and drained it before knowing)
            if (tid == 0)
                sh[1] = __hip_atomic_fetch_add((g_i32*)&tctr[it.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1;
            __syncthreads();
            fin = sh[1] != 0;
            double* const slot = pbuf + (size_t)it.z * SLOT;
            if (!fin) {
                part_store_m<RW>(slot, upd, ys, diag && !defer_y ? OPT : 0, m_ra, m_rb);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) __hip_atomic_fetch_add((g_i32*)&stored1[it.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (defer_y) {   // the y terms, then their count
                    y_terms();
                    for (int u2 = 0; u2 < OPT; ++u2)
                        __hip_atomic_store((g_u64*)&slot[(4 * NW + u2) * NTH + tid], (unsigned long long)__double_as_longlong(ys[u2]),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                    if (tid == 0) __hip_atomic_fetch_add((g_i32*)&stored2[it.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                if (tid == 0) {
                    wait_at(&stored1[it.x], n - 1);   // every other part's product stored
                    tctr[it.x] = 0;                   // nobody else touches them in this launch
                    stored1[it.x] = 0;
                    if (!early_dst) wait_ver(tver_id(a, b), nd.w);
                }
                __syncthreads();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the loads below
                if (!early_dst) {
                    tile_regs_wt(t, dst, npad);
                    if (diag)
                        for (int e = tid; e < NB * RW; e += NTH) sm.ra[e] = ld_wt(&R[(size_t)a0 * RW + e]);
                }
                __syncthreads();
                const double* base = pbuf + (size_t)(it.z - j) * SLOT;   // slot of source 0 of this task
                const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
                for (int jj = 0; jj < n; ++jj) {
                    const double* sl = base + (size_t)jj * SLOT;
                    // the part's row masks (its item is tk - j + jj): the tiles it stored; the rest are zeros
                    const int pm = jj == j ? mx : __builtin_amdgcn_readfirstlane(imask[tk - j + jj].x);
                    const int pra = pm & 15, prb = (pm >> 4) & 15;
                    if ((pra >> wv) & 1)
#pragma unroll
                        for (int c = 0; c < NW; ++c)
                            if ((prb >> c) & 1)
#pragma unroll
                                for (int r = 0; r < 4; ++r) t[c][r] -= (jj == j) ? upd[c][r] : ld_wt(&sl[(4 * c + r) * NTH + tid]);
                    if (diag && !defer_y) {
#pragma unroll
                        for (int u = 0; u < OPT; ++u) {
                            const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                            const double y = (jj == j) ? ys[u] : ld_wt(&sl[(4 * NW + u) * NTH + tid]);
                            if (tid % TPO == 0) sm.ra[i * RW + q] -= y;
                        }
                    }
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < NW; ++c) t[c] -= upd[c];
            if (diag && !defer_y) {
#pragma unroll
                for (int u = 0; u < OPT; ++u) {
                    const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                    if (tid % TPO == 0) sm.ra[i * RW + q] -= ys[u];
                }
            }
        }
        CHOL_TRACE(tk, 6);
        if (fin) {
            __syncthreads();
            if (defer_y) {
                CHOL_TRACE(tk, 7);
                // the y terms in source order (the immediate path's arithmetic and order), once W_a is out
                auto later = [&]() {
                    y_terms();
                    if (n > 1 && tid == 0) {
                        wait_at(&stored2[it.x], n - 1);   // every other part's y terms stored
                        stored2[it.x] = 0;
                    }
                    __syncthreads();
                    const double* base = pbuf + (size_t)(it.z - j) * SLOT;
                    for (int jj = 0; jj < n; ++jj) {
                        const double* sl = base + (size_t)jj * SLOT;
#pragma unroll
                        for (int u = 0; u < OPT; ++u) {
                            const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                            const double y = (jj == j) ? ys[u] : ld_wt(&sl[(4 * NW + u) * NTH + tid]);
                            if (tid % TPO == 0) sm.ra[i * RW + q] -= y;
                        }
                    }
                    __syncthreads();
                };
                chol_diag_tile<RW, true>(t, a, W + (size_t)a * NB * NB, R, sm.ra, sm.wv, contrib, fail, sm.n, sm.dws,
                                         &tver[tver_id(a, a)], m_pad, tk, m_pre, later);
            } else {
                tile_store_wt(t, dst, npad);
                if (diag)
                    for (int e = tid; e < NB * RW; e += NTH) st_wt(&R[(size_t)a0 * RW + e], sm.ra[e]);
            }
            done_id = tver_id(a, b);
        }
        upper_k0 = diag ? k0 : -1;
        upper_a0 = a0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains before the version add
    __syncthreads();
    CHOL_TRACE(tk, 13);
    if (tid == 0) {
        if (done_id >= 0) __hip_atomic_fetch_add((g_i32*)&tver[done_id], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add((g_i32*)&ctr[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nitems - 1)
            for (int e = 0; e < nver + 2; ++e) __hip_atomic_store((g_i32*)&ctr[e], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (upper_k0 >= 0)   // a diagonal part: upper tile (k, a) = G^T (row k0 + j, column a0 + i holds G[i][j]), from sm.m
#pragma unroll
        for (int c = 0; c < NW; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                S[(size_t)(upper_k0 + 16 * c + tcol()) * npad + upper_a0 + 16 * w + trow(r)] = sm.m[16 * w + trow(r)][16 * c + tcol()];
}

// ---------------------------------------------------------------------------------------------
// chol_factor on NW x NW waves (SFMX_BA_WIDE=1, diagnostic build: measured no faster, ba_solver.hip ensure_plan).  The NW-wave form
// above gives each wave a 16-row strip of NW column tiles, so a 64^3 tile product is NW x 16 MFMA
// steps per wave and a 64 x 64 tile load NB^2 / (2 NTH) 16-B loads per thread: on the level chain
// (r02q stamps: loads 2.7 us, the two products 2.9 + 3.4 us per level) every workgroup of the launch
// waits on one CU's worth of issue.  Here wave w owns the single 16 x 16 tile (wr, wc) = (w % NW,
// w / NW): the products are 16 MFMA steps per wave, the loads a quarter as many per thread.  Every
// output element is accumulated by the same MFMA sequence as in mfma_nn / mfma_nt (k ascending), the
// diagonal inverse runs the same sweeps (the inner 16 x 16 inverse on wave 0, M per strip, the rank-16
// update per tile) and the right-hand-side terms (y_a, w = W y, contrib) run on the first NTH threads
// with NTH's partition: bit-identical to chol_factor and to the per-level launches.
constexpr int NWW = NW * NW, NTW = 64 * NWW;   // waves / threads of the wide form
__device__ __forceinline__ int wrow() { return (threadIdx.x >> 6) % NW; }
__device__ __forceinline__ int wcol() { return (threadIdx.x >> 6) / NW; }
__device__ __forceinline__ void tile_load_w(double (*dst)[LDT], const double* __restrict__ src, int ld) {
#pragma unroll
    for (int q = 0; q < NB * NB / (2 * NTW); ++q) {
        const int e = q * (2 * NTW) + 2 * threadIdx.x;
        *reinterpret_cast<double2*>(&dst[e / NB][e % NB]) = *reinterpret_cast<const double2*>(src + (size_t)(e / NB) * ld + e % NB);
    }
}
__device__ __forceinline__ void tile_load_w_wt(double (*dst)[LDT], __amdgpu_buffer_rsrc_t rs, size_t src, int ld) {
#pragma unroll
    for (int q = 0; q < NB * NB / (2 * NTW); ++q) {
        const int e = q * (2 * NTW) + 2 * threadIdx.x;
        *reinterpret_cast<double2*>(&dst[e / NB][e % NB]) = ld_wt2(rs, src + (size_t)(e / NB) * ld + e % NB);
    }
}
// this wave's tile (wr, wc) of a row-major NB x NB block at src (leading dimension ld)
__device__ __forceinline__ size_t wtile_at(int r, int ld) {
    return (size_t)(16 * wrow() + trow(r)) * ld + 16 * wcol() + tcol();
}
__device__ __forceinline__ void wtile_regs(f64x4& t, const double* __restrict__ src, int ld) {
#pragma unroll
    for (int r = 0; r < 4; ++r) t[r] = src[wtile_at(r, ld)];
}
__device__ __forceinline__ void wtile_regs_wt(f64x4& t, const double* __restrict__ src, int ld) {
#pragma unroll
    for (int r = 0; r < 4; ++r) t[r] = ld_wt(&src[wtile_at(r, ld)]);
}
__device__ __forceinline__ void wtile_store_wt(const f64x4& t, double* __restrict__ dst, int ld) {
#pragma unroll
    for (int r = 0; r < 4; ++r) st_wt(&dst[wtile_at(r, ld)], t[r]);
}
// acc = A[strip wr] * B[:, tile wc]   (= mfma_nn's acc[wc] of wave wr)
__device__ __forceinline__ f64x4 wmfma_nn(const double (*A)[LDT], const double (*B)[LDT]) {
    const int wr = wrow(), wc = wcol(), l = threadIdx.x & 63, m = l & 15, kq = l >> 4;
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int st = 0; st < NB / 4; ++st)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[16 * wr + m][4 * st + kq], B[4 * st + kq][16 * wc + m], acc, 0, 0, 0);
    return acc;
}
// acc = A[strip wr] * X[tile wc rows]^T   (= mfma_nt's acc[wc] of wave wr)
__device__ __forceinline__ f64x4 wmfma_nt(const double (*A)[LDT], const double (*X)[LDT]) {
    const int wr = wrow(), wc = wcol(), l = threadIdx.x & 63, m = l & 15, kq = l >> 4;
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int st = 0; st < NB / 4; ++st)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[16 * wr + m][4 * st + kq], X[16 * wc + m][4 * st + kq], acc, 0, 0, 0);
    return acc;
}
// chol_diag_tile on the NW x NW waves: t is this wave's tile (wr, wc) of the final diagonal tile k.
// ws: the sweeps' workspace, DIAG_WS_W doubles (two tile buffers: sm.m | sm.n, dead by now); buf: a
// tile buffer for W (the first of them: the sweeps are over when W is written into it).
constexpr int DIAG_WS_W = NB * LDP + 16 * LDP + 32 + NWW * 16 * LDP;
static_assert(DIAG_WS_W <= 2 * NB * LDT, "the wide sweeps' workspace spans two tile buffers");
template <int RW>
__device__ __forceinline__ void chol_diag_tile_w(f64x4& t, int k, double* __restrict__ Wk, double* __restrict__ R,
                                                 const double* __restrict__ y, double* __restrict__ wv,
                                                 double* __restrict__ contrib, int* __restrict__ fail,
                                                 double (*buf)[LDT], double* ws, int* wver) {
    const int tid = threadIdx.x, w = tid >> 6, wr = wrow(), wc = wcol(), l = tid & 63, m = l & 15, kq = l >> 4, k0 = k * NB;
    double* Pc = ws;                       // [64][LDP]  column panel A_:B
    double* Qn = ws + NB * LDP;            // [16][LDP]  -A_BB^-1
    double* ipan = Qn + 16 * LDP;          // [16][2]    inner column panel
    double* Mw = ipan + 32 + 16 * LDP * w; // [16][LDP]  this wave's -M strip (strip wr)
    bool bad = false;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const bool rowB = (wr == s);
        if (wc == s)
#pragma unroll
            for (int r = 0; r < 4; ++r) Pc[(16 * wr + trow(r)) * LDP + tcol()] = t[r];
        __syncthreads();
        if (tid < 64) inner_inverse16(Pc, s, Qn, ipan, bad);
        __syncthreads();
        f64x4 mm = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 4; ++st)
            mm = __builtin_amdgcn_mfma_f64_16x16x4f64(Pc[(16 * wr + m) * LDP + 4 * st + kq], Qn[(4 * st + kq) * LDP + m], mm, 0, 0, 0);
        f64x4 mv;
#pragma unroll
        for (int r = 0; r < 4; ++r) mv[r] = rowB ? Qn[trow(r) * LDP + tcol()] : -mm[r];
        if (wc == s) {
            t = mv;
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) Mw[trow(r) * LDP + tcol()] = -mv[r];
            __builtin_amdgcn_wave_barrier();
            f64x4 acc = rowB ? f64x4{0.0, 0.0, 0.0, 0.0} : t;
#pragma unroll
            for (int st = 0; st < 4; ++st)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Mw[m * LDP + 4 * st + kq], Pc[(16 * wc + m) * LDP + 4 * st + kq], acc, 0, 0, 0);
            t = acc;
        }
        __syncthreads();   // Pc is rewritten by the next sweep
    }
    if (bad) atomicOr(fail, 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 16 * wr + trow(r), j = 16 * wc + tcol();
        buf[i][j] = -t[r];
        st_wt(&Wk[i * NB + j], -t[r]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // W_k drained before its version add
    __syncthreads();
    if (wver && tid == 0) __hip_atomic_fetch_add((g_i32*)wver, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // W_k ready
    if (tid < NTH) {   // w = W y: chol_diag_tile's partition and order
        static_assert(RW % 2 == 0, "RW is k + 1 with k odd");
        const int i = tid >> 2, cp = tid & 3;
        double acc[RW];
#pragma unroll
        for (int q = 0; q < RW; ++q) acc[q] = 0.0;
#pragma unroll
        for (int cc = 0; cc < NB / 4; cc += 2) {
            const int c = cp * (NB / 4) + cc;
            const double2 wi = *reinterpret_cast<const double2*>(&buf[i][c]);
#pragma unroll
            for (int q = 0; q < RW; q += 2) {
                const double2 y0 = *reinterpret_cast<const double2*>(&y[c * RW + q]);
                const double2 y1 = *reinterpret_cast<const double2*>(&y[(c + 1) * RW + q]);
                acc[q] = fma(wi.x, y0.x, acc[q]);
                acc[q + 1] = fma(wi.x, y0.y, acc[q + 1]);
                acc[q] = fma(wi.y, y1.x, acc[q]);
                acc[q + 1] = fma(wi.y, y1.y, acc[q + 1]);
            }
        }
#pragma unroll
        for (int q = 0; q < RW; ++q) {
            acc[q] += __shfl_xor(acc[q], 1);
            acc[q] += __shfl_xor(acc[q], 2);
        }
        if (cp == 0) {
#pragma unroll
            for (int q = 0; q < RW; ++q) {
                wv[i * RW + q] = acc[q];
                st_wt(&R[(size_t)(k0 + i) * RW + q], acc[q]);
            }
        }
    }
    __syncthreads();
    if (tid < NTH)   // contrib_k[i][j] = sum_r y[r][i] w[r][j]
        for (int o = tid >> 4; o < (RW - 1) * RW; o += NTH / 16) {
            const int i = o / RW, j = o % RW, rp = tid & 15;
            double sacc = 0.0;
#pragma unroll
            for (int h = 0; h < NB / 16; ++h) sacc = fma(y[(rp + 16 * h) * RW + i], wv[(rp + 16 * h) * RW + j], sacc);
            sacc += __shfl_xor(sacc, 1);
            sacc += __shfl_xor(sacc, 2);
            sacc += __shfl_xor(sacc, 4);
            sacc += __shfl_xor(sacc, 8);
            if (rp == 0) contrib[(size_t)k * (RW - 1) * RW + o] = sacc;
        }
}

// pbuf slot of the wide form: the product (4 doubles per thread of NTW) | the y terms (OPT per thread
// of the first NTH, NTH's partition)
template <int RW>
struct WideSlot {
    static constexpr int TPO = (NTH / (NB * RW)) > 0 ? NTH / (NB * RW) : 1;
    static constexpr int OPT = (NB * RW) / (NTH / TPO);
    static constexpr int SIZE = 4 * NTW + OPT * NTH;
};

template <int RW>
__global__ __launch_bounds__(NTW)
void chol_factor_w(double* __restrict__ S, int npad, double* __restrict__ R, const int4* __restrict__ tasks,
                   const int4* __restrict__ items, const int4* __restrict__ need, const int* __restrict__ src,
                   double* __restrict__ W, double* __restrict__ contrib, int* __restrict__ fail, double* pbuf,
                   int* tctr, int* ctr, int nitems, int nver, long long tmo) {
    if (step_gated(fail + 1)) return;
    __shared__ CholLds<RW> sm;
    __shared__ int sh[2];
    constexpr int TPO = WideSlot<RW>::TPO, OPT = WideSlot<RW>::OPT, SLOT = WideSlot<RW>::SIZE;
    const int tid = threadIdx.x;
    int* tver = ctr + 2;
    if (tid == 0) sh[0] = __hip_atomic_fetch_add((g_i32*)ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int tk = sh[0];
    const int4 it = items[tk], nd = need[tk];
    auto wait_ver = [&](int id, int v) {   // as chol_factor's
        long long t0 = wall_clock64();
        int last = -1;
        for (;;) {
            const int cur = __hip_atomic_load((g_i32*)&tver[id], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur >= v) return;
            if (cur != last) { last = cur; t0 = wall_clock64(); }
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > tmo) { atomicOr(fail, FAIL_FACTOR_WAIT); return; }
        }
    };
    const __amdgpu_buffer_rsrc_t rS = wt_rsrc(S), rW = wt_rsrc(W);
    double* ws = &sm.m[0][0];   // the inverse's workspace: sm.m | sm.n (contiguous, dead by then)
    int done_id = -1;
    if (it.y < 0) {     // leaf
        const int k = it.x, k0 = k * NB;
        f64x4 t;
        wtile_regs(t, S + (size_t)k0 * npad + k0, npad);
        for (int e = tid; e < NB * RW; e += NTW) sm.ra[e] = R[(size_t)k0 * RW + e];
        __syncthreads();
        chol_diag_tile_w<RW>(t, k, W + (size_t)k * NB * NB, R, sm.ra, sm.wv, contrib, fail, sm.a, ws, &tver[tver_id(k, k)]);
        done_id = tver_id(k, k);
    } else {
        const int4 task = tasks[it.x];
        const int a = task.x, b = task.y, a0 = a * NB, b0 = b * NB, n = it.w & 0xffff, j = it.y - task.z;
        const bool diag = (a == b), inv = (it.w >> 16) != 0;
        const int k = src[it.y], k0 = k * NB;
        double* dst = S + (size_t)a0 * npad + b0;
        if (tid == 0) {
            wait_ver(tver_id(a, k), nd.x);
            if (!diag) wait_ver(tver_id(b, k), nd.y);
            if (n == 1) wait_ver(tver_id(a, b), nd.w);
        }
        __syncthreads();
        f64x4 t = {0.0, 0.0, 0.0, 0.0};
        if (n == 1) {
            wtile_regs_wt(t, dst, npad);
            if (diag)
                for (int e = tid; e < NB * RW; e += NTW) sm.ra[e] = ld_wt(&R[(size_t)a0 * RW + e]);
        }
        tile_load_w_wt(sm.a, rS, (size_t)a0 * npad + k0, npad);                 // A_ak
        if (!diag) tile_load_w_wt(sm.n, rS, (size_t)b0 * npad + k0, npad);      // A_bk
        if (tid == 0) wait_ver(tver_id(k, k), nd.z - 1);   // W_k stored
        __syncthreads();
        tile_load_w_wt(sm.m, rW, (size_t)k * NB * NB, NB);                      // W_k
        __syncthreads();
        const f64x4 g = wmfma_nn(sm.a, sm.m);   // G = A_ak W_k (tile (wr, wc))
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.m[16 * wrow() + trow(r)][16 * wcol() + tcol()] = g[r];
        __syncthreads();
        const f64x4 upd = wmfma_nt(sm.m, diag ? sm.a : sm.n);   // G X^T
        double ys[OPT];
#pragma unroll
        for (int u = 0; u < OPT; ++u) ys[u] = 0.0;
        if (diag) {
            if (tid == 0) wait_ver(tver_id(k, k), nd.z);   // w_k (the R rows of k) stored
            __syncthreads();
            for (int e = tid; e < NB * RW; e += NTW) sm.rk[e] = ld_wt(&R[(size_t)k0 * RW + e]);
            __syncthreads();
            if (tid < NTH) {
                const int pp = tid % TPO;
#pragma unroll
                for (int u = 0; u < OPT; ++u) {
                    const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                    double sum = 0.0;
                    for (int c = pp; c < NB; c += TPO) sum = fma(sm.a[i][c], sm.rk[c * RW + q], sum);
                    if (TPO >= 2) sum += __shfl_xor(sum, 1);
                    if (TPO >= 4) sum += __shfl_xor(sum, 2);
                    ys[u] = sum;
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
                S[(size_t)(k0 + 16 * wcol() + tcol()) * npad + a0 + 16 * wrow() + trow(r)] = g[r];
        }
        bool fin = true;
        if (n > 1) {   // publish this part; the last arriver finishes the task
            double* slot = pbuf + (size_t)it.z * SLOT;
#pragma unroll
            for (int r = 0; r < 4; ++r) st_wt(&slot[r * NTW + tid], upd[r]);
            if (diag && tid < NTH)
#pragma unroll
                for (int u = 0; u < OPT; ++u) st_wt(&slot[4 * NTW + u * NTH + tid], ys[u]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                const bool last = __hip_atomic_fetch_add((g_i32*)&tctr[it.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1;
                if (last) {
                    tctr[it.x] = 0;
                    wait_ver(tver_id(a, b), nd.w);
                }
                sh[1] = last;
            }
            __syncthreads();
            fin = sh[1] != 0;
            if (fin) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                wtile_regs_wt(t, dst, npad);
                if (diag)
                    for (int e = tid; e < NB * RW; e += NTW) sm.ra[e] = ld_wt(&R[(size_t)a0 * RW + e]);
                __syncthreads();
                const double* base = pbuf + (size_t)(it.z - j) * SLOT;
                for (int jj = 0; jj < n; ++jj) {
                    const double* sl = base + (size_t)jj * SLOT;
#pragma unroll
                    for (int r = 0; r < 4; ++r) t[r] -= (jj == j) ? upd[r] : ld_wt(&sl[r * NTW + tid]);
                    if (diag && tid < NTH) {
#pragma unroll
                        for (int u = 0; u < OPT; ++u) {
                            const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                            const double y = (jj == j) ? ys[u] : ld_wt(&sl[4 * NTW + u * NTH + tid]);
                            if (tid % TPO == 0) sm.ra[i * RW + q] -= y;
                        }
                    }
                }
            }
        } else {
            t -= upd;
            if (diag && tid < NTH) {
#pragma unroll
                for (int u = 0; u < OPT; ++u) {
                    const int o = tid / TPO + u * (NTH / TPO), i = o / RW, q = o % RW;
                    if (tid % TPO == 0) sm.ra[i * RW + q] -= ys[u];
                }
            }
        }
        if (fin) {
            __syncthreads();
            if (diag && inv) {
                chol_diag_tile_w<RW>(t, a, W + (size_t)a * NB * NB, R, sm.ra, sm.wv, contrib, fail, sm.a, ws,
                                     &tver[tver_id(a, a)]);
            } else {
                wtile_store_wt(t, dst, npad);
                if (diag)
                    for (int e = tid; e < NB * RW; e += NTW) st_wt(&R[(size_t)a0 * RW + e], sm.ra[e]);
            }
            done_id = tver_id(a, b);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains before the version add
    __syncthreads();
    if (tid == 0) {
        if (done_id >= 0) __hip_atomic_fetch_add((g_i32*)&tver[done_id], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add((g_i32*)&ctr[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nitems - 1)
            for (int e = 0; e < nver + 2; ++e) __hip_atomic_store((g_i32*)&ctr[e], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Cross-rank all-reduce of the reduced system, compacted: the structurally nonzero lower tiles of
// S_cc (incl. the diagonal ones) + R | D | r_i, packed into one contiguous buffer and back.
// One workgroup per tile; the tail block (blockIdx.x == ntiles) moves the rest.
__global__ __launch_bounds__(256)
void chol_pack(const double* __restrict__ S, int npad, const int2* __restrict__ tiles, int ntiles, int tail,
               double* __restrict__ buf, int unpack_dir, const int* __restrict__ gate) {
    if (step_gated(gate)) return;
    if ((int)blockIdx.x < ntiles) {
        const int2 t = tiles[blockIdx.x];
        double* sp = const_cast<double*>(S) + (size_t)t.x * NB * npad + (size_t)t.y * NB;
        double* bp = buf + (size_t)blockIdx.x * NB * NB;
        for (int e = threadIdx.x; e < NB * NB; e += 256) {
            double* g = sp + (size_t)(e / NB) * npad + e % NB;
            if (unpack_dir) *g = bp[e]; else bp[e] = *g;
        }
    } else {
        double* rest = const_cast<double*>(S) + (size_t)npad * npad;
        double* bp = buf + (size_t)ntiles * NB * NB;
        for (int e = threadIdx.x; e < tail; e += 256) {
            if (unpack_dir) rest[e] = bp[e]; else bp[e] = rest[e];
        }
    }
}

// The intrinsics: D' = D - sum_k contrib_k[:, :K], r' = r_i - sum_k contrib_k[:, K] (panel order),
// K x K Cholesky (non-positive pivot -> bad), x_i = D'^-1 r' -> v (thread 0).  Threads t < K (K + 1)
// fill Dp; the caller's workgroup must reach the barrier inside.
template <int K>
__device__ __forceinline__ void intr_solve(const double* __restrict__ Dm, const double* __restrict__ ri,
                                           const double* __restrict__ contrib, int T, double* __restrict__ Dp,
                                           double (&v)[K], bool& bad) {
    constexpr int RW = K + 1;
    const int t = threadIdx.x;
    if (t < K * RW) {
        const int i = t / RW, j = t % RW;
        double s = j < K ? Dm[i * K + j] : ri[i];
#pragma unroll 8
        for (int k = 0; k < T; ++k) s -= contrib[(size_t)k * K * RW + t];   // loads issued 8 ahead, same order
        Dp[t] = s;
    }
    __syncthreads();
    bad = false;
    if (t == 0) {
        double L[K][K];
        for (int j = 0; j < K; ++j) {   // lower Cholesky of D' (its lower triangle), Eigen LLT order
            double d = Dp[j * RW + j];
            for (int m = 0; m < j; ++m) d -= L[j][m] * L[j][m];
            if (!(d > 0.0) || !isfinite(d)) { bad = true; d = 1.0; }
            L[j][j] = sqrt(d);
            for (int i = j + 1; i < K; ++i) {
                double s = Dp[i * RW + j];
                for (int m = 0; m < j; ++m) s -= L[i][m] * L[j][m];
                L[i][j] = s / L[j][j];
            }
        }
        for (int i = 0; i < K; ++i) {
            double s = Dp[i * RW + K];
            for (int m = 0; m < i; ++m) s -= L[i][m] * v[m];
            v[i] = s / L[i][i];
        }
        for (int i = K - 1; i >= 0; --i) {
            double s = v[i];
            for (int m = i + 1; m < K; ++m) s -= L[m][i] * v[m];
            v[i] = s / L[i][i];
        }
    }
}

// Back solve, one workgroup per panel in ONE launch (replaces chol_intr + chol_back, bit-identical
// results).  A workgroup takes a ticket (atomic counter) and the panel border[ticket]; border lists
// the panels root first (level descending), so every panel it waits for (its ancestors k, the
// upper tiles (i, k)) holds an earlier ticket and is already running or done: no residency or
// dispatch-order assumption.  Per workgroup:
//   * prefetch its ancestor tiles U(i, k) (written by earlier launches) into LDS;
//   * x_i = D'^-1 r' (intr_solve, every workgroup the same; ticket 0 also writes sol_i);
//   * z_i = w_i(r_c) - w_i(B) x_i - sum_k U(i, k) z_k once every ancestor's z_k is published;
//   * publish z_i: write-through (sc1) stores, every wave drains, then one lane's sc1 flag store;
//     the consumer polls the flags with sc1 loads (one lane) and reads z only with sc1 loads
//     behind the workgroup barrier, so no L1 line can be stale and no acquire fence is needed
//     (MI355X_MICROARCH.md, inter-workgroup visibility: the valid sc1-load form, table row 1).
// Spins are bounded (`tmo` ticks of the 100 MHz wall clock per ancestor): a timed-out wait sets fail
// bit 4 and the host re-runs the step with the per-level launches.  ctr = [ticket, finished, zdone[T]] is zero at launch; the
// last workgroup to finish zeroes it for the next launch (nobody polls by then).
constexpr int BS_PF = 4;                   // ancestor tiles prefetched into LDS per workgroup

template <int RW>
__global__ __launch_bounds__(NTH)
void chol_backsolve(const double* __restrict__ S, int npad, const double* __restrict__ R,
                    const double* __restrict__ Dm, const double* __restrict__ ri, const double* __restrict__ contrib,
                    int T, const int* __restrict__ border, const int* __restrict__ bs_start,
                    const int* __restrict__ bs_k, const int* __restrict__ rowmap, double* z,
                    double* __restrict__ xout, double* __restrict__ sol_i, int* ctr, int* __restrict__ fail,
                    long long tmo) {
    if (step_gated(fail + 1)) return;
    constexpr int K = RW - 1;
    __shared__ double Ut[BS_PF][NB / 4][NTH];   // thread-private: its 16 U values per prefetched tile
    __shared__ double Dp[K * RW], xs[K];
    __shared__ int sh[2];
    const int tid = threadIdx.x;
    if (tid == 0) sh[0] = __hip_atomic_fetch_add((g_i32*)ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int tk = sh[0], i = border[tk];
    const int row = tid >> 2, q = tid & 3, r = i * NB + row;
    const int e0 = bs_start[i], e1 = bs_start[i + 1];
    for (int e = e0; e < e1 && e - e0 < BS_PF; ++e) {
        const double* U = S + (size_t)r * npad + bs_k[e] * NB;
#pragma unroll
        for (int m = 0; m < NB / 4; ++m) Ut[e - e0][m][tid] = U[4 * m + q];
    }
    {
        double v[K];
        bool bad;
        intr_solve<K>(Dm, ri, contrib, T, Dp, v, bad);
        if (tid == 0) {
            for (int a = 0; a < K; ++a) xs[a] = v[a];
            if (tk == 0) {
                if (bad) atomicOr(fail, 1);
                for (int a = 0; a < K; ++a) sol_i[a] = v[a];
            }
        }
    }
    __syncthreads();
    double s = R[(size_t)r * RW + RW - 1];
#pragma unroll
    for (int a = 0; a < K; ++a) s -= R[(size_t)r * RW + a] * xs[a];
    if (tid == 0) {   // ONE lane polls (relaxed), then ONE agent acquire
        bool ok = true;
        for (int e = e0; e < e1 && ok; ++e) {   // each ancestor's flag gets its own bound (progress restarts it)
            const long long t0 = wall_clock64();
            while (__hip_atomic_load((g_i32*)&ctr[2 + bs_k[e]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - t0 > tmo) { atomicOr(fail, FAIL_BACK_WAIT); ok = false; break; }
            }
        }
        sh[1] = ok;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps the z loads below
    double t = 0.0;
    if (sh[1]) {
        for (int e = e0; e < e1; ++e) {
            const int k0 = bs_k[e] * NB;
            if (e - e0 < BS_PF) {
#pragma unroll
                for (int m = 0; m < NB / 4; ++m) t = fma(Ut[e - e0][m][tid], ld_wt(&z[k0 + 4 * m + q]), t);
            } else {
                const double* U = S + (size_t)r * npad + k0;
#pragma unroll
                for (int m = 0; m < NB / 4; ++m) t = fma(U[4 * m + q], ld_wt(&z[k0 + 4 * m + q]), t);
            }
        }
    }
    t += __shfl_xor(t, 1);
    t += __shfl_xor(t, 2);
    if (q == 0) {
        s -= t;
        __hip_atomic_store((g_u64*)&z[r], (unsigned long long)__double_as_longlong(s), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);   // write-through
        const int o = rowmap[r];
        if (o >= 0) xout[o] = s;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains before the flag
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_store((g_i32*)&ctr[2 + i], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add((g_i32*)&ctr[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == T - 1)
            for (int w = 0; w < T + 2; ++w) __hip_atomic_store((g_i32*)&ctr[w], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The intrinsics (one workgroup of 64): x_i -> xi (device scalars for chol_back) and sol_i.
template <int K>
__global__ __launch_bounds__(64)
void chol_intr(const double* __restrict__ Dm, const double* __restrict__ ri, const double* __restrict__ contrib,
               int T, double* __restrict__ xi, double* __restrict__ sol_i, int* __restrict__ fail) {
    if (step_gated(fail + 1)) return;
    __shared__ double Dp[K * (K + 1)];
    double v[K];
    bool bad;
    intr_solve<K>(Dm, ri, contrib, T, Dp, v, bad);
    if (threadIdx.x == 0) {
        if (bad) atomicOr(fail, 1);
        for (int i = 0; i < K; ++i) { xi[i] = v[i]; sol_i[i] = v[i]; }
    }
}
// Back solve in one workgroup of 1024: z = w(r_c) - w(B) x_i, then per level, from the root down,
// z_i -= sum_k U(i, k) z_k over the ancestors k of panel i (upper tiles (i, k) = L~_ki^T); the
// camera solution leaves through rowmap (natural order 6c + d).  z lives in LDS (npad <= 16384).
template <int RW>
__global__ __launch_bounds__(1024)
void chol_back(const double* __restrict__ S, int npad, const double* __restrict__ R, const double* __restrict__ xi,
               int height, const int* __restrict__ lvl_start, const int* __restrict__ lvl_panels,
               const int* __restrict__ bs_start, const int* __restrict__ bs_k, const int* __restrict__ rowmap,
               double* __restrict__ xout, const int* __restrict__ gate) {
    if (step_gated(gate)) return;
    extern __shared__ double z[];
    const int tid = threadIdx.x;
    double xv[RW - 1];
#pragma unroll
    for (int i = 0; i < RW - 1; ++i) xv[i] = xi[i];
    for (int r = tid; r < npad; r += 1024) {
        double s = R[(size_t)r * RW + RW - 1];
#pragma unroll
        for (int i = 0; i < RW - 1; ++i) s -= R[(size_t)r * RW + i] * xv[i];
        z[r] = s;
    }
    __syncthreads();
    for (int l = height - 1; l >= 0; --l) {
        const int p0 = lvl_start[l], np = lvl_start[l + 1] - p0;
        // items: (panel, row), 4 lanes per item, 256 items per pass
        for (int it = tid >> 2; it < np * NB; it += 256) {
            const int i = lvl_panels[p0 + it / NB], row = i * NB + it % NB, q = tid & 3;
            double t = 0.0;
            for (int e = bs_start[i]; e < bs_start[i + 1]; ++e) {
                const int k0 = bs_k[e] * NB;
                const double* U = S + (size_t)row * npad + k0;
#pragma unroll
                for (int m = 0; m < NB / 4; ++m) t = fma(U[4 * m + q], z[k0 + 4 * m + q], t);
            }
            t += __shfl_xor(t, 1);
            t += __shfl_xor(t, 2);
            if (q == 0) z[row] -= t;
        }
        __syncthreads();
    }
    for (int r = tid; r < npad; r += 1024) {
        const int o = rowmap[r];
        if (o >= 0) xout[o] = z[r];
    }
}

}  // namespace ba
}  // namespace sfmx
