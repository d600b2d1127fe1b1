// SPDX-License-Identifier: MIT
// sfmx per-pair homography RANSAC for gfx950.
//
// Replaces SfM::calculateHomography (src/photogrammetrie/sfm/SfM.cpp:599-637):
// for every image pair, cv::findHomography(left, right, cv::RANSAC, thr, mask)
// on the aligned keypoints of its matches and the inlier ratio of the mask.
// OpenCV 4.5.1's RANSAC is deterministic (cv::RNG((uint64)-1)), so the whole
// computation is restated exactly (oracle/homography_oracle.cpp) and this
// kernel follows the same operation order with FMA contraction off (this file
// is compiled with -ffp-contract=off): the ratios agree bit for bit.
//
// One 256-thread workgroup per pair.  RANSAC iterations are processed in
// batches of B = 64 (32 in the first round) in iteration order:
//   1. wave 0 draws the next B minimal subsets: getSubset's attempts speculated
//      64 at a time (the RNG stream cut into attempts as the redraw loop reads
//      it, checkSubset on one lane each, the passing ones taken in order; r05);
//   2. lanes 0..B-1 fit one homography each (normalised DLT of the minimal
//      sample: its 8x8 system solved in registers, fp64);
//   3. each wave counts the inliers of a quarter of the hypotheses over the
//      pair's correspondences (fp32 reprojection error, ballot + popcount);
//   4. lane 0 replays the batch in order: best-so-far (strict >, at least 4
//      inliers) and the adaptive iteration count RANSACUpdateNumIters.
// Hypotheses past the (shrinking) iteration count are discarded.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/sfmx_homography.h"
#include "diag.hpp"
#include "match_common.hpp"

namespace sfmx {
namespace homog {

struct PairH {
    int32_t left, right;
    double thr;
};

// cv::RNG::next / uniform(0, count)
__device__ __forceinline__ uint32_t rng_next(unsigned long long& st) {
    st = (unsigned long long)(uint32_t)st * 4164903690ull + (uint32_t)(st >> 32);
    return (uint32_t)st;
}

// old with lane j set to the (uniform) v
__device__ __forceinline__ uint32_t wlane(uint32_t v, int j, uint32_t old) { return (threadIdx.x & 63) == (unsigned)j ? v : old; }
__device__ __forceinline__ int wlane(int v, int j, int old) { return (threadIdx.x & 63) == (unsigned)j ? v : old; }

// cv::RNG::next on the state's two halves in scalar registers (uniform)
__device__ __forceinline__ void rng_step_s(uint32_t& lo, uint32_t& hi) {
    const uint32_t m0 = lo * 4164903690u, m1 = __umulhi(lo, 4164903690u);
    lo = m0 + hi;
    hi = m1 + (lo < m0 ? 1u : 0u);
}
// the next 64 values of the stream, value j into lane j of x (v_writelane with an immediate lane: the
// value's SGPR is the instruction's one constant-bus read)
template <int J>
__device__ __forceinline__ void wlane_imm(uint32_t& x, uint32_t v) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(x) : "s"(v), "n"(J));
}
template <int... J>
__device__ __forceinline__ void rng64(uint32_t& x, uint32_t& y, uint32_t& lo, uint32_t& hi, std::integer_sequence<int, J...>) {
    ((rng_step_s(lo, hi), wlane_imm<J>(x, lo), wlane_imm<J>(y, hi)), ...);
}

// Minimal-sample solve (the oracle's solve8): [Lx; Ly] h = 0 of 4 normalised
// correspondences with h8 = 1, Gaussian elimination with the compare-and-swap
// pivot sweep, back substitution.  Fully unrolled: every index is static, so
// the 8x9 system lives in registers.
__device__ __forceinline__ bool solve8(double (&a)[8][9], double (&h)[9]) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
        for (int r = c + 1; r < 8; ++r) {
            const bool sw = fabs(a[r][c]) > fabs(a[c][c]);
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                const double u = a[r][j], v = a[c][j];
                a[r][j] = sw ? v : u;
                a[c][j] = sw ? u : v;
            }
        }
        ok = ok && a[c][c] != 0.0;
        const double piv = a[c][c] != 0.0 ? a[c][c] : 1.0;
#pragma unroll
        for (int r = c + 1; r < 8; ++r) {
            const double f = a[r][c] / piv;
#pragma unroll
            for (int j = c + 1; j < 9; ++j) a[r][j] -= f * a[c][j];
        }
    }
#pragma unroll
    for (int r = 7; r >= 0; --r) {
        double t = a[r][8];
#pragma unroll
        for (int j = r + 1; j < 8; ++j) t -= a[r][j] * h[j];
        h[r] = t / (a[r][r] != 0.0 ? a[r][r] : 1.0);
    }
    h[8] = 1.0;
    return ok;
}

// HomographyEstimatorCallback::runKernel on the 4 correspondences of a minimal
// sample, c[i] = (src.x, src.y, dst.x, dst.y) -> H (row-major, H[8] = 1);
// false if degenerate.  scales_only: stop after runKernel's own failure test (zero spread).
__device__ bool dlt4(const float4 (&c)[4], double (&H)[9], bool scales_only = false) {
    const int count = 4;
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
#pragma unroll
    for (int i = 0; i < count; ++i) {
        cmx += c[i].z; cmy += c[i].w;
        cMx += c[i].x; cMy += c[i].y;
    }
    cmx /= count; cmy /= count; cMx /= count; cMy /= count;
#pragma unroll
    for (int i = 0; i < count; ++i) {
        smx += fabs(c[i].z - cmx); smy += fabs(c[i].w - cmy);
        sMx += fabs(c[i].x - cMx); sMy += fabs(c[i].y - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
        return false;
    if (scales_only) return true;
    smx = count / smx; smy = count / smy; sMx = count / sMx; sMy = count / sMy;
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double a[8][9];
#pragma unroll
    for (int i = 0; i < count; ++i) {
        const double x = (c[i].z - cmx) * smx, y = (c[i].w - cmy) * smy;
        const double X = (c[i].x - cMx) * sMx, Y = (c[i].y - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[2 * i][j] = Lx[j]; a[2 * i + 1][j] = Ly[j]; }
        a[2 * i][8] = -Lx[8];
        a[2 * i + 1][8] = -Ly[8];
    }
    double H0[9];
    if (!solve8(a, H0)) return false;
    double Ht[9], H1[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s += invHnorm[3 * r + k] * H0[3 * k + cc];
            Ht[3 * r + cc] = s;
        }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s += Ht[3 * r + k] * Hnorm2[3 * k + cc];
            H1[3 * r + cc] = s;
        }
    const double sc = 1. / H1[8];
#pragma unroll
    for (int i = 0; i < 9; ++i) H[i] = H1[i] * sc;
    return true;
}

// haveCollinearPoints(m, 4) on one side of the subset (x at stride 4, from offset o)
__device__ __forceinline__ bool collinear4(const float (&q)[4][4], int o) {
    const int i = 3;
#pragma unroll
    for (int j = 0; j < i; ++j) {
        const double dx1 = (double)q[j][o] - q[i][o], dy1 = (double)q[j][o + 1] - q[i][o + 1];
#pragma unroll
        for (int k = 0; k < j; ++k) {
            const double dx2 = (double)q[k][o] - q[i][o], dy2 = (double)q[k][o + 1] - q[i][o + 1];
            if (fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return true;
        }
    }
    return false;
}

__device__ __forceinline__ double det3(double a0, double a1, double b0, double b1, double c0, double c1) {
    return a0 * (b1 - c1) - a1 * (b0 - c0) + (b0 * c1 - b1 * c0);
}

__device__ __forceinline__ bool check_subset(const float (&q)[4][4]) {
    if (collinear4(q, 0) || collinear4(q, 2)) return false;
    const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {1, 3, 0}};
    int negative = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int* t = tt[i];
        const double dA = det3(q[t[0]][0], q[t[0]][1], q[t[1]][0], q[t[1]][1], q[t[2]][0], q[t[2]][1]);
        const double dB = det3(q[t[0]][2], q[t[0]][3], q[t[1]][2], q[t[1]][3], q[t[2]][2], q[t[2]][3]);
        negative += dA * dB < 0;
    }
    return negative == 0 || negative == 4;
}

__device__ int update_num_iters(double p, double ep, int max_iters) {
    p = fmax(p, 0.); p = fmin(p, 1.);
    ep = fmax(ep, 0.); ep = fmin(ep, 1.);
    double num = fmax(1. - p, DBL_MIN);
    const double q = 1. - ep, q2 = q * q;
    double denom = 1. - q2 * q2;
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)rint(num / denom);
}

#ifdef SFMX_HOMOG_STAMPS   // tools/micro/homog_stamps.hip: phase timestamps of workgroup 0 (never in the product build)
__device__ long long g_h_stamps[256];
__device__ int g_h_nst;
#define H_STAMP(tag) do { if (threadIdx.x == 0 && blockIdx.x == 0 && g_h_nst < 254) { g_h_stamps[g_h_nst++] = (wall_clock64() << 8) | (tag); } } while (0)
#else
#define H_STAMP(tag) do { } while (0)
#endif

constexpr int CAP = 2048;   // correspondences kept in LDS (larger pairs read the global scratch copy)
constexpr int BATCH = 64;   // hypotheses per round (the first round draws 16)

__global__ __launch_bounds__(256)
void homography_ransac_kernel(const float2* const* __restrict__ kp, const int32_t* __restrict__ nkp,
                              const PairH* __restrict__ pairs, const DMatchDev* __restrict__ matches,
                              const int64_t* __restrict__ off, float4* __restrict__ scratch, int64_t scratch_cap,
                              int max_iters, double confidence, double* __restrict__ out, int serial) {
    __shared__ float4 pts[CAP];
    __shared__ int sub[BATCH][4];
    __shared__ float hf[BATCH][8];
    __shared__ int okb[BATCH], good[BATCH];
    __shared__ int s_nb, s_fail_at, s_done, s_niters, s_maxgood, s_it;
    constexpr int NV = 320;   // RNG values per speculation round (> 64 attempts unless n is tiny)
    __shared__ int s_idx[NV];
    __shared__ uint32_t s_stl[NV], s_sth[NV];
    __shared__ int4 s_att[64];
    __shared__ int s_aend[64];
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t o0 = off[p];
    const int n = (int)(off[p + 1] - o0);
    if (n < 4) {
        if (tid == 0) out[p] = -1.0;
        return;
    }
    if (n > CAP && (o0 < 0 || o0 + n > scratch_cap)) {   // (device inputs: a list past the scratch bound)
        if (tid == 0) out[p] = __builtin_nan("");
        return;
    }
    const PairH P = pairs[p];
    const float2* kl = kp[P.left];
    const float2* kr = kp[P.right];
    const int nl = nkp[P.left], nr = nkp[P.right];
    bool bad = false;
    for (int i = tid; i < n; i += 256) {
        const DMatchDev d = matches[o0 + i];
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (d.queryIdx < 0 || d.queryIdx >= nl || d.trainIdx < 0 || d.trainIdx >= nr) bad = true;
        else {
            const float2 a = kl[d.queryIdx], b = kr[d.trainIdx];
            v = make_float4(a.x, a.y, b.x, b.y);
        }
        if (n <= CAP) pts[i] = v;
        else scratch[o0 + i] = v;
    }
    if (__syncthreads_or(bad)) {
        if (tid == 0) out[p] = __builtin_nan("");
        return;
    }
    const float4* C = n <= CAP ? pts : scratch + o0;
    H_STAMP(1);
    if (n == 4) {   // findHomography: 4 points -> result = runKernel > 0 (fails only on zero spread), mask all ones
        if (tid == 0) {
            const float4 c4[4] = {C[0], C[1], C[2], C[3]};
            double H[9];
            out[p] = dlt4(c4, H, true) ? 1.0 : 0.0;
        }
        return;
    }
    const float thr2 = (float)(P.thr * P.thr);
    unsigned long long rng = ~0ull;   // cv::RNG((uint64)-1): wave 0, the same value in every lane
    if (tid == 0) { s_niters = max(max_iters, 1); s_maxgood = 0; s_it = 0; s_done = 0; }
    __syncthreads();
    for (;;) {
        if (wid == 0 && !serial) {   // 1. the next minimal subsets, in iteration order (r05, wave 0)
            // getSubset's attempts are speculated 64 at a time: the RNG stream (uniform, scalar) is cut
            // into attempts of 4 distinct indices exactly as the redraw loop consumes it (a value equal
            // to one already drawn in the attempt is skipped), lane a checks attempt a (checkSubset),
            // and the attempts are then taken in order: every passing one is the next subset until the
            // batch is full, and getSubset fails after 10000 consecutive rejected attempts.  The RNG
            // resumes after the last attempt taken.  The same subsets as the serial draw, 64 checks at a
            // time instead of one (the serial lane-0 draw was most of the kernel: ~3 us per subset).
            const int want = min(s_it == 0 ? BATCH / 2 : BATCH, s_niters - s_it);
            int b = 0, fail_at = -1, natt = 0;
            // the stream in scalar registers (uniform): cv::RNG::next on two 32-bit halves
            uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)rng), hi = __builtin_amdgcn_readfirstlane((uint32_t)(rng >> 32));
            int full = 0;   // (1: a round that formed no attempt is redone with every value slot)
            while (b < want) {
                const uint32_t lo0 = lo, hi0 = hi;
                // (a) nv values (enough for the attempts still wanted, ~4.1 values each, with margin):
                // value k's index (value % n) to LDS; the stream itself in scalar registers, each value
                // written into lane k % 64 by v_writelane (one VALU instruction per value)
                const int nr = full ? NV / 64 : min(NV / 64, (9 * (want - b) + 16 + 63) / 64), nv = 64 * nr;   // (checkSubset passes ~2/3)
                {
                    uint32_t vl[NV / 64], vh[NV / 64];   // (the state after each value: where the stream resumes)
#pragma unroll
                    for (int r = 0; r < NV / 64; ++r) {
                        vl[r] = vh[r] = 0u;
                        if (r < nr) rng64(vl[r], vh[r], lo, hi, std::make_integer_sequence<int, 64>{});
                    }
#pragma unroll
                    for (int r = 0; r < NV / 64; ++r)
                        if (r < nr) {
                            s_idx[64 * r + lane] = (int)(vl[r] % (uint32_t)n);
                            s_stl[64 * r + lane] = vl[r];
                            s_sth[64 * r + lane] = vh[r];
                        }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                H_STAMP(5);
                // (b) the attempts: runs without a repeated index are consecutive groups of 4 (lane a takes
                // the group at pos + 4a); the first group with a repeat is resolved as the redraw loop reads it
                int na = 0, pos = 0;
                while (na < 64 && pos + 4 <= nv) {
                    const int s0 = pos + 4 * lane;
                    bool ok = false;
                    int v0 = 0, v1 = 0, v2 = 0, v3 = 0;
                    if (na + lane < 64 && s0 + 4 <= nv) {
                        v0 = s_idx[s0]; v1 = s_idx[s0 + 1]; v2 = s_idx[s0 + 2]; v3 = s_idx[s0 + 3];
                        ok = v0 != v1 && v0 != v2 && v0 != v3 && v1 != v2 && v1 != v3 && v2 != v3;
                    }
                    const uint64_t okm = __ballot(ok);
                    const int f = ~okm ? (int)__builtin_ctzll(~okm) : 64;   // groups 0 .. f-1 are attempts as they stand
                    if (lane < f) { s_att[na + lane] = make_int4(v0, v1, v2, v3); s_aend[na + lane] = s0 + 3; }
                    na += f;
                    pos += 4 * f;
                    if (na >= 64 || pos + 4 > nv) break;
                    // group f: the redraw loop's own reading of the values from pos (uniform, scalar)
                    int c0 = 0, c1 = 0, c2 = 0, c3 = 0, ci = 0, k = pos;
                    for (; k < nv && ci < 4; ++k) {
                        const int v = __builtin_amdgcn_readfirstlane(s_idx[k]);
                        if (ci > 0 && (v == c0 || (ci > 1 && v == c1) || (ci > 2 && v == c2))) continue;   // redraw
                        if (ci == 0) c0 = v;
                        else if (ci == 1) c1 = v;
                        else if (ci == 2) c2 = v;
                        else c3 = v;
                        ++ci;
                    }
                    if (ci < 4) break;   // (the values ran out inside this attempt)
                    if (lane == 0) { s_att[na] = make_int4(c0, c1, c2, c3); s_aend[na] = k - 1; }
                    ++na;
                    pos = k;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                H_STAMP(6);
                if (na == 0) {   // fewer than 4 distinct indices in nv values (n tiny): never in practice
                    lo = lo0;
                    hi = hi0;
                    if (!full) { full = 1; continue; }
                    fail_at = s_it + b;   // (320 values without 4 distinct indices: a bound, not OpenCV's)
                    break;
                }
                // (c) checkSubset of every attempt, one per lane
                bool pass = false;
                int4 ai = make_int4(0, 0, 0, 0);
                if (lane < na) {
                    ai = s_att[lane];
                    float q[4][4];
                    const int id[4] = {ai.x, ai.y, ai.z, ai.w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float4 v = C[id[i]];
                        q[i][0] = v.x; q[i][1] = v.y; q[i][2] = v.z; q[i][3] = v.w;
                    }
                    pass = check_subset(q);
                }
                const uint64_t pm = __ballot(pass);
                H_STAMP(7);
                // (d) in order: the passing attempts are the next subsets until the batch is full; getSubset
                // fails after 10000 rejected attempts in a row
                const int need = want - b;
                const int npass = __popcll(pm);
                const int first = pm ? (int)__builtin_ctzll(pm) : na;
                if (natt + first >= 10000) { fail_at = s_it + b; break; }
                int last;   // the last attempt consumed
                if (npass >= need) {
                    uint64_t mm = pm;   // the need-th passing attempt
                    for (int i = 1; i < need; ++i) mm &= mm - 1;
                    last = (int)__builtin_ctzll(mm);
                } else {
                    last = na - 1;
                }
                const int rank = __popcll(pm & ((1ull << lane) - 1));
                if (pass && lane <= last) { sub[b + rank][0] = ai.x; sub[b + rank][1] = ai.y; sub[b + rank][2] = ai.z; sub[b + rank][3] = ai.w; }
                b += min(npass, need);
                if (b < want) {   // every attempt consumed: the rejections after the last pass carry over
                    const int lastpass = pm ? 63 - (int)__builtin_clzll(pm) : -1;
                    natt = pm ? na - 1 - lastpass : natt + na;
                    if (natt >= 10000) { fail_at = s_it + b; break; }
                }
                // the stream resumes after the last attempt taken
                const int kend = __builtin_amdgcn_readfirstlane(s_aend[last]);
                lo = __builtin_amdgcn_readfirstlane(s_stl[kend]);
                hi = __builtin_amdgcn_readfirstlane(s_sth[kend]);
            }
            rng = ((unsigned long long)hi << 32) | lo;
            if (lane == 0) { s_nb = b; s_fail_at = fail_at; }
        }
        if (tid == 0 && serial) {   // 1. (diagnostic A/B: r04's serial draw on lane 0, SFMX_HOMOG_SERIAL)
            int b = 0;
            s_fail_at = -1;
            const int want = s_it == 0 ? BATCH / 2 : BATCH;
            for (; b < want && s_it + b < s_niters; ++b) {
                float q[4][4];
                int att = 0;
                for (; att < 10000; ++att) {
                    int idx[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {   // static i: idx / q stay in registers
                        int idx_i;
                        bool dup;
                        do {
                            idx_i = (int)(rng_next(rng) % (uint32_t)n);
                            dup = false;
#pragma unroll
                            for (int j = 0; j < i; ++j) dup = dup || idx_i == idx[j];
                        } while (dup);
                        idx[i] = idx_i;
                        const float4 v = C[idx_i];
                        q[i][0] = v.x; q[i][1] = v.y; q[i][2] = v.z; q[i][3] = v.w;
                    }
                    if (!check_subset(q)) continue;
#pragma unroll
                    for (int i = 0; i < 4; ++i) sub[b][i] = idx[i];
                    break;
                }
                if (att >= 10000) { s_fail_at = s_it + b; break; }
            }
            s_nb = b;
        }
        __syncthreads();
        H_STAMP(2);
        const int nb = s_nb;
        if (tid < nb) {   // 2. one hypothesis per lane
            const float4 c4[4] = {C[sub[tid][0]], C[sub[tid][1]], C[sub[tid][2]], C[sub[tid][3]]};
            double H[9];
            const bool ok = dlt4(c4, H);
            okb[tid] = ok;
            good[tid] = 0;
            for (int i = 0; i < 8; ++i) hf[tid][i] = (float)H[i];
        }
        __syncthreads();
        H_STAMP(3);
        // 3. inlier counts (computeError + findInliers).  r05: wave w takes hypotheses w, w + 4, ... whole,
        // its lanes walk the correspondences and a ballot + popcount per 64 of them sums the count (r04: all
        // 256 threads per hypothesis, a shuffle reduction and an LDS atomic each: ~0.7 us per hypothesis)
        for (int b = wid; b < nb; b += 4) {
            if (!okb[b]) continue;
            const float h0 = hf[b][0], h1 = hf[b][1], h2 = hf[b][2], h3 = hf[b][3], h4 = hf[b][4], h5 = hf[b][5],
                        h6 = hf[b][6], h7 = hf[b][7];
            int cnt = 0;
            for (int i0 = 0; i0 < n; i0 += 4 * 64) {   // (4 loads in flight per lane)
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = i0 + 64 * u + lane;
                    v[u] = C[min(i, n - 1)];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float ww = 1.f / (h6 * v[u].x + h7 * v[u].y + 1.f);
                    const float dx = (h0 * v[u].x + h1 * v[u].y + h2) * ww - v[u].z;
                    const float dy = (h3 * v[u].x + h4 * v[u].y + h5) * ww - v[u].w;
                    cnt += __popcll(__ballot(i0 + 64 * u + lane < n && (dx * dx + dy * dy) <= thr2));
                }
            }
            if (lane == 0) good[b] = cnt;
        }
        __syncthreads();
        H_STAMP(4);
        if (tid == 0) {   // 4. replay in iteration order
            for (int b = 0; b < nb; ++b) {
                if (s_it + b >= s_niters) { s_done = 1; break; }
                if (!okb[b]) continue;
                const int g = good[b];
                if (g > max(s_maxgood, 3)) {
                    s_maxgood = g;
                    s_niters = update_num_iters(confidence, (double)(n - g) / n, s_niters);
                }
            }
            s_it += nb;
            if (s_fail_at >= 0) {
                if (s_fail_at == 0) s_maxgood = 0;   // getSubset failed at iteration 0: RANSAC fails
                s_done = 1;
            }
            if (s_it >= s_niters) s_done = 1;
        }
        __syncthreads();
        if (s_done) break;
    }
    if (tid == 0) out[p] = s_maxgood > 0 ? (double)s_maxgood / (double)n : 0.0;
}

thread_local float g_last_ms = -1.f;

// Per device, kept between calls (r05): the device check's result, one device block for the call's
// tables / outputs / scratch (regrown with headroom), pinned staging for the small uploads and the
// ratios, two timing events.  r04 made ~7 hipMalloc / hipFree pairs, a device-properties query, a D2H
// of the pair offsets and pageable copies per call: twice the kernel's time around a 0.3 ms kernel.
struct Slot {
    bool checked = false;
    char* dev = nullptr;
    size_t dev_cap = 0;
    char* pin = nullptr;
    size_t pin_cap = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::mutex mu;   // one call per device at a time; calls on different devices run concurrently
};
Slot g_slot[64];
size_t r256(size_t b) { return (std::max<size_t>(b, 1) + 255) & ~(size_t)255; }

}  // namespace homog
}  // namespace sfmx

using namespace sfmx;
using namespace sfmx::homog;

extern "C" {

float sfmx_homography_last_kernel_ms(void) { return g_last_ms; }

int sfmx_homography_ratios(const sfmx_point2f* const* keypoints, const int32_t* n_keypoints, int32_t n_imgs,
                           const int32_t* image_size, const int32_t* pairs, int32_t n_pairs,
                           const sfmx_dmatch* matches, const int64_t* pair_offsets, double threshold,
                           int32_t max_iters, double confidence, int32_t inputs_on_device, int32_t device,
                           void* stream, double* out_ratio) {
    if (n_pairs < 0 || n_imgs < 0) { set_last_error("negative count"); return SFMX_EINVAL; }
    if (n_pairs == 0) return SFMX_OK;
    if (!keypoints || !n_keypoints || !image_size || !pairs || !pair_offsets || !out_ratio) {
        set_last_error("null argument");
        return SFMX_EINVAL;
    }
    if (!(confidence > 0.0 && confidence < 1.0)) { set_last_error("confidence must be in (0, 1)"); return SFMX_EINVAL; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { set_last_error("no HIP device visible"); return SFMX_EDEVICE; }
    if (device < 0 || device >= ndev) { set_last_error("device index out of range"); return SFMX_EINVAL; }
    if (device >= 64) { set_last_error("device index out of range"); return SFMX_EINVAL; }
    Slot& S = g_slot[device];
    std::lock_guard<std::mutex> lock(S.mu);
    if (!S.checked) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            set_last_error("sfmx kernels are built for gfx950 only");
            return SFMX_EDEVICE;
        }
        S.checked = true;
    }
    std::vector<PairH> ph(n_pairs);
    int64_t bound = 0;   // device inputs: the scratch bound (at most one match per query keypoint)
    for (int p = 0; p < n_pairs; ++p) {
        const int L = pairs[2 * p], R = pairs[2 * p + 1];
        if (L < 0 || L >= n_imgs || R < 0 || R >= n_imgs) { set_last_error("pair image index out of range"); return SFMX_EINVAL; }
        const double thr = threshold < 0 ? -threshold
                                         : std::max({image_size[2 * L], image_size[2 * L + 1], image_size[2 * R + 1],
                                                     image_size[2 * R + 1]}) * threshold;   // SfM.cpp:615-619
        ph[p] = PairH{L, R, thr};
        bound += std::max(n_keypoints[L], 0);
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    const hipStream_t st = (hipStream_t)stream;
    int rc = SFMX_OK;
    {
        int64_t total = bound, nk = 0;
        if (!inputs_on_device) {
            total = pair_offsets[n_pairs];
            for (int p = 0; p < n_pairs; ++p) {
                if (pair_offsets[p + 1] < pair_offsets[p]) { set_last_error("pair offsets not ascending"); rc = SFMX_EINVAL; goto done; }
                const int L = pairs[2 * p], R = pairs[2 * p + 1];
                for (int64_t i = pair_offsets[p]; i < pair_offsets[p + 1]; ++i)
                    if (matches[i].queryIdx < 0 || matches[i].queryIdx >= n_keypoints[L] || matches[i].trainIdx < 0 ||
                        matches[i].trainIdx >= n_keypoints[R]) {
                        set_last_error("match index outside its image's keypoints");
                        rc = SFMX_EINVAL;
                        goto done;
                    }
            }
            for (int i = 0; i < n_imgs; ++i) nk += n_keypoints[i];
        }
        {
            // device block: [keypoint table | counts | pairs | ratios | scratch | (host inputs: keypoints,
            // matches, offsets)]; the first three parts staged back to back and copied up at once
            const size_t b_kp = r256(sizeof(float2*) * std::max(n_imgs, 1)), b_nk = r256(sizeof(int32_t) * std::max(n_imgs, 1)),
                         b_ph = r256(sizeof(PairH) * n_pairs), b_out = r256(sizeof(double) * n_pairs),
                         b_scr = r256(sizeof(float4) * std::max<int64_t>(total, 1));
            const size_t b_kd = inputs_on_device ? 0 : r256(sizeof(float2) * nk),
                         b_md = inputs_on_device ? 0 : r256(sizeof(sfmx_dmatch) * total),
                         b_od = inputs_on_device ? 0 : r256(sizeof(int64_t) * (n_pairs + 1));
            const size_t need = b_kp + b_nk + b_ph + b_out + b_scr + b_kd + b_md + b_od;
            if (S.dev_cap < need) {
                if (S.dev) (void)hipFree(S.dev);
                S.dev = nullptr;
                S.dev_cap = 0;
                if (hipMalloc(reinterpret_cast<void**>(&S.dev), need + need / 4) != hipSuccess) {
                    S.dev = nullptr;
                    (void)hipGetLastError();
                    rc = SFMX_ENOMEM;
                    goto done;
                }
                S.dev_cap = need + need / 4;
            }
            const size_t need_pin = b_kp + b_nk + b_ph + b_out;
            if (S.pin_cap < need_pin) {
                if (S.pin) (void)hipHostFree(S.pin);
                S.pin = nullptr;
                S.pin_cap = 0;
                if (hipHostMalloc(reinterpret_cast<void**>(&S.pin), need_pin + need_pin / 4, hipHostMallocDefault) != hipSuccess) {
                    S.pin = nullptr;
                    rc = SFMX_ENOMEM;
                    goto done;
                }
                S.pin_cap = need_pin + need_pin / 4;
            }
            if (!S.e0 && (hipEventCreate(&S.e0) != hipSuccess || hipEventCreate(&S.e1) != hipSuccess)) { rc = SFMX_EDEVICE; goto done; }
            char* d = S.dev;
            const float2** kpd = reinterpret_cast<const float2**>(d);
            int32_t* nkd = reinterpret_cast<int32_t*>(d + b_kp);
            PairH* phd = reinterpret_cast<PairH*>(d + b_kp + b_nk);
            double* outd = reinterpret_cast<double*>(d + b_kp + b_nk + b_ph);
            float4* scr = reinterpret_cast<float4*>(d + b_kp + b_nk + b_ph + b_out);
            char* hx = d + b_kp + b_nk + b_ph + b_out + b_scr;
            const float2** hk = reinterpret_cast<const float2**>(S.pin);
            const int64_t* doff = pair_offsets;
            if (inputs_on_device) {
                for (int i = 0; i < n_imgs; ++i) hk[i] = reinterpret_cast<const float2*>(keypoints[i]);
            } else {   // host inputs: keypoints, matches and offsets go up (pageable copies)
                float2* kd = reinterpret_cast<float2*>(hx);
                auto* md = reinterpret_cast<sfmx_dmatch*>(hx + b_kd);
                auto* od = reinterpret_cast<int64_t*>(hx + b_kd + b_md);
                int64_t o = 0;
                for (int i = 0; i < n_imgs; ++i) {
                    if (n_keypoints[i] &&
                        hipMemcpyAsync(kd + o, keypoints[i], sizeof(float2) * n_keypoints[i], hipMemcpyHostToDevice, st) != hipSuccess) {
                        rc = SFMX_EDEVICE; goto done;
                    }
                    hk[i] = kd + o;
                    o += n_keypoints[i];
                }
                if ((total && hipMemcpyAsync(md, matches, sizeof(sfmx_dmatch) * total, hipMemcpyHostToDevice, st) != hipSuccess) ||
                    hipMemcpyAsync(od, pair_offsets, sizeof(int64_t) * (n_pairs + 1), hipMemcpyHostToDevice, st) != hipSuccess) {
                    rc = SFMX_EDEVICE; goto done;
                }
                matches = md;
                doff = od;
            }
            std::memcpy(S.pin + b_kp, n_keypoints, sizeof(int32_t) * n_imgs);
            std::memcpy(S.pin + b_kp + b_nk, ph.data(), sizeof(PairH) * n_pairs);
            double* hout = reinterpret_cast<double*>(S.pin + b_kp + b_nk + b_ph);
            if (hipMemcpyAsync(d, S.pin, b_kp + b_nk + b_ph, hipMemcpyHostToDevice, st) != hipSuccess) { rc = SFMX_EDEVICE; goto done; }
            (void)hipEventRecord(S.e0, st);
            homography_ransac_kernel<<<n_pairs, 256, 0, st>>>(kpd, nkd, phd, reinterpret_cast<const DMatchDev*>(matches),
                                                              doff, scr, std::max<int64_t>(total, 1), max_iters, confidence, outd,
                                                              SFMX_DIAG_ENV("SFMX_HOMOG_SERIAL") ? 1 : 0);
            (void)hipEventRecord(S.e1, st);
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(hout, outd, sizeof(double) * n_pairs, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                rc = SFMX_EDEVICE;
            } else {
                std::memcpy(out_ratio, hout, sizeof(double) * n_pairs);
                float ms = -1.f;
                (void)hipEventElapsedTime(&ms, S.e0, S.e1);
                g_last_ms = ms;
            }
        }
    done:;
        if (rc != SFMX_OK) (void)hipStreamSynchronize(st);   // nothing in flight from the pinned staging
    }
    if (rc == SFMX_EDEVICE) set_last_error("HIP error in sfmx_homography_ratios");
    if (rc == SFMX_ENOMEM) set_last_error("device allocation failed");
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
}

}  // extern "C"
