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
// batches of B = 64 in iteration order:
//   1. lane 0 draws the next B minimal subsets (the RNG stream and the
//      checkSubset rejections are sequential by definition);
//   2. lanes 0..B-1 fit one homography each (normalised DLT: 9x9 LtL, Jacobi
//      eigen-decomposition with OpenCV's pivot search, fp64);
//   3. all 256 threads count the inliers of every hypothesis over the pair's
//      correspondences (fp32 reprojection error, ballot + popcount);
//   4. lane 0 replays the batch in order: best-so-far (strict >, at least 4
//      inliers) and the adaptive iteration count RANSACUpdateNumIters.
// Hypotheses past the (shrinking) iteration count are discarded.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sfmx_homography.h"
#include "match_common.hpp"

namespace sfmx {
namespace homog {

struct PairH {
    int32_t left, right;
    double thr;
};

__device__ __forceinline__ double rhypot(double a, double b) { return sqrt(a * a + b * b); }

// cv::RNG::next / uniform(0, count)
__device__ __forceinline__ uint32_t rng_next(unsigned long long& st) {
    st = (unsigned long long)(uint32_t)st * 4164903690ull + (uint32_t)(st >> 32);
    return (uint32_t)st;
}

// hal::Jacobi on a symmetric 9x9 (eigenvectors as rows of V, eigenvalues descending).
__device__ void jacobi9(double (&A)[9][9], double (&W)[9], double (&V)[9][9]) {
    const int n = 9;
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) V[i][j] = 0.0;
        V[i][i] = 1.0;
    }
    int indR[9], indC[9];
    int k, m, i;
    double mv;
    for (k = 0; k < n; ++k) {
        W[k] = A[k][k];
        if (k < n - 1) {
            for (m = k + 1, mv = fabs(A[k][m]), i = k + 2; i < n; ++i) {
                const double v = fabs(A[k][i]);
                if (mv < v) mv = v, m = i;
            }
            indR[k] = m;
        }
        if (k > 0) {
            for (m = 0, mv = fabs(A[0][k]), i = 1; i < k; ++i) {
                const double v = fabs(A[i][k]);
                if (mv < v) mv = v, m = i;
            }
            indC[k] = m;
        }
    }
    const int maxIters = n * n * 30;
    for (int iters = 0; iters < maxIters; ++iters) {
        for (k = 0, mv = fabs(A[0][indR[0]]), i = 1; i < n - 1; ++i) {
            const double v = fabs(A[i][indR[i]]);
            if (mv < v) mv = v, k = i;
        }
        int l = indR[k];
        for (i = 1; i < n; ++i) {
            const double v = fabs(A[indC[i]][i]);
            if (mv < v) mv = v, k = indC[i], l = i;
        }
        const double p = A[k][l];
        if (fabs(p) <= DBL_EPSILON) break;
        const double y = (W[l] - W[k]) * 0.5;
        double t = fabs(y) + rhypot(p, y);
        double s = rhypot(p, t);
        const double c = t / s;
        s = p / s;
        t = (p / t) * p;
        if (y < 0) s = -s, t = -t;
        A[k][l] = 0;
        W[k] -= t;
        W[l] += t;
        double a0, b0;
#define ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
        for (i = 0; i < k; ++i) ROT(A[i][k], A[i][l]);
        for (i = k + 1; i < l; ++i) ROT(A[k][i], A[i][l]);
        for (i = l + 1; i < n; ++i) ROT(A[k][i], A[l][i]);
        for (i = 0; i < n; ++i) ROT(V[k][i], V[l][i]);
#undef ROT
        for (int j = 0; j < 2; ++j) {
            const int idx = j == 0 ? k : l;
            if (idx < n - 1) {
                for (m = idx + 1, mv = fabs(A[idx][m]), i = idx + 2; i < n; ++i) {
                    const double v = fabs(A[idx][i]);
                    if (mv < v) mv = v, m = i;
                }
                indR[idx] = m;
            }
            if (idx > 0) {
                for (m = 0, mv = fabs(A[0][idx]), i = 1; i < idx; ++i) {
                    const double v = fabs(A[i][idx]);
                    if (mv < v) mv = v, m = i;
                }
                indC[idx] = m;
            }
        }
    }
    for (k = 0; k < n - 1; ++k) {
        m = k;
        for (i = k + 1; i < n; ++i)
            if (W[m] < W[i]) m = i;
        if (k != m) {
            const double tw = W[m]; W[m] = W[k]; W[k] = tw;
            for (i = 0; i < n; ++i) { const double tv = V[m][i]; V[m][i] = V[k][i]; V[k][i] = tv; }
        }
    }
}

// HomographyEstimatorCallback::runKernel on `count` correspondences
// c[i] = (src.x, src.y, dst.x, dst.y) -> H (row-major, H[8] = 1); false if degenerate.
__device__ bool dlt(const float4* c, int count, double (&H)[9]) {
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
    for (int i = 0; i < count; ++i) {
        const float4 q = c[i];
        cmx += q.z; cmy += q.w;
        cMx += q.x; cMy += q.y;
    }
    cmx /= count; cmy /= count; cMx /= count; cMy /= count;
    for (int i = 0; i < count; ++i) {
        const float4 q = c[i];
        smx += fabs(q.z - cmx); smy += fabs(q.w - cmy);
        sMx += fabs(q.x - cMx); sMy += fabs(q.y - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
        return false;
    smx = count / smx; smy = count / smy; sMx = count / sMx; sMy = count / sMy;
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double LtL[9][9];
    for (int j = 0; j < 9; ++j)
        for (int k = 0; k < 9; ++k) LtL[j][k] = 0.0;
    for (int i = 0; i < count; ++i) {
        const float4 q = c[i];
        const double x = (q.z - cmx) * smx, y = (q.w - cmy) * smy;
        const double X = (q.x - cMx) * sMx, Y = (q.y - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        for (int j = 0; j < 9; ++j)
            for (int k = j; k < 9; ++k) LtL[j][k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    for (int j = 0; j < 9; ++j)
        for (int k = 0; k < j; ++k) LtL[j][k] = LtL[k][j];
    double W[9], V[9][9];
    jacobi9(LtL, W, V);
    double Ht[9], H1[9];
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += invHnorm[3 * r + k] * V[8][3 * k + cc];
            Ht[3 * r + cc] = s;
        }
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += Ht[3 * r + k] * Hnorm2[3 * k + cc];
            H1[3 * r + cc] = s;
        }
    const double sc = 1. / H1[8];
    for (int i = 0; i < 9; ++i) H[i] = H1[i] * sc;
    return true;
}

// haveCollinearPoints(m, 4) on one side of the subset (x at stride 4, from offset o)
__device__ bool collinear4(const float (&q)[4][4], int o) {
    const int i = 3;
    for (int j = 0; j < i; ++j) {
        const double dx1 = (double)q[j][o] - q[i][o], dy1 = (double)q[j][o + 1] - q[i][o + 1];
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

__device__ bool check_subset(const float (&q)[4][4]) {
    if (collinear4(q, 0) || collinear4(q, 2)) return false;
    const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {1, 3, 0}};
    int negative = 0;
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

constexpr int CAP = 2048;   // correspondences kept in LDS (larger pairs read the global scratch copy)
constexpr int BATCH = 64;   // hypotheses per round

__global__ __launch_bounds__(256)
void homography_ransac_kernel(const float2* const* __restrict__ kp, const int32_t* __restrict__ nkp,
                              const PairH* __restrict__ pairs, const DMatchDev* __restrict__ matches,
                              const int64_t* __restrict__ off, float4* __restrict__ scratch, int max_iters,
                              double confidence, double* __restrict__ out) {
    __shared__ float4 pts[CAP];
    __shared__ int sub[BATCH][4];
    __shared__ float hf[BATCH][8];
    __shared__ int okb[BATCH], good[BATCH];
    __shared__ int s_nb, s_fail_at, s_done, s_niters, s_maxgood, s_it;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int64_t o0 = off[p];
    const int n = (int)(off[p + 1] - o0);
    if (n < 4) {
        if (tid == 0) out[p] = -1.0;
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
    if (n == 4) {   // findHomography: 4 points -> the kernel directly, mask all ones
        if (tid == 0) {
            double H[9];
            out[p] = dlt(C, 4, H) ? 1.0 : 0.0;
        }
        return;
    }
    const float thr2 = (float)(P.thr * P.thr);
    unsigned long long rng = ~0ull;   // cv::RNG((uint64)-1), lane 0 only
    if (tid == 0) { s_niters = max(max_iters, 1); s_maxgood = 0; s_it = 0; s_done = 0; }
    __syncthreads();
    for (;;) {
        if (tid == 0) {   // 1. the next minimal subsets, in iteration order
            int b = 0;
            s_fail_at = -1;
            for (; b < BATCH && s_it + b < s_niters; ++b) {
                float q[4][4];
                int att = 0;
                for (; att < 10000; ++att) {
                    int idx[4];
                    for (int i = 0; i < 4; ++i) {
                        int idx_i, j;
                        for (;;) {
                            idx_i = idx[i] = (int)(rng_next(rng) % (uint32_t)n);
                            for (j = 0; j < i; ++j)
                                if (idx_i == idx[j]) break;
                            if (j == i) break;
                        }
                        const float4 v = C[idx_i];
                        q[i][0] = v.x; q[i][1] = v.y; q[i][2] = v.z; q[i][3] = v.w;
                        sub[b][i] = idx_i;
                    }
                    if (!check_subset(q)) continue;
                    break;
                }
                if (att >= 10000) { s_fail_at = s_it + b; break; }
            }
            s_nb = b;
        }
        __syncthreads();
        const int nb = s_nb;
        if (tid < nb) {   // 2. one hypothesis per lane
            float4 c4[4];
            for (int i = 0; i < 4; ++i) c4[i] = C[sub[tid][i]];
            double H[9];
            const bool ok = dlt(c4, 4, H);
            okb[tid] = ok;
            good[tid] = 0;
            for (int i = 0; i < 8; ++i) hf[tid][i] = (float)H[i];
        }
        __syncthreads();
        for (int b = 0; b < nb; ++b) {   // 3. inlier counts (computeError + findInliers)
            if (!okb[b]) continue;
            const float h0 = hf[b][0], h1 = hf[b][1], h2 = hf[b][2], h3 = hf[b][3], h4 = hf[b][4], h5 = hf[b][5],
                        h6 = hf[b][6], h7 = hf[b][7];
            int cnt = 0;
            for (int i = tid; i < n; i += 256) {
                const float4 v = C[i];
                const float ww = 1.f / (h6 * v.x + h7 * v.y + 1.f);
                const float dx = (h0 * v.x + h1 * v.y + h2) * ww - v.z;
                const float dy = (h3 * v.x + h4 * v.y + h5) * ww - v.w;
                cnt += (dx * dx + dy * dy) <= thr2;
            }
            for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
            if ((tid & 63) == 0 && cnt) atomicAdd(&good[b], cnt);
        }
        __syncthreads();
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

struct Bufs {
    std::vector<void*> ptrs;
    ~Bufs() { for (void* q : ptrs) (void)hipFree(q); }
    void* alloc(size_t bytes) {
        void* q = nullptr;
        if (hipMalloc(&q, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        ptrs.push_back(q);
        return q;
    }
};

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
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_last_error("sfmx kernels are built for gfx950 only");
        return SFMX_EDEVICE;
    }
    std::vector<PairH> ph(n_pairs);
    for (int p = 0; p < n_pairs; ++p) {
        const int L = pairs[2 * p], R = pairs[2 * p + 1];
        if (L < 0 || L >= n_imgs || R < 0 || R >= n_imgs) { set_last_error("pair image index out of range"); return SFMX_EINVAL; }
        const double thr = threshold < 0 ? -threshold
                                         : std::max({image_size[2 * L], image_size[2 * L + 1], image_size[2 * R + 1],
                                                     image_size[2 * R + 1]}) * threshold;   // SfM.cpp:615-619
        ph[p] = PairH{L, R, thr};
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    const hipStream_t st = (hipStream_t)stream;
    int rc = SFMX_OK;
    {
        Bufs b;
        std::vector<int64_t> hoff;
        const int64_t* doff = pair_offsets;
        int64_t total = 0;
        if (inputs_on_device) {
            hoff.resize(n_pairs + 1);
            if (hipMemcpyAsync(hoff.data(), pair_offsets, sizeof(int64_t) * (n_pairs + 1), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) { rc = SFMX_EDEVICE; goto done; }
            total = hoff[n_pairs];
        } else {
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
        }
        {
            std::vector<const float2*> kptr(std::max(n_imgs, 1));
            if (inputs_on_device) {
                for (int i = 0; i < n_imgs; ++i) kptr[i] = reinterpret_cast<const float2*>(keypoints[i]);
            } else {
                int64_t nk = 0;
                for (int i = 0; i < n_imgs; ++i) nk += n_keypoints[i];
                auto* kd = static_cast<float2*>(b.alloc(sizeof(float2) * nk));
                if (!kd) { rc = SFMX_ENOMEM; goto done; }
                int64_t o = 0;
                for (int i = 0; i < n_imgs; ++i) {
                    if (n_keypoints[i] &&
                        hipMemcpyAsync(kd + o, keypoints[i], sizeof(float2) * n_keypoints[i], hipMemcpyHostToDevice, st) != hipSuccess) {
                        rc = SFMX_EDEVICE; goto done;
                    }
                    kptr[i] = kd + o;
                    o += n_keypoints[i];
                }
                auto* md = static_cast<sfmx_dmatch*>(b.alloc(sizeof(sfmx_dmatch) * total));
                auto* od = static_cast<int64_t*>(b.alloc(sizeof(int64_t) * (n_pairs + 1)));
                if (!md || !od) { rc = SFMX_ENOMEM; goto done; }
                if ((total && hipMemcpyAsync(md, matches, sizeof(sfmx_dmatch) * total, hipMemcpyHostToDevice, st) != hipSuccess) ||
                    hipMemcpyAsync(od, pair_offsets, sizeof(int64_t) * (n_pairs + 1), hipMemcpyHostToDevice, st) != hipSuccess) {
                    rc = SFMX_EDEVICE; goto done;
                }
                matches = md;
                doff = od;
            }
            auto* kpd = static_cast<const float2**>(b.alloc(sizeof(float2*) * kptr.size()));
            auto* nkd = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * std::max(n_imgs, 1)));
            auto* phd = static_cast<PairH*>(b.alloc(sizeof(PairH) * n_pairs));
            auto* scr = static_cast<float4*>(b.alloc(sizeof(float4) * std::max<int64_t>(total, 1)));
            auto* outd = static_cast<double*>(b.alloc(sizeof(double) * n_pairs));
            if (!kpd || !nkd || !phd || !scr || !outd) { rc = SFMX_ENOMEM; goto done; }
            hipEvent_t e0 = nullptr, e1 = nullptr;
            if (hipMemcpyAsync(kpd, kptr.data(), sizeof(float2*) * kptr.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
                hipMemcpyAsync(nkd, n_keypoints, sizeof(int32_t) * n_imgs, hipMemcpyHostToDevice, st) != hipSuccess ||
                hipMemcpyAsync(phd, ph.data(), sizeof(PairH) * n_pairs, hipMemcpyHostToDevice, st) != hipSuccess ||
                hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
                rc = SFMX_EDEVICE; goto done;
            }
            (void)hipEventRecord(e0, st);
            homography_ransac_kernel<<<n_pairs, 256, 0, st>>>(kpd, nkd, phd, reinterpret_cast<const DMatchDev*>(matches),
                                                              doff, scr, max_iters, confidence, outd);
            (void)hipEventRecord(e1, st);
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(out_ratio, outd, sizeof(double) * n_pairs, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                rc = SFMX_EDEVICE;
            } else {
                float ms = -1.f;
                (void)hipEventElapsedTime(&ms, e0, e1);
                g_last_ms = ms;
            }
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
    done:;
    }
    if (rc == SFMX_EDEVICE) set_last_error("HIP error in sfmx_homography_ratios");
    if (rc == SFMX_ENOMEM) set_last_error("device allocation failed");
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
}

}  // extern "C"
