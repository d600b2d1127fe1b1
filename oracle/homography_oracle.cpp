// SPDX-License-Identifier: MIT
//
// sfmx ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's per-pair homography step:
//   SfM::calculateHomography(Scene&)            src/photogrammetrie/sfm/SfM.cpp:599-637
//     - pairs with < 4 matches are skipped (ratio stays -1, Scene.h:56)       :606-609
//     - aligned keypoints: left[queryIdx], right[trainIdx] (Scene.cpp:58-71)  :612-613
//     - threshold: t < 0 ? -t : max(wL, hL, hR, hR) * t  (the reference reads
//       rightSize.height twice; kept)                                          :615-619
//     - cv::findHomography(left, right, cv::RANSAC, threshold, mask)         :621-624
//     - ratio = countNonZero(mask) / matches.size()  (0 if H is empty)        :625-628
//   consumer: the initial-pair choice in SfM::triangulate, SfM.cpp:176-188.
//
// Third-party algorithm restated (absent from /root/reference): OpenCV 4.5.1
// calib3d [ext], cv::findHomography with its defaults maxIters = 2000,
// confidence = 0.995:
//   * 4 points: the direct kernel on all points, mask = all ones (0 if the
//     kernel fails).
//   * RANSACPointSetRegistrator::run with cv::RNG((uint64)-1) (multiply-with-
//     carry, coefficient 4164903690): getSubset draws 4 distinct indices by
//     rng.uniform(0, count) (= next() % count), rejecting duplicates, then
//     HomographyEstimatorCallback::checkSubset (haveCollinearPoints of the
//     last point vs. the pairs before it, in both sets, FLT_EPSILON test; the
//     orientation test on the 4 triangles {0,1,2},{1,2,3},{0,2,3},{1,3,0}:
//     det(A)*det(B) < 0 must hold for none or all), up to 10000 attempts.
//   * runKernel: normalised DLT — centroids, mean absolute deviations, the
//     normalised correspondences' equations, H0 = their null vector,
//     denormalised invHnorm * H0 * Hnorm2, scaled by 1/H(2,2).  OpenCV takes
//     H0 as the eigenvector of the smallest eigenvalue of the 9x9 LtL
//     (cv::eigen, Jacobi).  RANSAC only ever fits minimal samples (4 points,
//     8 equations of rank 8), whose null vector is unique up to scale, so
//     this restatement solves the 8x8 system with h8 = 1 instead (solve8):
//     the same H up to rounding, after the final 1/H(2,2) scaling.
//   * computeError in float: ww = 1/(h6 x + h7 y + 1), err = dx^2 + dy^2;
//     inlier iff err <= (float)(thr^2); a model replaces the best iff its
//     count > max(best, 3); niters = RANSACUpdateNumIters(0.995, outlier
//     fraction, 4, niters) after each improvement.
// The LM refinement that follows in findHomography changes H, not the mask,
// so it does not affect the ratio and is not restated.
// Deviations (documented in DESIGN.md): the minimal-sample null vector by an
// 8x8 solve instead of a 9x9 Jacobi eigen-decomposition (same H up to
// rounding; a RANSAC sample whose 8x8 system is exactly singular is skipped,
// where OpenCV would score cv::eigen's vector); (1-ep)^4 as two squarings; 3x3
// products sum in k order.  orc_homography_set_arith(1) switches the oracle to
// the LtL + Jacobi null vector for measuring that gap (tools/arith_gap.py).  The GPU
// kernel (csrc/homography.hip) follows the same operation order with FMA
// contraction off, so the two agree bit for bit; parity against OpenCV itself
// is unpinned (no OpenCV here).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <omp.h>

namespace {

struct Rng {
    uint64_t state;
    explicit Rng(uint64_t s) : state(s ? s : 0xffffffffull) {}
    uint32_t next() {
        state = (uint64_t)(uint32_t)state * 4164903690u + (uint32_t)(state >> 32);
        return (uint32_t)state;
    }
    int uniform(int a, int b) { return a == b ? a : (int)(next() % (uint32_t)(b - a) + (uint32_t)a); }
};

// Minimal-sample solve: the 8 equations [Lx; Ly] h = 0 of 4 normalised
// correspondences with h8 = 1 (augmented 8x9, right-hand side -L[:, 8]),
// Gaussian elimination with a compare-and-swap pivot sweep (for r > c: swap
// rows r and c when |a[r][c]| > |a[c][c]|), then back substitution.
bool solve8(double a[8][9], double h[9]) {
    for (int c = 0; c < 8; ++c) {
        for (int r = c + 1; r < 8; ++r)
            if (std::fabs(a[r][c]) > std::fabs(a[c][c]))
                for (int j = 0; j < 9; ++j) std::swap(a[r][j], a[c][j]);
        if (a[c][c] == 0.0) return false;
        for (int r = c + 1; r < 8; ++r) {
            const double f = a[r][c] / a[c][c];
            for (int j = c + 1; j < 9; ++j) a[r][j] -= f * a[c][j];
        }
    }
    for (int r = 7; r >= 0; --r) {
        double t = a[r][8];
        for (int j = r + 1; j < 8; ++j) t -= a[r][j] * h[j];
        h[r] = t / a[r][r];
    }
    h[8] = 1.0;
    return true;
}

// ---- OpenCV-arithmetic model (orc_homography_set_arith; measurement only) ----
// 1: the minimal-sample null vector as OpenCV 4.5.1 computes it: LtL = sum Lx^T Lx + Ly^T Ly
// (upper triangle, j <= k, then completeSymm), cv::eigen -> hal::Jacobi (cyclic-max pivot with the
// indR / indC row and column maxima, hypot rotations, |p| <= DBL_EPSILON stop, n*n*30 rotations at
// most, eigenvalues sorted descending with their rows of V), H0 = the last row of V.
int g_harith = 0;

void jacobi9(double A[9][9], double W[9], double V[9][9]) {
    const int n = 9;
    const double eps = DBL_EPSILON;
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) V[i][j] = 0;
        V[i][i] = 1;
    }
    int indR[9] = {0}, indC[9] = {0};
    auto row_max = [&](int k) {   // argmax_{i > k} |A[k][i]|
        int m = k + 1;
        double mv = std::fabs(A[k][m]);
        for (int i = k + 2; i < n; i++) {
            const double v = std::fabs(A[k][i]);
            if (mv < v) mv = v, m = i;
        }
        indR[k] = m;
    };
    auto col_max = [&](int k) {   // argmax_{i < k} |A[i][k]|
        int m = 0;
        double mv = std::fabs(A[0][k]);
        for (int i = 1; i < k; i++) {
            const double v = std::fabs(A[i][k]);
            if (mv < v) mv = v, m = i;
        }
        indC[k] = m;
    };
    for (int k = 0; k < n; k++) {
        W[k] = A[k][k];
        if (k < n - 1) row_max(k);
        if (k > 0) col_max(k);
    }
    for (int iters = 0; iters < n * n * 30; iters++) {
        int k = 0;
        double mv = std::fabs(A[0][indR[0]]);
        for (int i = 1; i < n - 1; i++) {
            const double v = std::fabs(A[i][indR[i]]);
            if (mv < v) mv = v, k = i;
        }
        int l = indR[k];
        for (int i = 1; i < n; i++) {
            const double v = std::fabs(A[indC[i]][i]);
            if (mv < v) mv = v, k = indC[i], l = i;
        }
        const double p = A[k][l];
        if (std::fabs(p) <= eps) break;
        const double y = (W[l] - W[k]) * 0.5;
        double t = std::fabs(y) + std::hypot(p, y);
        double s = std::hypot(p, t);
        const double c = t / s;
        s = p / s;
        t = (p / t) * p;
        if (y < 0) s = -s, t = -t;
        A[k][l] = 0;
        W[k] -= t;
        W[l] += t;
        auto rot = [&](double& v0, double& v1) {
            const double a0 = v0, b0 = v1;
            v0 = a0 * c - b0 * s;
            v1 = a0 * s + b0 * c;
        };
        for (int i = 0; i < k; i++) rot(A[i][k], A[i][l]);
        for (int i = k + 1; i < l; i++) rot(A[k][i], A[i][l]);
        for (int i = l + 1; i < n; i++) rot(A[k][i], A[l][i]);
        for (int i = 0; i < n; i++) rot(V[k][i], V[l][i]);
        for (int j = 0; j < 2; j++) {
            const int idx = j == 0 ? k : l;
            if (idx < n - 1) row_max(idx);
            if (idx > 0) col_max(idx);
        }
    }
    for (int k = 0; k < n - 1; k++) {
        int m = k;
        for (int i = k + 1; i < n; i++)
            if (W[m] < W[i]) m = i;
        if (k != m) {
            std::swap(W[m], W[k]);
            for (int i = 0; i < n; i++) std::swap(V[m][i], V[k][i]);
        }
    }
}

// HomographyEstimatorCallback::runKernel on `count` correspondences
// (M = left/src, m = right/dst, float x,y interleaved) -> H (row-major, H[8] = 1).  runKernel
// itself fails only on the zero-spread test (cv::eigen always returns a vector); solve8 also
// reports a singular minimal system.  scales_only: stop after the spread test (findHomography's
// 4-point path needs only runKernel's return value).
bool dlt(const float* M, const float* m, int count, double H[9], bool scales_only = false) {
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
    for (int i = 0; i < count; ++i) {
        cmx += m[2 * i]; cmy += m[2 * i + 1];
        cMx += M[2 * i]; cMy += M[2 * i + 1];
    }
    cmx /= count; cmy /= count; cMx /= count; cMy /= count;
    for (int i = 0; i < count; ++i) {
        smx += std::fabs(m[2 * i] - cmx); smy += std::fabs(m[2 * i + 1] - cmy);
        sMx += std::fabs(M[2 * i] - cMx); sMy += std::fabs(M[2 * i + 1] - cMy);
    }
    if (std::fabs(smx) < DBL_EPSILON || std::fabs(smy) < DBL_EPSILON || std::fabs(sMx) < DBL_EPSILON ||
        std::fabs(sMy) < DBL_EPSILON)
        return false;
    if (scales_only) return true;
    smx = count / smx; smy = count / smy; sMx = count / sMx; sMy = count / sMy;
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double a[8][9], LtL[9][9] = {{0}};
    for (int i = 0; i < count; ++i) {   // count == 4: the minimal sample
        const double x = (m[2 * i] - cmx) * smx, y = (m[2 * i + 1] - cmy) * smy;
        const double X = (M[2 * i] - cMx) * sMx, Y = (M[2 * i + 1] - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        if (g_harith & 1) {
            for (int j = 0; j < 9; j++)
                for (int k = j; k < 9; k++) LtL[j][k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
            continue;
        }
        for (int j = 0; j < 8; ++j) { a[2 * i][j] = Lx[j]; a[2 * i + 1][j] = Ly[j]; }
        a[2 * i][8] = -Lx[8];
        a[2 * i + 1][8] = -Ly[8];
    }
    double H0[9];
    if (g_harith & 1) {
        for (int j = 0; j < 9; j++)
            for (int k = 0; k < j; k++) LtL[j][k] = LtL[k][j];
        double W[9], V[9][9];
        jacobi9(LtL, W, V);
        for (int i = 0; i < 9; ++i) H0[i] = V[8][i];
    } else if (!solve8(a, H0)) {
        return false;
    }
    double Ht[9], H1[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += invHnorm[3 * r + k] * H0[3 * k + c];
            Ht[3 * r + c] = s;
        }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += Ht[3 * r + k] * Hnorm2[3 * k + c];
            H1[3 * r + c] = s;
        }
    const double sc = 1. / H1[8];
    for (int i = 0; i < 9; ++i) H[i] = H1[i] * sc;
    return true;
}

bool collinear(const float* p, int count) {   // haveCollinearPoints: last point vs. earlier pairs
    const int i = count - 1;
    for (int j = 0; j < i; ++j) {
        const double dx1 = (double)p[2 * j] - p[2 * i], dy1 = (double)p[2 * j + 1] - p[2 * i + 1];
        for (int k = 0; k < j; ++k) {
            const double dx2 = (double)p[2 * k] - p[2 * i], dy2 = (double)p[2 * k + 1] - p[2 * i + 1];
            if (std::fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (std::fabs(dx1) + std::fabs(dy1) + std::fabs(dx2) + std::fabs(dy2)))
                return true;
        }
    }
    return false;
}

double det3(double a0, double a1, double b0, double b1, double c0, double c1) {
    // Matx33d {a0 a1 1; b0 b1 1; c0 c1 1} determinant by the rule of Sarrus, row 0 expansion
    return a0 * (b1 - c1) - a1 * (b0 - c0) + (b0 * c1 - b1 * c0);
}

bool check_subset(const float* s, const float* d) {
    if (collinear(s, 4) || collinear(d, 4)) return false;
    static const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {1, 3, 0}};
    int negative = 0;
    for (int i = 0; i < 4; ++i) {
        const int* t = tt[i];
        const double dA = det3(s[2 * t[0]], s[2 * t[0] + 1], s[2 * t[1]], s[2 * t[1] + 1], s[2 * t[2]], s[2 * t[2] + 1]);
        const double dB = det3(d[2 * t[0]], d[2 * t[0] + 1], d[2 * t[1]], d[2 * t[1] + 1], d[2 * t[2]], d[2 * t[2] + 1]);
        negative += dA * dB < 0;
    }
    return negative == 0 || negative == 4;
}

int count_inliers(const float* M, const float* m, int count, const double H[9], float thr2) {
    const float h0 = (float)H[0], h1 = (float)H[1], h2 = (float)H[2], h3 = (float)H[3], h4 = (float)H[4],
                h5 = (float)H[5], h6 = (float)H[6], h7 = (float)H[7];
    int nz = 0;
    for (int i = 0; i < count; ++i) {
        const float X = M[2 * i], Y = M[2 * i + 1];
        const float ww = 1.f / (h6 * X + h7 * Y + 1.f);
        const float dx = (h0 * X + h1 * Y + h2) * ww - m[2 * i];
        const float dy = (h3 * X + h4 * Y + h5) * ww - m[2 * i + 1];
        nz += (dx * dx + dy * dy) <= thr2;
    }
    return nz;
}

int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = std::max(p, 0.); p = std::min(p, 1.);
    ep = std::max(ep, 0.); ep = std::min(ep, 1.);
    double num = std::max(1. - p, DBL_MIN);
    const double q = 1. - ep, q2 = q * q;
    double denom = 1. - q2 * q2;           // (1 - ep)^4 for model_points = 4
    (void)model_points;
    if (denom < DBL_MIN) return 0;
    num = std::log(num);
    denom = std::log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)std::lrint(num / denom);
}

// Inlier count of cv::findHomography(..., RANSAC, thr) on `count` aligned
// correspondences; -1 if the homography comes back empty.
int ransac_inliers(const float* M, const float* m, int count, double thr, int max_iters, double confidence) {
    double H[9];
    // findHomography with 4 points: result = runKernel > 0, mask all ones (fundam.cpp); runKernel
    // fails only on zero spread, a degenerate (e.g. collinear) 4-point set still yields ratio 1
    if (count == 4) return dlt(M, m, 4, H, true) ? 4 : -1;
    Rng rng((uint64_t)-1);
    const float thr2 = (float)(thr * thr);
    int niters = std::max(max_iters, 1), max_good = 0;
    float s[8], d[8];
    for (int iter = 0; iter < niters; ++iter) {
        // getSubset (maxAttempts = 10000)
        int attempts = 0, i = 0;
        for (; attempts < 10000; ++attempts) {
            int idx[4];
            for (i = 0; i < 4; ++i) {
                int idx_i, j;
                for (;;) {
                    idx_i = idx[i] = rng.uniform(0, count);
                    for (j = 0; j < i; ++j)
                        if (idx_i == idx[j]) break;
                    if (j == i) break;
                }
                s[2 * i] = M[2 * idx_i]; s[2 * i + 1] = M[2 * idx_i + 1];
                d[2 * i] = m[2 * idx_i]; d[2 * i + 1] = m[2 * idx_i + 1];
            }
            if (!check_subset(s, d)) continue;
            break;
        }
        if (attempts >= 10000) {
            if (iter == 0) return -1;
            break;
        }
        if (!dlt(s, d, 4, H)) continue;
        const int good = count_inliers(M, m, count, H, thr2);
        if (good > std::max(max_good, 3)) {
            max_good = good;
            niters = update_num_iters(confidence, (double)(count - good) / count, 4, niters);
        }
    }
    return max_good > 0 ? max_good : -1;
}

}  // namespace

extern "C" {

// Selects the arithmetic model (1: cv::eigen minimal-sample null vector) for later calls; returns
// the previous flags.  Not thread safe: set it before a call, not during one.
int orc_homography_set_arith(int flags) {
    const int old = g_harith;
    g_harith = flags;
    return old;
}

// Per pair p: matches m[off[p] .. off[p+1]) (sfmx_dmatch / cv::DMatch, 16 B),
// left image pairs[2p], right pairs[2p+1]; kp[i] = image i's keypoints (x, y
// float pairs); size[2i] = width, size[2i+1] = height.  out[p] = inlier ratio
// (-1 for < 4 matches).  OpenMP over pairs (SfM.cpp:603).
int orc_homography_ratios(const float* const* kp, const int32_t* size, const int32_t* pairs, int npairs,
                          const void* matches_v, const int64_t* off, double threshold, int max_iters,
                          double confidence, double* out, int nthreads) {
    struct DM { int32_t q, t, img; float dist; };
    const DM* matches = (const DM*)matches_v;
    const int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
    #pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
    for (int p = 0; p < npairs; ++p) {
        const int L = pairs[2 * p], R = pairs[2 * p + 1];
        const int64_t n = off[p + 1] - off[p];
        if (n < 4) { out[p] = -1.0; continue; }
        std::vector<float> M(2 * n), m(2 * n);
        for (int64_t i = 0; i < n; ++i) {
            const DM& d = matches[off[p] + i];
            M[2 * i] = kp[L][2 * d.q]; M[2 * i + 1] = kp[L][2 * d.q + 1];
            m[2 * i] = kp[R][2 * d.t]; m[2 * i + 1] = kp[R][2 * d.t + 1];
        }
        const double thr = threshold < 0 ? -threshold
                                         : std::max({size[2 * L], size[2 * L + 1], size[2 * R + 1], size[2 * R + 1]}) * threshold;
        const int inl = ransac_inliers(M.data(), m.data(), (int)n, thr, max_iters, confidence);
        out[p] = inl < 0 ? 0.0 : (double)inl / (double)n;
    }
    return 0;
}

}  // extern "C"
