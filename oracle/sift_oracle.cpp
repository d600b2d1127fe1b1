// SPDX-License-Identifier: MIT
// TEST INFRASTRUCTURE ONLY (see oracle/README.md): CPU restatement of the
// reference's feature extraction, SfM::extractFeatures (sfm/SfM.cpp:577-597)
// with cv::SIFT::create(featureLimit, 3, 0.09) (cli/PhotogrammetrieCli.cpp:354):
// OpenCV 4.5.1's SIFT::detectAndCompute (features2d/src/sift.dispatch.cpp +
// sift.simd.hpp; OpenCV is an external dependency absent here), restated from
// its published scalar code paths:
//   createInitialImage   u8 -> float, 2x resize INTER_LINEAR, GaussianBlur(sqrt(sigma^2 - 1))
//   buildGaussianPyramid sig[i] = sqrt((k^i s)^2 - (k^(i-1) s)^2), k = 2^(1/layers);
//                        next octave = INTER_NEAREST half of layer `layers`
//   GaussianBlur (float) getGaussianKernel(cvRound(8 sigma + 1) | 1, CV_32F); row
//                        filter (taps in order) then symmetric column filter,
//                        BORDER_REFLECT_101
//   buildDoGPyramid, findScaleSpaceExtrema (26-neighbour >= / <= test,
//                        threshold floor(0.5 c / layers * 255)), adjustLocalExtrema
//                        (Matx33f::solve = Cramer's rule, 5 steps, contrast and
//                        edge tests), calcOrientationHist (36 bins, 1-4-6-4-1
//                        smoothing, 80 % peaks, parabolic bin), calcSIFTDescriptor
//                        (4 x 4 x 8, trilinear, 0.2 clamp, 512 / norm, saturate_cast<uchar>)
//   KeyPointsFilter::removeDuplicatedSorted, retainBest, firstOctave = -1 rescale.
// Deviations, shared with csrc/sift_features.hip and documented in DESIGN.md:
//   * cv::hal::exp32f / sinf / cosf / powf are replaced by fixed float
//     formulas (sx_expf, sx_sincosf) so that CPU and GPU agree bit for bit;
//     fastAtan2 is OpenCV's own polynomial;
//   * histogram bins accumulate in 2^-30 fixed point (int64, order-free) instead
//     of float in pixel order;
//   * retainBest keeps the response-ranked set in the sorted order of
//     removeDuplicatedSorted (OpenCV's order after nth_element is libstdc++'s).
// Parity against OpenCV itself is unpinned.
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Kp { float x, y, size, angle, response; int32_t octave, class_id; };

constexpr int IMG_BORDER = 5, MAX_INTERP = 5, ORI_BINS = 36, D = 4, NB = 8;
constexpr float ORI_SIG = 1.5f, ORI_RADIUS = 3 * ORI_SIG, ORI_PEAK = 0.8f, DESCR_SCL = 3.f, DESCR_MAG_THR = 0.2f,
                INT_DESCR = 512.f, INIT_SIGMA = 0.5f;
constexpr double FIX = 1073741824.0;   // 2^30

struct Img {
    int w = 0, h = 0;
    std::vector<float> p;
    Img() = default;
    Img(int w_, int h_) : w(w_), h(h_), p((size_t)w_ * h_) {}
    float at(int y, int x) const { return p[(size_t)y * w + x]; }
    float& at(int y, int x) { return p[(size_t)y * w + x]; }
};

int round_f(float v) { return (int)std::nearbyint(v); }      // cvRound(float)
int round_d(double v) { return (int)std::nearbyint(v); }     // cvRound(double)

float sx_expf(float x) {
    if (!(x > -80.f)) return 0.f;
    if (x > 88.f) x = 88.f;
    const float k = std::nearbyint(x * 1.44269504088896341f);
    const float r = (x - k * 0.693145751953125f) - k * 1.42860682030941723e-6f;
    float p = 1.38888889e-3f;
    p = p * r + 8.33333333e-3f;
    p = p * r + 4.16666667e-2f;
    p = p * r + 1.66666667e-1f;
    p = p * r + 0.5f;
    p = p * r + 1.0f;
    p = p * r + 1.0f;
    return std::ldexp(p, (int)k);
}

void sx_sincosf(float a, float* s, float* c) {
    const float q = std::nearbyint(a * 0.636619772367581343f);
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

// cv::fastAtan2 (degrees), OpenCV's polynomial
float atan2_deg(float y, float x) {
    constexpr float R2D = (float)(180 / 3.14159265358979323846);
    constexpr float P1 = 0.9997878412794807f * R2D, P3 = -0.3258083974640975f * R2D, P5 = 0.1555786518463281f * R2D,
                    P7 = -0.04432655554792128f * R2D;
    const float ax = std::fabs(x), ay = std::fabs(y);
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

// ---- OpenCV-arithmetic model (orc_sift_set_arith; measurement only, never the GPU-parity mode) ----
// Bit flags; 0 (the default) is the arithmetic csrc/sift_features.hip shares.  The flags restate
// what OpenCV 4.5.1 itself executes on an x86-64 host whose dispatcher picks the AVX2/FMA3 code
// paths (core mathfuncs_core, imgproc filter, features2d sift are CPU-dispatched):
enum {
    AR_EXP32F = 1,      // cv::hal::exp32f (64-entry 2^(i/64) table x degree-4 polynomial) for the weights
    AR_TRIG = 2,        // libm sinf / cosf (calcSIFTDescriptor calls them directly)
    AR_POWF = 4,        // libm powf(2, (layer + xi) / L) for the keypoint size
    AR_FLOATHIST = 8,   // histogram bins accumulate in float, in pixel order
    AR_FMAVEC = 16,     // FMA3 in the vectorised exp32f / fastAtan2 / magnitude / smoothing / norm
    AR_FMAFILT = 32,    // FMA3 in the separable Gaussian row / column filters
};
int g_arith = 0;

constexpr double EXPPOLY_A0 = .9670371139572337719125840413672004409288e-2;

struct ExpTab {
    float t[64];
    ExpTab() {
        for (int i = 0; i < 64; ++i) t[i] = (float)(std::exp2(i / 64.0) * EXPPOLY_A0);
    }
};
const ExpTab g_exptab;

// cv::hal::exp32f, one element.  fused: the vector body (FMA3 polynomial); else the scalar loop.
float cv_exp32f(float x, bool fused) {
    const float A4 = (float)(1.000000000000002438532970795181890933776 / EXPPOLY_A0),
                A3 = (float)(.6931471805521448196800669615864773144641 / EXPPOLY_A0),
                A2 = (float)(.2402265109513301490103372422686535526573 / EXPPOLY_A0),
                A1 = (float)(.5550339366753125211915322047004666939128e-1 / EXPPOLY_A0);
    const double prescale = 1.4426950408889634073599246810019 * 64, maxv = 3000. * 64;
    const float minval = (float)(-maxv / prescale), maxval = (float)(maxv / prescale);
    float x0 = std::min(std::max(x, minval), maxval) * (float)prescale;
    const int xi = (int)std::nearbyint(x0);
    x0 = (x0 - (float)xi) * (float)(1. / 64);
    int t = (xi >> 6) + 127;
    t = !(t & ~255) ? t : t < 0 ? 0 : 255;
    uint32_t bits = (uint32_t)t << 23;
    float p2;
    std::memcpy(&p2, &bits, 4);
    float poly;
    if (fused) poly = std::fma(std::fma(std::fma(x0 + A1, x0, A2), x0, A3), x0, A4);
    else poly = (((x0 + A1) * x0 + A2) * x0 + A3) * x0 + A4;
    return p2 * g_exptab.t[xi & 63] * poly;
}

// exp of element k of an in-place exp32f over len elements (the AVX2 body covers whole 16-element
// blocks; an in-place call finishes the rest in the scalar loop)
float weight_exp(float x, int k, int len) {
    if (!(g_arith & AR_EXP32F)) return sx_expf(x);
    return cv_exp32f(x, (g_arith & AR_FMAVEC) && k < (len / 16) * 16);
}

// fastAtan2 / magnitude32f of one element of a len-element (not in-place) call: len >= 16 runs the
// vector body for every element (the last block overlaps), FMA3 polynomial / x*x + y*y
float ori_deg(float y, float x, int len) {
    if (!((g_arith & AR_FMAVEC) && len >= 16)) return atan2_deg(y, x);
    constexpr float R2D = (float)(180 / 3.14159265358979323846);
    constexpr float P1 = 0.9997878412794807f * R2D, P3 = -0.3258083974640975f * R2D, P5 = 0.1555786518463281f * R2D,
                    P7 = -0.04432655554792128f * R2D;
    const float ax = std::fabs(x), ay = std::fabs(y);
    const float c = std::min(ax, ay) / (std::max(ax, ay) + (float)DBL_EPSILON);
    const float cc = c * c;
    float a = std::fma(std::fma(std::fma(cc, P7, P5), cc, P3), cc, P1) * c;
    if (!(ax >= ay)) a = 90.f - a;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

float magnitude(float dx, float dy, int len) {
    if ((g_arith & AR_FMAVEC) && len >= 16) return std::sqrt(std::fma(dx, dx, dy * dy));
    return std::sqrt(dx * dx + dy * dy);
}

int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

// getGaussianKernel(cvRound(sigma * 4 * 2 + 1) | 1, sigma, CV_32F)
std::vector<float> gauss_kernel(double sigma) {
    const int n = round_d(sigma * 4 * 2 + 1) | 1;
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

Img blur(const Img& src, double sigma) {
    const std::vector<float> f = gauss_kernel(sigma);
    const int n = (int)f.size(), r = n / 2;
    Img tmp(src.w, src.h), dst(src.w, src.h);
    const bool fused = g_arith & AR_FMAFILT;
    for (int y = 0; y < src.h; ++y)
        for (int x = 0; x < src.w; ++x) {
            float s = f[0] * src.at(y, reflect101(x - r, src.w));
            for (int k = 1; k < n; ++k) {
                const float v = src.at(y, reflect101(x - r + k, src.w));
                s = fused ? std::fma(v, f[k], s) : s + f[k] * v;
            }
            tmp.at(y, x) = s;
        }
    for (int y = 0; y < src.h; ++y)
        for (int x = 0; x < src.w; ++x) {
            float s = f[r] * tmp.at(y, x);
            for (int k = 1; k <= r; ++k) {
                const float v = tmp.at(reflect101(y + k, src.h), x) + tmp.at(reflect101(y - k, src.h), x);
                s = fused ? std::fma(v, f[r + k], s) : s + f[r + k] * v;
            }
            dst.at(y, x) = s;
        }
    return dst;
}

// resize(src, 2x, INTER_LINEAR) on float: horizontal then vertical pass
void lin_coef(int d, int ssize, int& s, float& f0, float& f1) {
    float fx = (float)((d + 0.5) * 0.5 - 0.5);
    int sx = (int)std::floor(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx >= ssize - 1) { fx = 0; sx = ssize - 1; }
    s = sx;
    f0 = 1.f - fx;
    f1 = fx;
}

Img upsample2(const Img& src) {
    Img dst(src.w * 2, src.h * 2);
    for (int Y = 0; Y < dst.h; ++Y) {
        int sy; float b0, b1;
        lin_coef(Y, src.h, sy, b0, b1);
        const int sy1 = std::min(sy + 1, src.h - 1);
        for (int X = 0; X < dst.w; ++X) {
            int sx; float a0, a1;
            lin_coef(X, src.w, sx, a0, a1);
            const int sx1 = std::min(sx + 1, src.w - 1);
            const float h0 = src.at(sy, sx) * a0 + src.at(sy, sx1) * a1;
            const float h1 = src.at(sy1, sx) * a0 + src.at(sy1, sx1) * a1;
            dst.at(Y, X) = h0 * b0 + h1 * b1;
        }
    }
    return dst;
}

Img half_nn(const Img& src) {
    Img dst(src.w / 2, src.h / 2);
    const double ifx = 1. / ((double)dst.w / src.w), ify = 1. / ((double)dst.h / src.h);
    for (int y = 0; y < dst.h; ++y) {
        const int sy = std::min((int)std::floor(y * ify), src.h - 1);
        for (int x = 0; x < dst.w; ++x) dst.at(y, x) = src.at(sy, std::min((int)std::floor(x * ifx), src.w - 1));
    }
    return dst;
}

struct Refined { int o, layer, r, c; Kp kp; };

bool adjust(const std::vector<Img>& dog, int L, Kp& kpt, int octv, int& layer, int& r, int& c, float contrastThreshold,
            float edgeThreshold, float sigma) {
    const float img_scale = 1.f / 255, deriv_scale = img_scale * 0.5f, second_deriv_scale = img_scale,
                cross_deriv_scale = img_scale * 0.25f;
    float xi = 0, xr = 0, xc = 0, contr = 0;
    int i = 0;
    for (; i < MAX_INTERP; i++) {
        const int idx = octv * (L + 2) + layer;
        const Img &img = dog[idx], &prev = dog[idx - 1], &next = dog[idx + 1];
        const float d0 = (img.at(r, c + 1) - img.at(r, c - 1)) * deriv_scale;
        const float d1 = (img.at(r + 1, c) - img.at(r - 1, c)) * deriv_scale;
        const float d2 = (next.at(r, c) - prev.at(r, c)) * deriv_scale;
        const float v2 = img.at(r, c) * 2;
        const float dxx = (img.at(r, c + 1) + img.at(r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (img.at(r + 1, c) + img.at(r - 1, c) - v2) * second_deriv_scale;
        const float dss = (next.at(r, c) + prev.at(r, c) - v2) * second_deriv_scale;
        const float dxy = (img.at(r + 1, c + 1) - img.at(r + 1, c - 1) - img.at(r - 1, c + 1) + img.at(r - 1, c - 1)) *
                          cross_deriv_scale;
        const float dxs = (next.at(r, c + 1) - next.at(r, c - 1) - prev.at(r, c + 1) + prev.at(r, c - 1)) * cross_deriv_scale;
        const float dys = (next.at(r + 1, c) - next.at(r - 1, c) - prev.at(r + 1, c) + prev.at(r - 1, c)) * cross_deriv_scale;
        // Matx33f H(dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss); X = H.solve(dD) (Cramer, zeros if singular)
        const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs, a21 = dys, a22 = dss;
        float x0 = 0, x1 = 0, x2 = 0;
        float det = (float)(double)(a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11));
        if (det != 0) {
            det = 1 / det;
            x0 = det * (d0 * (a11 * a22 - a12 * a21) - a01 * (d1 * a22 - a12 * d2) + a02 * (d1 * a21 - a11 * d2));
            x1 = det * (a00 * (d1 * a22 - a12 * d2) - d0 * (a10 * a22 - a12 * a20) + a02 * (a10 * d2 - d1 * a20));
            x2 = det * (a00 * (a11 * d2 - d1 * a21) - a01 * (a10 * d2 - d1 * a20) + d0 * (a10 * a21 - a11 * a20));
        }
        xi = -x2; xr = -x1; xc = -x0;
        if (std::fabs(xi) < 0.5f && std::fabs(xr) < 0.5f && std::fabs(xc) < 0.5f) break;
        if (std::fabs(xi) > (float)(INT_MAX / 3) || std::fabs(xr) > (float)(INT_MAX / 3) || std::fabs(xc) > (float)(INT_MAX / 3))
            return false;
        c += round_f(xc);
        r += round_f(xr);
        layer += round_f(xi);
        if (layer < 1 || layer > L || c < IMG_BORDER || c >= img.w - IMG_BORDER || r < IMG_BORDER || r >= img.h - IMG_BORDER)
            return false;
    }
    if (i >= MAX_INTERP) return false;
    {
        const int idx = octv * (L + 2) + layer;
        const Img &img = dog[idx], &prev = dog[idx - 1], &next = dog[idx + 1];
        const float d0 = (img.at(r, c + 1) - img.at(r, c - 1)) * deriv_scale;
        const float d1 = (img.at(r + 1, c) - img.at(r - 1, c)) * deriv_scale;
        const float d2 = (next.at(r, c) - prev.at(r, c)) * deriv_scale;
        float t = 0;
        t += d0 * xc;
        t += d1 * xr;
        t += d2 * xi;
        contr = img.at(r, c) * img_scale + t * 0.5f;
        if (std::fabs(contr) * L < contrastThreshold) return false;
        const float v2 = img.at(r, c) * 2.f;
        const float dxx = (img.at(r, c + 1) + img.at(r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (img.at(r + 1, c) + img.at(r - 1, c) - v2) * second_deriv_scale;
        const float dxy = (img.at(r + 1, c + 1) - img.at(r + 1, c - 1) - img.at(r - 1, c + 1) + img.at(r - 1, c - 1)) *
                          cross_deriv_scale;
        const float tr = dxx + dyy;
        const float det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * edgeThreshold >= (edgeThreshold + 1) * (edgeThreshold + 1) * det) return false;
    }
    kpt.x = (c + xc) * (1 << octv);
    kpt.y = (r + xr) * (1 << octv);
    kpt.octave = octv + (layer << 8) + (round_d((xi + 0.5) * 255) << 16);
    kpt.size = sigma *
               ((g_arith & AR_POWF) ? std::pow(2.f, (layer + xi) / L) : sx_expf(((layer + xi) / L) * 0.693147180559945309f)) *
               (1 << octv) * 2;
    kpt.response = std::fabs(contr);
    kpt.angle = -1;
    kpt.class_id = -1;
    return true;
}

float orientation_hist(const Img& img, int px, int py, int radius, float sigma, float* hist) {
    const int n = ORI_BINS;
    const float expf_scale = -1.f / (2.f * sigma * sigma);
    // the window's samples in pixel order (calcOrientationHist's X / Y / W arrays)
    struct S { float dx, dy, w; };
    std::vector<S> smp;
    smp.reserve((size_t)(2 * radius + 1) * (2 * radius + 1));
    for (int i = -radius; i <= radius; i++) {
        const int y = py + i;
        if (y <= 0 || y >= img.h - 1) continue;
        for (int j = -radius; j <= radius; j++) {
            const int x = px + j;
            if (x <= 0 || x >= img.w - 1) continue;
            smp.push_back({img.at(y, x + 1) - img.at(y, x - 1), img.at(y - 1, x) - img.at(y + 1, x), (i * i + j * j) * expf_scale});
        }
    }
    const int len = (int)smp.size();
    int64_t acc[ORI_BINS] = {0};
    float t[ORI_BINS + 4] = {0};
    float* temphist = t + 2;
    for (int k = 0; k < len; ++k) {
        const float w = weight_exp(smp[k].w, k, len);
        const float ori = ori_deg(smp[k].dy, smp[k].dx, len);
        const float mag = magnitude(smp[k].dx, smp[k].dy, len);
        int bin = round_f((n / 360.f) * ori);
        if (bin >= n) bin -= n;
        if (bin < 0) bin += n;
        if (g_arith & AR_FLOATHIST) temphist[bin] += w * mag;
        else acc[bin] += (int64_t)(w * mag * 1073741824.f);
    }
    if (!(g_arith & AR_FLOATHIST))
        for (int b = 0; b < n; ++b) temphist[b] = (float)((double)acc[b] * (1.0 / FIX));
    temphist[-1] = temphist[n - 1];
    temphist[-2] = temphist[n - 2];
    temphist[n] = temphist[0];
    temphist[n + 1] = temphist[1];
    for (int b = 0; b < n; b++) {
        const float tn2 = temphist[b - 2] + temphist[b + 2], tn1 = temphist[b - 1] + temphist[b + 1];
        if ((g_arith & AR_FMAVEC) && b < (n / 8) * 8)   // the 8-lane body: fma(tn2, 1/16, fma(tn1, 4/16, t0 * 6/16))
            hist[b] = std::fma(tn2, 1.f / 16.f, std::fma(tn1, 4.f / 16.f, temphist[b] * (6.f / 16.f)));
        else
            hist[b] = tn2 * (1.f / 16.f) + tn1 * (4.f / 16.f) + temphist[b] * (6.f / 16.f);
    }
    float maxval = hist[0];
    for (int b = 1; b < n; b++) maxval = std::max(maxval, hist[b]);
    return maxval;
}

void descriptor(const Img& img, float ptx, float pty, float ori, float scl, float* dst) {
    const int d = D, n = NB;
    const int ptX = round_f(ptx), ptY = round_f(pty);
    float sin_t, cos_t;
    if (g_arith & AR_TRIG) {
        cos_t = std::cos(ori * (float)(3.14159265358979323846 / 180));
        sin_t = std::sin(ori * (float)(3.14159265358979323846 / 180));
    } else {
        sx_sincosf(ori * (float)(3.14159265358979323846 / 180), &sin_t, &cos_t);
    }
    const float bins_per_rad = n / 360.f;
    const float exp_scale = -1.f / (d * d * 0.5f);
    const float hist_width = DESCR_SCL * scl;
    int radius = round_f(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
    radius = std::min(radius, (int)std::sqrt(((double)img.w) * img.w + ((double)img.h) * img.h));
    cos_t /= hist_width;
    sin_t /= hist_width;
    // the window's samples in pixel order (calcSIFTDescriptor's X / Y / RBin / CBin / W arrays)
    struct S { float dx, dy, rbin, cbin, w; };
    std::vector<S> smp;
    smp.reserve((size_t)(2 * radius + 1) * (2 * radius + 1));
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            const float c_rot = j * cos_t - i * sin_t;
            const float r_rot = j * sin_t + i * cos_t;
            const float rbin = r_rot + d / 2 - 0.5f;
            const float cbin = c_rot + d / 2 - 0.5f;
            const int r = ptY + i, c = ptX + j;
            if (!(rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < img.h - 1 && c > 0 && c < img.w - 1))
                continue;
            smp.push_back({img.at(r, c + 1) - img.at(r, c - 1), img.at(r - 1, c) - img.at(r + 1, c), rbin, cbin,
                           (c_rot * c_rot + r_rot * r_rot) * exp_scale});
        }
    const int len_s = (int)smp.size();
    const bool fhist = g_arith & AR_FLOATHIST;
    int64_t hist[(D + 2) * (D + 2) * (NB + 2)] = {0};
    float fh[(D + 2) * (D + 2) * (NB + 2)] = {0};
    for (int k = 0; k < len_s; ++k) {
        {
            const float dx = smp[k].dx, dy = smp[k].dy;
            float rbin = smp[k].rbin, cbin = smp[k].cbin;
            const float w = weight_exp(smp[k].w, k, len_s);
            const float o = ori_deg(dy, dx, len_s);
            const float m = magnitude(dx, dy, len_s);
            float obin = (o - ori) * bins_per_rad;
            const float mag = m * w;
            const int r0 = (int)std::floor(rbin), c0 = (int)std::floor(cbin);
            int o0 = (int)std::floor(obin);
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
            const int tgt[8] = {idx, idx + 1, idx + (n + 2), idx + (n + 3), idx + (d + 2) * (n + 2),
                                idx + (d + 2) * (n + 2) + 1, idx + (d + 3) * (n + 2), idx + (d + 3) * (n + 2) + 1};
            const float val[8] = {v_rco000, v_rco001, v_rco010, v_rco011, v_rco100, v_rco101, v_rco110, v_rco111};
            for (int q = 0; q < 8; ++q) {
                if (fhist) fh[tgt[q]] += val[q];
                else hist[tgt[q]] += (int64_t)(val[q] * 1073741824.f);
            }
        }
    }
    for (int i = 0; i < d; i++)
        for (int j = 0; j < d; j++) {
            const int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
            if (fhist) {
                fh[idx] += fh[idx + n];
                fh[idx + 1] += fh[idx + n + 1];
                for (int k = 0; k < n; k++) dst[(i * d + j) * n + k] = fh[idx + k];
            } else {
                hist[idx] += hist[idx + n];
                hist[idx + 1] += hist[idx + n + 1];
                for (int k = 0; k < n; k++) dst[(i * d + j) * n + k] = (float)((double)hist[idx + k] * (1.0 / FIX));
            }
        }
    const int len = d * d * n;
    float nrm2 = 0;
    if (g_arith & AR_FMAVEC) {   // 8-lane fma accumulation, then v_reduce_sum ((l0+l4)+(l1+l5)) + ((l2+l6)+(l3+l7))
        float lane[8] = {0};
        for (int k = 0; k < len; k++) lane[k & 7] = std::fma(dst[k], dst[k], lane[k & 7]);
        const float s0 = lane[0] + lane[4], s1 = lane[1] + lane[5], s2 = lane[2] + lane[6], s3 = lane[3] + lane[7];
        nrm2 = (s0 + s1) + (s2 + s3);
    } else {
        for (int k = 0; k < len; k++) nrm2 += dst[k] * dst[k];
    }
    const float thr = std::sqrt(nrm2) * DESCR_MAG_THR;
    nrm2 = 0;
    for (int k = 0; k < len; k++) {
        const float val = std::min(dst[k], thr);
        dst[k] = val;
        nrm2 += val * val;
    }
    nrm2 = INT_DESCR / std::max(std::sqrt(nrm2), FLT_EPSILON);
    for (int k = 0; k < len; k++) dst[k] = (float)std::min(std::max(round_f(dst[k] * nrm2), 0), 255);
}

bool kp_less(const Kp& a, const Kp& b) {   // KeyPointsFilter::removeDuplicatedSorted's order
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle < b.angle;
    if (a.response != b.response) return a.response > b.response;
    if (a.octave != b.octave) return a.octave > b.octave;
    return a.class_id > b.class_id;
}

}  // namespace

extern "C" {

// Selects the arithmetic model (AR_* flags above) for later orc_sift / orc_sift_batch calls;
// returns the previous flags.  Not thread safe: set it before a call, not during one.
int orc_sift_set_arith(int flags) {
    const int old = g_arith;
    g_arith = flags;
    return old;
}

// SIFT::detectAndCompute restated; returns the keypoint count n (writes min(n, cap)).
int orc_sift(const uint8_t* image, int W, int H, int64_t pitch, int nfeatures, int L, double contrastThreshold,
             double edgeThreshold, double sigma_d, void* kps_out, float* desc_out, int cap) {
    const int firstOctave = -1;
    const float sigma = (float)sigma_d;
    Img gray(W, H);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) gray.at(y, x) = (float)image[y * pitch + x];
    const float sig_diff = std::sqrt(std::max(sigma * sigma - INIT_SIGMA * INIT_SIGMA * 4, 0.01f));
    const Img base = blur(upsample2(gray), sig_diff);
    const int nOct = round_d(std::log((double)std::min(base.w, base.h)) / std::log(2.) - 2) - firstOctave;
    std::vector<double> sig(L + 3);
    sig[0] = sigma;
    const double k = std::pow(2., 1. / L);
    for (int i = 1; i < L + 3; i++) {
        const double sig_prev = std::pow(k, (double)(i - 1)) * sigma;
        const double sig_total = sig_prev * k;
        sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
    std::vector<Img> gp((size_t)nOct * (L + 3)), dog((size_t)nOct * (L + 2));
    for (int o = 0; o < nOct; o++)
        for (int i = 0; i < L + 3; i++) {
            Img& dst = gp[o * (L + 3) + i];
            if (o == 0 && i == 0) dst = base;
            else if (i == 0) dst = half_nn(gp[(o - 1) * (L + 3) + L]);
            else dst = blur(gp[o * (L + 3) + i - 1], sig[i]);
        }
    for (int o = 0; o < nOct; o++)
        for (int i = 0; i < L + 2; i++) {
            const Img &a = gp[o * (L + 3) + i], &b = gp[o * (L + 3) + i + 1];
            Img& d = dog[o * (L + 2) + i];
            d = Img(a.w, a.h);
            for (size_t q = 0; q < d.p.size(); ++q) d.p[q] = b.p[q] - a.p[q];
        }
    const int threshold = (int)std::floor(0.5 * contrastThreshold / L * 255);
    std::vector<Kp> kps;
    for (int o = 0; o < nOct; o++)
        for (int i = 1; i <= L; i++) {
            const Img &img = dog[o * (L + 2) + i], &prev = dog[o * (L + 2) + i - 1], &next = dog[o * (L + 2) + i + 1];
            for (int r = IMG_BORDER; r < img.h - IMG_BORDER; r++)
                for (int c = IMG_BORDER; c < img.w - IMG_BORDER; c++) {
                    const float val = img.at(r, c);
                    if (!(std::fabs(val) > threshold)) continue;
                    bool mx = val > 0, mn = val < 0;
                    for (int dy = -1; dy <= 1; ++dy)
                        for (int dx = -1; dx <= 1; ++dx) {
                            const float a = img.at(r + dy, c + dx), b = prev.at(r + dy, c + dx), e = next.at(r + dy, c + dx);
                            mx = mx && val >= a && val >= b && val >= e;
                            mn = mn && val <= a && val <= b && val <= e;
                        }
                    if (!mx && !mn) continue;
                    int r1 = r, c1 = c, layer = i;
                    Kp kpt;
                    if (!adjust(dog, L, kpt, o, layer, r1, c1, (float)contrastThreshold, (float)edgeThreshold, sigma)) continue;
                    const float scl_octv = kpt.size * 0.5f / (1 << o);
                    float hist[ORI_BINS];
                    const float omax = orientation_hist(gp[o * (L + 3) + layer], c1, r1, round_f(ORI_RADIUS * scl_octv),
                                                        ORI_SIG * scl_octv, hist);
                    const float mag_thr = omax * ORI_PEAK;
                    for (int j = 0; j < ORI_BINS; j++) {
                        const int l = j > 0 ? j - 1 : ORI_BINS - 1, r2 = j < ORI_BINS - 1 ? j + 1 : 0;
                        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
                            float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
                            bin = bin < 0 ? ORI_BINS + bin : bin >= ORI_BINS ? bin - ORI_BINS : bin;
                            kpt.angle = 360.f - (float)((360.f / ORI_BINS) * bin);
                            if (std::fabs(kpt.angle - 360.f) < FLT_EPSILON) kpt.angle = 0.f;
                            kps.push_back(kpt);
                        }
                    }
                }
        }
    // removeDuplicatedSorted, retainBest, firstOctave rescale
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
    // KeypointResponseGreater, then std::partition of the tail by response >= the boundary response.
    // Both reorder the kept keypoints in place; the descriptor rows follow that order.
    if (nfeatures > 0 && (int)kps.size() > nfeatures) {
        std::nth_element(kps.begin(), kps.begin() + nfeatures - 1, kps.end(),
                         [](const Kp& a, const Kp& b) { return a.response > b.response; });
        const float amb = kps[nfeatures - 1].response;
        auto new_end = std::partition(kps.begin() + nfeatures, kps.end(), [amb](const Kp& q) { return q.response >= amb; });
        kps.resize(new_end - kps.begin());
    }
    for (Kp& q : kps) {
        q.octave = (q.octave & ~255) | ((q.octave + firstOctave) & 255);
        q.x *= 0.5f;
        q.y *= 0.5f;
        q.size *= 0.5f;
    }
    // SfM.cpp:586-587 calls detect() and compute() separately. compute() (useProvidedKeypoints) rebuilds the
    // pyramid from firstOctave = min(0, min keypoint octave) with maxOctave - firstOctave + 1 octaves, so when
    // no kept keypoint comes from the upsampled octave the descriptors are taken from an un-doubled pyramid.
    int cFirst = 0, cMaxOct = INT_MIN;
    for (const Kp& q : kps) {
        int o = q.octave & 255;
        o = o < 128 ? o : (-128 | o);
        cFirst = std::min(cFirst, o);
        cMaxOct = std::max(cMaxOct, o);
    }
    std::vector<Img> gp0;
    if (!kps.empty() && cFirst == 0 && desc_out) {
        const float sd0 = std::sqrt(std::max(sigma * sigma - INIT_SIGMA * INIT_SIGMA, 0.01f));
        const int nOc = cMaxOct + 1;
        gp0.resize((size_t)nOc * (L + 3));
        for (int o = 0; o < nOc; o++)
            for (int i = 0; i < L + 3; i++) {
                Img& dst = gp0[o * (L + 3) + i];
                if (o == 0 && i == 0) dst = blur(gray, sd0);
                else if (i == 0) dst = half_nn(gp0[(o - 1) * (L + 3) + L]);
                else dst = blur(gp0[o * (L + 3) + i - 1], sig[i]);
            }
    }
    const std::vector<Img>& dgp = gp0.empty() ? gp : gp0;
    const int dFirst = gp0.empty() ? firstOctave : 0;
    const int n = (int)kps.size();
    Kp* out = static_cast<Kp*>(kps_out);
    for (int q = 0; q < n && q < cap; ++q) {
        out[q] = kps[q];
        if (!desc_out) continue;
        int octave = kps[q].octave & 255, layer = (kps[q].octave >> 8) & 255;
        octave = octave < 128 ? octave : (-128 | octave);
        const float scale = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
        const float size = kps[q].size * scale;
        const Img& img = dgp[(octave - dFirst) * (L + 3) + layer];
        float angle = 360.f - kps[q].angle;
        if (std::fabs(angle - 360.f) < FLT_EPSILON) angle = 0.f;
        descriptor(img, kps[q].x * scale, kps[q].y * scale, angle, size * 0.5f, desc_out + (size_t)q * 128);
    }
    return n;
}

}  // extern "C"

extern "C" {
// orc_sift over a batch of equally sized images, OpenMP over images (as the
// reference's omp loop over shots, SfM.cpp:582); `cap` keypoint / descriptor
// rows per image, counts in n_out.
void orc_sift_batch(const uint8_t* const* images, int n_images, int W, int H, int nfeatures, int L,
                    double contrastThreshold, double edgeThreshold, double sigma, void* kps_out, float* desc_out,
                    int cap, int* n_out, int nthreads) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int i = 0; i < n_images; ++i)
        n_out[i] = orc_sift(images[i], W, H, W, nfeatures, L, contrastThreshold, edgeThreshold, sigma,
                            static_cast<char*>(kps_out) + (size_t)i * cap * 28,
                            desc_out ? desc_out + (size_t)i * cap * 128 : nullptr, cap);
}
}  // extern "C"
