// SPDX-License-Identifier: MIT
//
// sfmx ORACLE — TEST INFRASTRUCTURE ONLY (bundle adjustment).
//
// CPU restatement of the reference's bundle adjustment: the problem built by
// BundleAdjustment::doBundleAdjustment (src/photogrammetrie/common/BundleAdjustment.cpp:29-91)
// and solved by CeresUtils::solve (util/CeresUtils.cpp:38-56) with
//   linear_solver_type = DENSE_SCHUR, max_num_iterations = 5000 (:43-50)
// and every other option at its Ceres 1.14 default [ext]:
//   TRUST_REGION + LEVENBERG_MARQUARDT, initial radius 1e4, max 1e16, min 1e-32,
//   min/max LM diagonal 1e-6 / 1e32, min_relative_decrease 1e-3,
//   function/gradient/parameter tolerance 1e-6 / 1e-10 / 1e-8, jacobi_scaling,
//   max_num_consecutive_invalid_steps 5, monotonic steps, squared loss.
// Residuals: the reference's three templated functors, differentiated the way
// ceres::AutoDiffCostFunction does it (forward-mode dual numbers, "Jets"):
//   SimpleRadialCameraCostFunction  common/SimpleRadialCamera.cpp:69-115
//   SimpleCameraCostFunction        common/SimpleCamera.cpp:63-103
//   DistortionCameraCostFunction    common/DistortionCamera.cpp:62-110
// ceres::AngleAxisRotatePoint restated from Ceres 1.14 rotation.h [ext].
// Linear solve: Schur complement of the 3-dof point blocks, dense reduced
// camera system (6C + k)^2, Cholesky (Eigen LLT in Ceres), back-substitution.
// Trust-region loop: Ceres 1.14 trust_region_minimizer.cc / levenberg_marquardt_strategy.cc [ext].
//
// Parity status: unpinned against Ceres itself (not installed, no network);
// pinned by noise-free problems (cost -> 0, known optimum) and by the
// GPU-vs-oracle final-cost tolerance 1e-5 relative (north_star).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>
#include <omp.h>

namespace {

// ---- forward-mode dual numbers (ceres::Jet semantics) --------------------
template <int N>
struct Jet {
    double a;
    double v[N];
    Jet() : a(0) { for (int i = 0; i < N; ++i) v[i] = 0; }
    explicit Jet(double x) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; }
    Jet(double x, int k) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; v[k] = 1.0; }
};
template <int N> Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) { Jet<N> r; r.a = f.a + g.a; for (int i = 0; i < N; ++i) r.v[i] = f.v[i] + g.v[i]; return r; }
template <int N> Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) { Jet<N> r; r.a = f.a - g.a; for (int i = 0; i < N; ++i) r.v[i] = f.v[i] - g.v[i]; return r; }
template <int N> Jet<N> operator-(const Jet<N>& f) { Jet<N> r; r.a = -f.a; for (int i = 0; i < N; ++i) r.v[i] = -f.v[i]; return r; }
template <int N> Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) { Jet<N> r; r.a = f.a * g.a; for (int i = 0; i < N; ++i) r.v[i] = f.a * g.v[i] + f.v[i] * g.a; return r; }
template <int N> Jet<N> operator*(double s, const Jet<N>& f) { Jet<N> r; r.a = s * f.a; for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i]; return r; }
template <int N> Jet<N> operator*(const Jet<N>& f, double s) { return s * f; }
template <int N> Jet<N> operator+(const Jet<N>& f, double s) { Jet<N> r = f; r.a += s; return r; }
template <int N> Jet<N> operator-(double s, const Jet<N>& f) { Jet<N> r = -f; r.a += s; return r; }
template <int N> Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {
    const double gi = 1.0 / g.a, fg = f.a * gi;
    Jet<N> r; r.a = f.a * gi;
    for (int i = 0; i < N; ++i) r.v[i] = (f.v[i] - fg * g.v[i]) * gi;
    return r;
}
template <int N> Jet<N> sqrt(const Jet<N>& f) {
    const double s = std::sqrt(f.a), t = 1.0 / (2.0 * s);
    Jet<N> r; r.a = s; for (int i = 0; i < N; ++i) r.v[i] = t * f.v[i]; return r;
}
template <int N> Jet<N> cos(const Jet<N>& f) {
    const double s = -std::sin(f.a);
    Jet<N> r; r.a = std::cos(f.a); for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i]; return r;
}
template <int N> Jet<N> sin(const Jet<N>& f) {
    const double c = std::cos(f.a);
    Jet<N> r; r.a = std::sin(f.a); for (int i = 0; i < N; ++i) r.v[i] = c * f.v[i]; return r;
}
inline double scalar(double x) { return x; }
template <int N> double scalar(const Jet<N>& x) { return x.a; }

using std::sqrt; using std::sin; using std::cos;

// ceres::AngleAxisRotatePoint (rotation.h, Ceres 1.14) [ext]
template <typename T>
void angle_axis_rotate_point(const T aa[3], const T pt[3], T result[3]) {
    const T theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
    if (scalar(theta2) > std::numeric_limits<double>::epsilon()) {
        const T theta = sqrt(theta2);
        const T costheta = cos(theta);
        const T sintheta = sin(theta);
        const T theta_inverse = T(1.0) / theta;
        const T w[3] = {aa[0] * theta_inverse, aa[1] * theta_inverse, aa[2] * theta_inverse};
        const T wx[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
        const T tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (T(1.0) - costheta);
        for (int i = 0; i < 3; ++i) result[i] = pt[i] * costheta + wx[i] * sintheta + w[i] * tmp;
    } else {
        const T wx[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]};
        for (int i = 0; i < 3; ++i) result[i] = pt[i] + wx[i];
    }
}

enum { CAM_SIMPLE = 1, CAM_SIMPLE_RADIAL = 3, CAM_DISTORTION = 7 };

// The reference functors (operator() bodies restated, same operation order).
template <int K, typename T>
void residual(const T* X, const T* pose, const T* intr, double ox, double oy, double cx, double cy, T* res) {
    T p[3];
    angle_axis_rotate_point(pose, X, p);
    p[0] = p[0] + pose[3]; p[1] = p[1] + pose[4]; p[2] = p[2] + pose[5];
    const T xp = p[0] / p[2];
    const T yp = p[1] / p[2];
    const T& focal = intr[0];
    const T xd = focal * xp;
    const T yd = focal * yp;
    if constexpr (K == CAM_SIMPLE) {
        res[0] = xd - T(ox - cx);
        res[1] = yd - T(oy - cy);
    } else if constexpr (K == CAM_SIMPLE_RADIAL) {
        const T& k1 = intr[1]; const T& k2 = intr[2];
        const T r2 = (xp * xp) + (yp * yp);
        const T r4 = r2 * r2;
        const T xu = xd + xd * (k1 * r2 + k2 * r4);
        const T yu = yd + yd * (k1 * r2 + k2 * r4);
        res[0] = xu - (T(ox) - T(cx));
        res[1] = yu - (T(oy) - T(cy));
    } else {   // Distortion: [f, cx, cy, k1, k2, p1, p2]
        const T& k1 = intr[3]; const T& k2 = intr[4]; const T& p1 = intr[5]; const T& p2 = intr[6];
        const T r2 = (xp * xp) + (yp * yp);
        const T r4 = r2 * r2;
        const T xu = xd + xd * (k1 * r2 + k2 * r4) + (p1 * (r2 + 2.0 * (xd * xd)) + 2.0 * p2 * xd * yd);
        const T yu = yd + yd * (k1 * r2 + k2 * r4) + (2.0 * p1 * xd * yd + p2 * (r2 + 2.0 * (yd * yd)));
        res[0] = xu - (T(ox) - intr[1]);
        res[1] = yu - (T(oy) - intr[2]);
    }
}

template <int K>
void eval_jet(const double* X, const double* pose, const double* intr, double ox, double oy, double cx,
              double cy, double* r, double* Je, double* Jc, double* Ji) {
    constexpr int N = 9 + K;
    Jet<N> x[3], ps[6], in[K], res[2];
    for (int i = 0; i < 3; ++i) x[i] = Jet<N>(X[i], i);
    for (int i = 0; i < 6; ++i) ps[i] = Jet<N>(pose[i], 3 + i);
    for (int i = 0; i < K; ++i) in[i] = Jet<N>(intr[i], 9 + i);
    residual<K>(x, ps, in, ox, oy, cx, cy, res);
    for (int j = 0; j < 2; ++j) {
        r[j] = res[j].a;
        for (int i = 0; i < 3; ++i) Je[j * 3 + i] = res[j].v[i];
        for (int i = 0; i < 6; ++i) Jc[j * 6 + i] = res[j].v[3 + i];
        for (int i = 0; i < K; ++i) Ji[j * K + i] = res[j].v[9 + i];
    }
}

// The problem the reference builds (BundleAdjustment.cpp:45-91): every shot's residuals use
// ITS camera's intrinsics block (shot->getCamera(), :81-89), so per pose c: the camera's
// model k_c, the first column of its block among the intrinsics parameters of x, and the
// principal point the SIMPLE / SIMPLE_RADIAL functors capture (getCenter, :83 ->
// SimpleRadialCamera.cpp:118-124).  x = [points 3P | poses 6C | intrinsics kt]: the blocks some
// residual references, in camera order (Ceres knows only blocks AddResidualBlock named).
struct Problem {
    int P, C, O, kt;
    const int32_t* obs_point;
    const int32_t* obs_cam;
    const double* obs_xy;
    std::vector<int> cmodel, coff;      // per pose
    std::vector<double> ccx, ccy;       // per pose
    std::vector<int> isrc;              // intrinsics column j of x <- caller intr[isrc[j]]
};

constexpr int KMAX = 7;   // Ji rows are stored KMAX wide per observation, the first k_c used

struct Lin {   // linearisation at x: residuals + Jacobian blocks per observation
    std::vector<double> r, Je, Jc, Ji;
};

void residual_of(const Problem& pb, int c, const double* X, const double* ps, const double* intr, double ox, double oy,
                 double* res) {
    const double* in = intr + pb.coff[c];
    if (pb.cmodel[c] == 1) residual<1>(X, ps, in, ox, oy, pb.ccx[c], pb.ccy[c], res);
    else if (pb.cmodel[c] == 3) residual<3>(X, ps, in, ox, oy, pb.ccx[c], pb.ccy[c], res);
    else residual<7>(X, ps, in, ox, oy, pb.ccx[c], pb.ccy[c], res);
}

double eval_cost(const Problem& pb, const double* x) {
    const double* pts = x;
    const double* poses = x + 3 * (size_t)pb.P;
    const double* intr = poses + 6 * (size_t)pb.C;
    double cost = 0;
    #pragma omp parallel for reduction(+ : cost) schedule(static)
    for (int o = 0; o < pb.O; ++o) {
        double res[2];
        const int c = pb.obs_cam[o];
        const double* X = pts + 3 * (size_t)pb.obs_point[o];
        const double* ps = poses + 6 * (size_t)c;
        residual_of(pb, c, X, ps, intr, pb.obs_xy[2 * o], pb.obs_xy[2 * o + 1], res);
        cost += res[0] * res[0] + res[1] * res[1];
    }
    return 0.5 * cost;
}

double linearize(const Problem& pb, const double* x, Lin& L) {
    const double* pts = x;
    const double* poses = x + 3 * (size_t)pb.P;
    const double* intr = poses + 6 * (size_t)pb.C;
    L.r.resize(2 * (size_t)pb.O); L.Je.resize(6 * (size_t)pb.O); L.Jc.resize(12 * (size_t)pb.O);
    L.Ji.assign(2 * (size_t)KMAX * pb.O, 0.0);
    double cost = 0;
    #pragma omp parallel for reduction(+ : cost) schedule(static)
    for (int o = 0; o < pb.O; ++o) {
        const int c = pb.obs_cam[o];
        const double* X = pts + 3 * (size_t)pb.obs_point[o];
        const double* ps = poses + 6 * (size_t)c;
        const double* in = intr + pb.coff[c];
        double* r = &L.r[2 * (size_t)o];
        double* Je = &L.Je[6 * (size_t)o];
        double* Jc = &L.Jc[12 * (size_t)o];
        double Jk[2 * KMAX];
        const double ox = pb.obs_xy[2 * o], oy = pb.obs_xy[2 * o + 1];
        const int k = pb.cmodel[c];
        if (k == 1) eval_jet<1>(X, ps, in, ox, oy, pb.ccx[c], pb.ccy[c], r, Je, Jc, Jk);
        else if (k == 3) eval_jet<3>(X, ps, in, ox, oy, pb.ccx[c], pb.ccy[c], r, Je, Jc, Jk);
        else eval_jet<7>(X, ps, in, ox, oy, pb.ccx[c], pb.ccy[c], r, Je, Jc, Jk);
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < k; ++i) L.Ji[2 * (size_t)KMAX * o + KMAX * j + i] = Jk[j * k + i];
        cost += r[0] * r[0] + r[1] * r[1];
    }
    return 0.5 * cost;
}
// the observation's intrinsics entry i (< k_c) of row j, and its column among the frame parameters
inline double ji(const Lin& L, int o, int j, int i) { return L.Ji[2 * (size_t)KMAX * o + KMAX * j + i]; }

// Column functionals of J (squared column norms or J^T r), parameter order
// [points 3P | poses 6C | intrinsics k].  Deterministic: per-thread partials
// reduced in thread order.
void column_reduce(const Problem& pb, const Lin& L, const double* scale, bool squares, std::vector<double>& out) {
    const int kt = pb.kt;
    const size_t n = 3 * (size_t)pb.P + 6 * (size_t)pb.C + kt;
    out.assign(n, 0.0);
    const int T = omp_get_max_threads();
    std::vector<std::vector<double>> part(T, std::vector<double>(6 * (size_t)pb.C + kt, 0.0));
    #pragma omp parallel
    {
        std::vector<double>& my = part[omp_get_thread_num()];
        #pragma omp for schedule(static)
        for (int o = 0; o < pb.O; ++o) {
            const int p = pb.obs_point[o], c = pb.obs_cam[o];
            const double* r = &L.r[2 * (size_t)o];
            for (int j = 0; j < 2; ++j) {
                const double w = squares ? 0.0 : r[j];
                for (int i = 0; i < 3; ++i) {
                    const double v = L.Je[6 * (size_t)o + 3 * j + i] * (scale ? scale[3 * (size_t)p + i] : 1.0);
                    #pragma omp atomic
                    out[3 * (size_t)p + i] += squares ? v * v : v * w;
                }
                for (int i = 0; i < 6; ++i) {
                    const double v = L.Jc[12 * (size_t)o + 6 * j + i] * (scale ? scale[3 * (size_t)pb.P + 6 * (size_t)c + i] : 1.0);
                    my[6 * (size_t)c + i] += squares ? v * v : v * w;
                }
                for (int i = 0; i < pb.cmodel[c]; ++i) {
                    const size_t col = 6 * (size_t)pb.C + pb.coff[c] + i;
                    const double v = ji(L, o, j, i) * (scale ? scale[3 * (size_t)pb.P + col] : 1.0);
                    my[col] += squares ? v * v : v * w;
                }
            }
        }
    }
    for (int t = 0; t < T; ++t)
        for (size_t i = 0; i < part[t].size(); ++i) out[3 * (size_t)pb.P + i] += part[t][i];
}

// In-place lower Cholesky of the dense n x n SPD matrix A (row-major, lower
// triangle used), right-looking blocked.  Returns false if not PD.
bool cholesky(double* A, int n) {
    const int B = 64;
    for (int k0 = 0; k0 < n; k0 += B) {
        const int kb = std::min(B, n - k0);
        // factor diagonal block
        for (int j = k0; j < k0 + kb; ++j) {
            double d = A[(size_t)j * n + j];
            for (int l = k0; l < j; ++l) d -= A[(size_t)j * n + l] * A[(size_t)j * n + l];
            if (!(d > 0.0) || !std::isfinite(d)) return false;
            d = std::sqrt(d);
            A[(size_t)j * n + j] = d;
            for (int i = j + 1; i < k0 + kb; ++i) {
                double s = A[(size_t)i * n + j];
                for (int l = k0; l < j; ++l) s -= A[(size_t)i * n + l] * A[(size_t)j * n + l];
                A[(size_t)i * n + j] = s / d;
            }
        }
        // panel below: L21 = A21 L11^-T
        #pragma omp parallel for schedule(static)
        for (int i = k0 + kb; i < n; ++i)
            for (int j = k0; j < k0 + kb; ++j) {
                double s = A[(size_t)i * n + j];
                for (int l = k0; l < j; ++l) s -= A[(size_t)i * n + l] * A[(size_t)j * n + l];
                A[(size_t)i * n + j] = s / A[(size_t)j * n + j];
            }
        // trailing update A22 -= L21 L21^T (lower)
        #pragma omp parallel for schedule(dynamic, 8)
        for (int i = k0 + kb; i < n; ++i) {
            const double* li = A + (size_t)i * n + k0;
            for (int j = k0 + kb; j <= i; ++j) {
                const double* lj = A + (size_t)j * n + k0;
                double s = 0;
                for (int l = 0; l < kb; ++l) s += li[l] * lj[l];
                A[(size_t)i * n + j] -= s;
            }
        }
    }
    return true;
}

void chol_solve(const double* L, int n, double* b) {
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int l = 0; l < i; ++l) s -= L[(size_t)i * n + l] * b[l];
        b[i] = s / L[(size_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int l = i + 1; l < n; ++l) s -= L[(size_t)l * n + i] * b[l];
        b[i] = s / L[(size_t)i * n + i];
    }
}

bool inv3_spd(const double* A, double* Ai) {   // via Cholesky of a 3x3 SPD matrix
    double l00 = A[0];
    if (!(l00 > 0)) return false;
    l00 = std::sqrt(l00);
    const double l10 = A[3] / l00, l20 = A[6] / l00;
    double l11 = A[4] - l10 * l10;
    if (!(l11 > 0)) return false;
    l11 = std::sqrt(l11);
    const double l21 = (A[7] - l20 * l10) / l11;
    double l22 = A[8] - l20 * l20 - l21 * l21;
    if (!(l22 > 0)) return false;
    l22 = std::sqrt(l22);
    // inverse of L (lower)
    const double i00 = 1 / l00, i11 = 1 / l11, i22 = 1 / l22;
    const double i10 = -l10 * i00 * i11;
    const double i21 = -l21 * i11 * i22;
    const double i20 = -(l20 * i00 + l21 * i10) * i22;
    // A^-1 = L^-T L^-1
    const double Li[9] = {i00, 0, 0, i10, i11, 0, i20, i21, i22};
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            double s = 0;
            for (int m = 0; m < 3; ++m) s += Li[m * 3 + a] * Li[m * 3 + b];
            Ai[a * 3 + b] = s;
        }
    return true;
}

// Solve (J^T J + diag(D^2)) x = J^T r by Schur elimination of the point blocks.
// J is the (column-scaled) Jacobian held in L, scaled by `scale`.
bool schur_solve(const Problem& pb, const Lin& L, const double* scale, const double* D, const std::vector<int>& pt_start,
                 const std::vector<int>& pt_obs, double* x) {
    const int P = pb.P, C = pb.C;
    const int nf = 6 * C + pb.kt, fb = 6 + KMAX;   // F / W / Y rows are fb wide, 6 + k_c of them used
    auto gcol = [&](int c, int u) { return u < 6 ? 6 * c + u : 6 * C + pb.coff[c] + (u - 6); };
    const size_t ne = 3 * (size_t)P;
    std::vector<double> S((size_t)nf * nf, 0.0), rhs(nf, 0.0);
    const int T = omp_get_max_threads();
    std::vector<std::vector<double>> Sp(T), rp(T);
    std::vector<double> Einv(9 * (size_t)P), ge(3 * (size_t)P);
    bool ok = true;
    #pragma omp parallel
    {
        const int t = omp_get_thread_num();
        std::vector<double>& Sl = Sp[t];
        std::vector<double>& rl = rp[t];
        Sl.assign((size_t)nf * nf, 0.0);
        rl.assign(nf, 0.0);
        std::vector<double> Fo, W, Y;
        #pragma omp for schedule(dynamic, 64)
        for (int p = 0; p < P; ++p) {
            const int o0 = pt_start[p], o1 = pt_start[p + 1], m = o1 - o0;
            double E[9] = {0}, g[3] = {0};
            Fo.assign((size_t)m * 2 * fb, 0.0);
            for (int a = 0; a < m; ++a) {
                const int o = pt_obs[o0 + a], c = pb.obs_cam[o];
                const double* r = &L.r[2 * (size_t)o];
                double je[6];
                for (int j = 0; j < 2; ++j)
                    for (int i = 0; i < 3; ++i) je[j * 3 + i] = L.Je[6 * (size_t)o + 3 * j + i] * scale[3 * (size_t)p + i];
                double* F = &Fo[(size_t)a * 2 * fb];
                for (int j = 0; j < 2; ++j) {
                    for (int i = 0; i < 6; ++i) F[j * fb + i] = L.Jc[12 * (size_t)o + 6 * j + i] * scale[ne + 6 * (size_t)c + i];
                    for (int i = 0; i < pb.cmodel[c]; ++i) F[j * fb + 6 + i] = ji(L, o, j, i) * scale[ne + gcol(c, 6 + i)];
                }
                for (int aa = 0; aa < 3; ++aa) {
                    for (int bb = 0; bb < 3; ++bb) E[aa * 3 + bb] += je[aa] * je[bb] + je[3 + aa] * je[3 + bb];
                    g[aa] += je[aa] * r[0] + je[3 + aa] * r[1];
                }
                // C block + rhs_f: F^T F, F^T r
                const int fo = 6 + pb.cmodel[c];
                for (int u = 0; u < fo; ++u) {
                    const int gu = gcol(c, u);
                    rl[gu] += F[u] * r[0] + F[fb + u] * r[1];
                    for (int v = 0; v < fo; ++v) {
                        const int gv = gcol(c, v);
                        Sl[(size_t)gu * nf + gv] += F[u] * F[v] + F[fb + u] * F[fb + v];
                    }
                }
            }
            for (int i = 0; i < 3; ++i) E[i * 4] += D[3 * (size_t)p + i] * D[3 * (size_t)p + i];
            double Ei[9];
            if (!inv3_spd(E, Ei)) { ok = false; continue; }
            std::memcpy(&Einv[9 * (size_t)p], Ei, sizeof Ei);
            std::memcpy(&ge[3 * (size_t)p], g, sizeof g);
            // W_a = Je_a^T F_a (3 x fb), Y_a = Einv W_a
            W.assign((size_t)m * 3 * fb, 0.0);
            Y.assign((size_t)m * 3 * fb, 0.0);
            for (int a = 0; a < m; ++a) {
                const int o = pt_obs[o0 + a];
                const int fo = 6 + pb.cmodel[pb.obs_cam[o]];
                double je[6];
                for (int j = 0; j < 2; ++j)
                    for (int i = 0; i < 3; ++i) je[j * 3 + i] = L.Je[6 * (size_t)o + 3 * j + i] * scale[3 * (size_t)p + i];
                const double* F = &Fo[(size_t)a * 2 * fb];
                double* Wa = &W[(size_t)a * 3 * fb];
                for (int i = 0; i < 3; ++i)
                    for (int u = 0; u < fo; ++u) Wa[i * fb + u] = je[i] * F[u] + je[3 + i] * F[fb + u];
                double* Ya = &Y[(size_t)a * 3 * fb];
                for (int i = 0; i < 3; ++i)
                    for (int u = 0; u < fo; ++u)
                        Ya[i * fb + u] = Ei[i * 3] * Wa[u] + Ei[i * 3 + 1] * Wa[fb + u] + Ei[i * 3 + 2] * Wa[2 * fb + u];
            }
            // S -= W_a^T Y_b ; rhs_f -= W_a^T Einv g
            double Eg[3];
            for (int i = 0; i < 3; ++i) Eg[i] = Ei[i * 3] * g[0] + Ei[i * 3 + 1] * g[1] + Ei[i * 3 + 2] * g[2];
            for (int a = 0; a < m; ++a) {
                const int ca = pb.obs_cam[pt_obs[o0 + a]], fa = 6 + pb.cmodel[ca];
                const double* Wa = &W[(size_t)a * 3 * fb];
                for (int u = 0; u < fa; ++u) {
                    const int gu = gcol(ca, u);
                    rl[gu] -= Wa[u] * Eg[0] + Wa[fb + u] * Eg[1] + Wa[2 * fb + u] * Eg[2];
                }
                for (int b = 0; b < m; ++b) {
                    const int cb = pb.obs_cam[pt_obs[o0 + b]], fbb = 6 + pb.cmodel[cb];
                    const double* Yb = &Y[(size_t)b * 3 * fb];
                    for (int u = 0; u < fa; ++u) {
                        const int gu = gcol(ca, u);
                        for (int v = 0; v < fbb; ++v) {
                            const int gv = gcol(cb, v);
                            Sl[(size_t)gu * nf + gv] -= Wa[u] * Yb[v] + Wa[fb + u] * Yb[fb + v] + Wa[2 * fb + u] * Yb[2 * fb + v];
                        }
                    }
                }
            }
        }
        #pragma omp barrier
        #pragma omp for schedule(static)
        for (int i = 0; i < nf; ++i) {
            for (int tt = 0; tt < T; ++tt) {
                rhs[i] += rp[tt][i];
                const double* src = &Sp[tt][(size_t)i * nf];
                double* dst = &S[(size_t)i * nf];
                for (int j = 0; j <= i; ++j) dst[j] += src[j];
            }
        }
    }
    if (!ok) return false;
    for (int i = 0; i < nf; ++i) S[(size_t)i * nf + i] += D[ne + i] * D[ne + i];
    if (!cholesky(S.data(), nf)) return false;
    chol_solve(S.data(), nf, rhs.data());
    double* xf = x + ne;
    for (int i = 0; i < nf; ++i) xf[i] = rhs[i];
    // back-substitute points: x_e = Einv (g_e - sum_a W_a x_f)
    #pragma omp parallel for schedule(dynamic, 64)
    for (int p = 0; p < P; ++p) {
        double q[3] = {ge[3 * (size_t)p], ge[3 * (size_t)p + 1], ge[3 * (size_t)p + 2]};
        for (int a = pt_start[p]; a < pt_start[p + 1]; ++a) {
            const int o = pt_obs[a], c = pb.obs_cam[o];
            const int kc = pb.cmodel[c];
            double je[6], F[2][16];
            for (int j = 0; j < 2; ++j) {
                for (int i = 0; i < 3; ++i) je[j * 3 + i] = L.Je[6 * (size_t)o + 3 * j + i] * scale[3 * (size_t)p + i];
                for (int i = 0; i < 6; ++i) F[j][i] = L.Jc[12 * (size_t)o + 6 * j + i] * scale[ne + 6 * (size_t)c + i];
                for (int i = 0; i < kc; ++i) F[j][6 + i] = ji(L, o, j, i) * scale[ne + gcol(c, 6 + i)];
            }
            double Fx[2] = {0, 0};
            for (int j = 0; j < 2; ++j) {
                for (int i = 0; i < 6; ++i) Fx[j] += F[j][i] * xf[6 * c + i];
                for (int i = 0; i < kc; ++i) Fx[j] += F[j][6 + i] * xf[gcol(c, 6 + i)];
            }
            for (int i = 0; i < 3; ++i) q[i] -= je[i] * Fx[0] + je[3 + i] * Fx[1];
        }
        const double* Ei = &Einv[9 * (size_t)p];
        for (int i = 0; i < 3; ++i) x[3 * (size_t)p + i] = Ei[i * 3] * q[0] + Ei[i * 3 + 1] * q[1] + Ei[i * 3 + 2] * q[2];
    }
    return true;
}

double norm2(const std::vector<double>& v) { double s = 0; for (double a : v) s += a * a; return std::sqrt(s); }

}  // namespace

extern "C" {

// Mirrors sfmx_ba_problem / sfmx_ba_options / sfmx_ba_summary of include/sfmx_ba.h.
struct orc_ba_problem {
    int32_t n_points, n_cams, n_obs, cam_model;
    double* points; double* poses; double* intr;
    const int32_t* obs_point; const int32_t* obs_cam; const double* obs_xy;
    double cx, cy;
    int32_t n_intr, reserved;
    const int32_t* intr_model; const int32_t* pose_intr; const double* intr_center;
};
struct orc_ba_options {
    int32_t max_num_iterations, max_num_consecutive_invalid_steps, jacobi_scaling, device;
    double function_tolerance, gradient_tolerance, parameter_tolerance;
    double initial_trust_region_radius, max_trust_region_radius, min_trust_region_radius;
    double min_lm_diagonal, max_lm_diagonal, min_relative_decrease;
};
struct orc_ba_summary {
    double initial_cost, final_cost;
    int32_t num_successful_steps, num_unsuccessful_steps, num_invalid_steps, termination_type;
    double total_ms, ms_per_iteration;
    double final_gradient_max_norm, final_radius;
};

enum { TERM_CONVERGENCE = 0, TERM_NO_CONVERGENCE = 1, TERM_FAILURE = 2 };

// The Ceres problem of the caller's arrays (BundleAdjustment.cpp:45-91): n_intr == 0 is the one
// camera (cam_model, cx, cy) every pose uses.  Returns the length of the caller's intr array, or -1.
int make_problem(const orc_ba_problem* in, Problem& pb) {
    pb.P = in->n_points; pb.C = in->n_cams; pb.O = in->n_obs;
    pb.obs_point = in->obs_point; pb.obs_cam = in->obs_cam; pb.obs_xy = in->obs_xy;
    const int M = in->n_intr > 0 ? in->n_intr : 1;
    std::vector<int> model(M), start(M + 1, 0), used(M, 0), first(M, -1);
    std::vector<double> mcx(M), mcy(M);
    for (int m = 0; m < M; ++m) {
        model[m] = in->n_intr > 0 ? in->intr_model[m] : in->cam_model;
        if (model[m] != 1 && model[m] != 3 && model[m] != 7) return -1;
        mcx[m] = in->n_intr > 0 ? in->intr_center[2 * m] : in->cx;
        mcy[m] = in->n_intr > 0 ? in->intr_center[2 * m + 1] : in->cy;
        start[m + 1] = start[m] + model[m];
    }
    auto cam_of = [&](int c) { return in->n_intr > 0 ? in->pose_intr[c] : 0; };
    for (int o = 0; o < pb.O; ++o) used[cam_of(pb.obs_cam[o])] = 1;
    pb.kt = 0;
    pb.isrc.clear();
    for (int m = 0; m < M; ++m)
        if (used[m]) {
            first[m] = pb.kt;
            for (int i = 0; i < model[m]; ++i) pb.isrc.push_back(start[m] + i);
            pb.kt += model[m];
        }
    pb.cmodel.assign(pb.C, 1); pb.coff.assign(pb.C, 0); pb.ccx.assign(pb.C, 0.0); pb.ccy.assign(pb.C, 0.0);
    for (int c = 0; c < pb.C; ++c) {
        const int m = cam_of(c);
        if (first[m] < 0) continue;   // a pose without observations is never evaluated
        pb.cmodel[c] = model[m]; pb.coff[c] = first[m]; pb.ccx[c] = mcx[m]; pb.ccy[c] = mcy[m];
    }
    return start[M];
}

void load_x(const orc_ba_problem* in, const Problem& pb, std::vector<double>& x) {
    const size_t ne = 3 * (size_t)pb.P;
    x.assign(ne + 6 * (size_t)pb.C + pb.kt, 0.0);
    std::memcpy(x.data(), in->points, sizeof(double) * ne);
    std::memcpy(x.data() + ne, in->poses, sizeof(double) * 6 * pb.C);
    for (int j = 0; j < pb.kt; ++j) x[ne + 6 * (size_t)pb.C + j] = in->intr[pb.isrc[j]];
}

double orc_ba_cost(const orc_ba_problem* in) {
    Problem pb;
    if (make_problem(in, pb) < 0) return -1.0;
    std::vector<double> x;
    load_x(in, pb, x);
    return eval_cost(pb, x.data());
}

// Residuals + Jacobian blocks of every observation (for the autodiff tests).  Ji rows are the
// caller's intr layout (its whole length), the observation's camera block filled, the rest 0.
int orc_ba_jacobian(const orc_ba_problem* in, double* r, double* Je, double* Jc, double* Ji) {
    Problem pb;
    const int kl = make_problem(in, pb);
    if (kl < 0) return -1;
    std::vector<double> x;
    load_x(in, pb, x);
    Lin L;
    linearize(pb, x.data(), L);
    std::memcpy(r, L.r.data(), sizeof(double) * L.r.size());
    std::memcpy(Je, L.Je.data(), sizeof(double) * L.Je.size());
    std::memcpy(Jc, L.Jc.data(), sizeof(double) * L.Jc.size());
    for (int o = 0; o < pb.O; ++o) {
        const int c = pb.obs_cam[o];
        for (int j = 0; j < 2; ++j) {
            double* row = Ji + 2 * (size_t)kl * o + (size_t)kl * j;
            for (int i = 0; i < kl; ++i) row[i] = 0.0;
            for (int i = 0; i < pb.cmodel[c]; ++i) row[pb.isrc[pb.coff[c] + i]] = ji(L, o, j, i);
        }
    }
    return 0;
}

// Levenberg-Marquardt (Ceres 1.14 trust-region loop) + DENSE_SCHUR.  Writes
// the solution back into problem->points/poses/intr (the reference's
// write-back, BundleAdjustment.cpp:97-138).  trace (optional, 3 doubles per
// iteration: cost, radius, accepted) receives the iterate sequence.
int orc_ba_solve(orc_ba_problem* in, const orc_ba_options* opt, orc_ba_summary* sum, double* trace, int trace_cap,
                 int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const auto t0 = std::chrono::steady_clock::now();
    Problem pb;
    if (make_problem(in, pb) < 0) return -1;
    const size_t ne = 3 * (size_t)pb.P, n = ne + 6 * (size_t)pb.C + pb.kt;
    std::vector<double> x, cand(n), delta(n), scale(n, 1.0), D(n), diag(n), step(n), g;
    load_x(in, pb, x);
    // point -> observation CSR (observations are point-major in the reference, but do not rely on it)
    std::vector<int> pt_start(pb.P + 1, 0), pt_obs(pb.O);
    for (int o = 0; o < pb.O; ++o) pt_start[pb.obs_point[o] + 1]++;
    for (int p = 0; p < pb.P; ++p) pt_start[p + 1] += pt_start[p];
    { std::vector<int> fill(pt_start.begin(), pt_start.end() - 1); for (int o = 0; o < pb.O; ++o) pt_obs[fill[pb.obs_point[o]]++] = o; }

    Lin L;
    double cost = linearize(pb, x.data(), L);
    column_reduce(pb, L, nullptr, false, g);   // unscaled gradient J^T r
    double gmax = 0; for (double v : g) gmax = std::max(gmax, std::fabs(v));
    if (opt->jacobi_scaling) {
        std::vector<double> cs;
        column_reduce(pb, L, nullptr, true, cs);
        for (size_t i = 0; i < n; ++i) scale[i] = 1.0 / (1.0 + std::sqrt(cs[i]));
    }
    auto refresh_diag = [&]() {
        std::vector<double> cs;
        column_reduce(pb, L, scale.data(), true, cs);
        for (size_t i = 0; i < n; ++i) diag[i] = std::min(std::max(cs[i], opt->min_lm_diagonal), opt->max_lm_diagonal);
    };
    refresh_diag();
    double x_norm = norm2(x);
    sum->initial_cost = cost;
    double radius = opt->initial_trust_region_radius, decrease = 2.0;
    bool successful = true;
    int iteration = 0, succ = 0, unsucc = 0, invalid_total = 0, consec_invalid = 0, ntrace = 0;
    int term = TERM_NO_CONVERGENCE;
    for (;;) {
        // FinalizeIterationAndCheckIfMinimizerCanContinue
        if (successful) ++succ; else ++unsucc;
        if (trace && ntrace < trace_cap) { trace[3 * ntrace] = cost; trace[3 * ntrace + 1] = radius; trace[3 * ntrace + 2] = successful; ++ntrace; }
        if (iteration >= opt->max_num_iterations) { term = TERM_NO_CONVERGENCE; break; }
        if (successful && gmax <= opt->gradient_tolerance) { term = TERM_CONVERGENCE; break; }
        if (radius <= opt->min_trust_region_radius) { term = TERM_CONVERGENCE; break; }
        ++iteration;
        // ComputeTrustRegionStep (LM strategy)
        for (size_t i = 0; i < n; ++i) D[i] = std::sqrt(diag[i] / radius);
        bool solved = schur_solve(pb, L, scale.data(), D.data(), pt_start, pt_obs, step.data());
        bool finite = solved;
        if (solved) for (size_t i = 0; i < n && finite; ++i) finite = std::isfinite(step[i]);
        double mcc = -1.0;
        if (finite) {
            for (size_t i = 0; i < n; ++i) step[i] = -step[i];
            // model residuals J_s step (per observation)
            double acc = 0;
            #pragma omp parallel for reduction(+ : acc) schedule(static)
            for (int o = 0; o < pb.O; ++o) {
                const int p = pb.obs_point[o], c = pb.obs_cam[o];
                const size_t i0 = ne + 6 * (size_t)pb.C + pb.coff[c];
                for (int j = 0; j < 2; ++j) {
                    double m = 0;
                    for (int i = 0; i < 3; ++i) m += L.Je[6 * (size_t)o + 3 * j + i] * scale[3 * (size_t)p + i] * step[3 * (size_t)p + i];
                    for (int i = 0; i < 6; ++i) m += L.Jc[12 * (size_t)o + 6 * j + i] * scale[ne + 6 * (size_t)c + i] * step[ne + 6 * (size_t)c + i];
                    for (int i = 0; i < pb.cmodel[c]; ++i) m += ji(L, o, j, i) * scale[i0 + i] * step[i0 + i];
                    acc += m * (L.r[2 * (size_t)o + j] + m / 2.0);
                }
            }
            mcc = -acc;
        }
        if (!(finite && mcc > 0.0)) {   // invalid step (HandleInvalidStep)
            ++invalid_total;
            if (++consec_invalid >= opt->max_num_consecutive_invalid_steps) { term = TERM_FAILURE; break; }
            radius /= decrease; decrease *= 2.0;
            successful = false;
            continue;
        }
        consec_invalid = 0;
        for (size_t i = 0; i < n; ++i) { delta[i] = step[i] * scale[i]; cand[i] = x[i] + delta[i]; }
        double ccost = eval_cost(pb, cand.data());
        if (!std::isfinite(ccost)) ccost = std::numeric_limits<double>::max();
        // ParameterToleranceReached
        double sn = 0; for (size_t i = 0; i < n; ++i) sn += (x[i] - cand[i]) * (x[i] - cand[i]);
        sn = std::sqrt(sn);
        if (sn <= opt->parameter_tolerance * (x_norm + opt->parameter_tolerance)) { term = TERM_CONVERGENCE; break; }
        // FunctionToleranceReached
        if (std::fabs(cost - ccost) <= opt->function_tolerance * cost) { term = TERM_CONVERGENCE; break; }
        const double rel = (cost - ccost) / mcc;
        if (rel > opt->min_relative_decrease) {   // HandleSuccessfulStep
            x.swap(cand);
            x_norm = norm2(x);
            cost = linearize(pb, x.data(), L);
            column_reduce(pb, L, nullptr, false, g);
            gmax = 0; for (double v : g) gmax = std::max(gmax, std::fabs(v));
            refresh_diag();
            radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rel - 1.0, 3));
            radius = std::min(opt->max_trust_region_radius, radius);
            decrease = 2.0;
            successful = true;
        } else {                                   // HandleUnsuccessfulStep
            radius /= decrease; decrease *= 2.0;
            successful = false;
        }
    }
    std::memcpy(in->points, x.data(), sizeof(double) * ne);
    std::memcpy(in->poses, x.data() + ne, sizeof(double) * 6 * pb.C);
    for (int j = 0; j < pb.kt; ++j) in->intr[pb.isrc[j]] = x[ne + 6 * (size_t)pb.C + j];   // unreferenced cameras untouched
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    sum->final_cost = cost;
    sum->num_successful_steps = succ;
    sum->num_unsuccessful_steps = unsucc;
    sum->num_invalid_steps = invalid_total;
    sum->termination_type = term;
    sum->total_ms = ms;
    sum->ms_per_iteration = ms / std::max(1, succ + unsucc);
    sum->final_gradient_max_norm = gmax;
    sum->final_radius = radius;
    return ntrace;
}

}  // extern "C"
