// SPDX-License-Identifier: MIT
// sfmx bundle adjustment — host driver behind include/sfmx_ba.h.
//
// Replaces BundleAdjustment::doBundleAdjustment (src/photogrammetrie/common/
// BundleAdjustment.cpp:29-141) + CeresUtils::solve (util/CeresUtils.cpp:38-56):
//   * problem assembly as flat CSR arrays in O(observations), instead of one
//     OpenMpUtils::find_if parallel region per observation (BundleAdjustment.cpp:66-69);
//   * the Ceres 1.14 trust-region / Levenberg-Marquardt loop with DENSE_SCHUR on the
//     host, every numeric step in the HIP kernels of ba_kernels.hpp; only a handful of
//     scalars cross PCIe per iteration.
// The controller mirrors oracle/ba_oracle.cpp (the CPU restatement) step for step.
#include "ba_kernels.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <cstdlib>
#include <unordered_map>
#include <vector>

#include "../../include/sfmx.h"
#include "../../include/sfmx_ba.h"
#include "match_common.hpp"

using namespace sfmx::ba;

namespace {

int fail(int code, const std::string& m) { sfmx::set_last_error(m.c_str()); return code; }

#define HIPCHK(expr)                                                                                \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail(e_ == hipErrorOutOfMemory ? SFMX_ENOMEM : SFMX_EDEVICE,                     \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                         \
    } while (0)
#define RC(expr) do { int rc_ = (expr); if (rc_) return rc_; } while (0)

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    int alloc(size_t b) {
        if (p) { (void)hipFree(p); p = nullptr; }
        bytes = std::max<size_t>(b, 64);
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) { p = nullptr; return fail(SFMX_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)); }
        return SFMX_OK;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

inline unsigned nblk(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

}  // namespace

struct sfmx_ba_ctx {
    int device = 0;
    hipStream_t st = nullptr;
    sfmx_ba_options opt{};
    int P = 0, C = 0, O = 0, K = 0;
    double cx = 0, cy = 0;
    int64_t n = 0, ne = 0;
    int nf = 0, npad = 0, T = 0, nblocks = 0, nvz = 0;
    sfmx_allreduce_fn ar = nullptr;
    void* ar_user = nullptr;
    // topology
    Buf obs_point, obs_cam, obs_xy, pt_start, pt_obs, cam_start, cam_obs, campos, blk_cam, blk_start, trip;
    Buf pgrp, pbig;   // ba_point_blocks_lds point groups (bounds) / points with more than PB_CAPO observations
    int ngrp = 0, nbig = 0;
    // state
    Buf x, cand, scale, colsq, grad, diag, D, J, partA, partB, scal, ipart;
    Buf Einv, EinvG, R1, R2, vzpart, Scc, Spi, Sii, rc, ri, Spp, SR, Linv, sol, step, failf;
    bool scaled = false;
    // locality order: internal point p' is caller point pperm[p']; internal
    // observation o' is caller observation operm[o'] (point-major)
    std::vector<int> pperm, operm;
    double phase_ms[4] = {0, 0, 0, 0};
    hipEvent_t ev[6] = {};
    ~sfmx_ba_ctx() {
        Buf* all[] = {&pgrp, &pbig, &obs_point, &obs_cam, &obs_xy, &pt_start, &pt_obs, &cam_start, &cam_obs, &campos, &blk_cam,
                      &blk_start, &trip, &x, &cand, &scale, &colsq, &grad, &diag, &D, &J, &partA, &partB, &scal,
                      &ipart, &Einv, &EinvG, &R1, &R2, &vzpart, &Scc, &Spi, &Sii, &rc, &ri, &Spp, &SR, &Linv, &sol,
                      &step, &failf};
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        for (Buf* b : all) b->release();
        for (auto& e : ev) if (e) (void)hipEventDestroy(e);
        if (st) (void)hipStreamDestroy(st);
        (void)hipSetDevice(prev);
    }
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) { (void)hipGetDevice(&prev); (void)hipSetDevice(d); }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

int allreduce(sfmx_ba_ctx* c, double* buf, int64_t count, int op) {
    if (!c->ar) return SFMX_OK;
    if (c->ar(buf, count, op, c->ar_user, (void*)c->st) != 0) return fail(SFMX_EDEVICE, "all-reduce callback failed");
    return SFMX_OK;
}

double* scal(sfmx_ba_ctx* c, int i) { return c->scal.as<double>() + i; }

int fetch_scalars(sfmx_ba_ctx* c, int i0, int cnt, double* out) {
    HIPCHK(hipMemcpyAsync(out, scal(c, i0), sizeof(double) * cnt, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return SFMX_OK;
}

// 1/2 sum ||r||^2 at parameters xp (all ranks); with JAC also r + Jacobian into c->J.
template <bool JAC>
int eval(sfmx_ba_ctx* c, const double* xp, double* cost_out) {
    const unsigned g = nblk(c->O);
    const double* pts = xp;
    const double* poses = xp + c->ne;
    const double* intr = poses + 6 * (size_t)c->C;
#define LIN(KK) hipLaunchKernelGGL((ba_linearize<KK, JAC>), dim3(g), dim3(256), 0, c->st, c->O, c->obs_point.as<int>(), \
                                   c->obs_cam.as<int>(), c->obs_xy.as<double>(), c->cx, c->cy, pts, poses, intr,         \
                                   c->J.as<double>(), c->partA.as<double>())
    if (c->K == 1) LIN(1); else if (c->K == 3) LIN(3); else LIN(7);
#undef LIN
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(ba_sum, dim3(1), dim3(256), 0, c->st, c->partA.as<double>(), (int)g, 0.5, scal(c, 0));
    RC(allreduce(c, scal(c, 0), 1, SFMX_REDUCE_SUM));
    RC(fetch_scalars(c, 0, 1, cost_out));
    return SFMX_OK;
}

// After a linearisation: unscaled column norms and gradient, the Jacobi scale
// (iteration 0 only), the clamped LM diagonal of the scaled Jacobian, |g|_max.
int columns(sfmx_ba_ctx* c, double* gmax) {
    double* cs = c->colsq.as<double>();
    double* gr = c->grad.as<double>();
    double* fcs = cs + c->ne;
    double* fgr = gr + c->ne;
#define COLS(KK)                                                                                                        \
    hipLaunchKernelGGL(ba_point_cols<KK>, dim3(nblk(c->P)), dim3(256), 0, c->st, c->P, c->O, c->pt_start.as<int>(),     \
                       c->pt_obs.as<int>(), c->J.as<double>(), cs, gr);                                                 \
    hipLaunchKernelGGL(ba_cam_cols<KK>, dim3(std::max(c->C, 1)), dim3(256), 0, c->st, c->O, c->cam_start.as<int>(),     \
                       c->cam_obs.as<int>(), c->J.as<double>(), fcs, fgr, c->ipart.as<double>());                       \
    hipLaunchKernelGGL(ba_intr_cols_final<KK>, dim3(1), dim3(64), 0, c->st, c->C, c->ipart.as<double>(),                \
                       fcs + 6 * (size_t)c->C, fgr + 6 * (size_t)c->C)
    if (c->K == 1) { COLS(1); } else if (c->K == 3) { COLS(3); } else { COLS(7); }
#undef COLS
    HIPCHK(hipGetLastError());
    RC(allreduce(c, fcs, c->nf, SFMX_REDUCE_SUM));   // camera / intrinsics columns: sums over all ranks' observations
    RC(allreduce(c, fgr, c->nf, SFMX_REDUCE_SUM));
    if (!c->scaled) {
        if (c->opt.jacobi_scaling)
            hipLaunchKernelGGL(ba_scale, dim3(nblk(c->n)), dim3(256), 0, c->st, (int)c->n, cs, c->scale.as<double>());
        c->scaled = true;
    }
    const unsigned g = nblk(c->n);
    hipLaunchKernelGGL(ba_diag, dim3(g), dim3(256), 0, c->st, (int)c->n, cs, c->scale.as<double>(), c->opt.min_lm_diagonal,
                       c->opt.max_lm_diagonal, c->diag.as<double>(), gr, c->partB.as<double>());
    hipLaunchKernelGGL(ba_max, dim3(1), dim3(256), 0, c->st, c->partB.as<double>(), (int)g, scal(c, 1));
    HIPCHK(hipGetLastError());
    RC(allreduce(c, scal(c, 1), 1, SFMX_REDUCE_MAX));
    RC(fetch_scalars(c, 1, 1, gmax));
    return SFMX_OK;
}

// sum of squares of v over [0, ne) (summed across ranks) + [ne, n) (replicated) -> sqrt
int split_norm(sfmx_ba_ctx* c, const double* v, double* out) {
    const unsigned ge = nblk(c->ne), gf = nblk(c->nf);
    hipLaunchKernelGGL(ba_sumsq, dim3(ge), dim3(256), 0, c->st, (int)c->ne, v, c->partA.as<double>());
    hipLaunchKernelGGL(ba_sum, dim3(1), dim3(256), 0, c->st, c->partA.as<double>(), (int)ge, 1.0, scal(c, 2));
    hipLaunchKernelGGL(ba_sumsq, dim3(gf), dim3(256), 0, c->st, c->nf, v + c->ne, c->partB.as<double>());
    hipLaunchKernelGGL(ba_sum, dim3(1), dim3(256), 0, c->st, c->partB.as<double>(), (int)gf, 1.0, scal(c, 3));
    HIPCHK(hipGetLastError());
    RC(allreduce(c, scal(c, 2), 1, SFMX_REDUCE_SUM));
    double s[2];
    RC(fetch_scalars(c, 2, 2, s));
    *out = std::sqrt(s[0] + s[1]);
    return SFMX_OK;
}

// Schur solve of (J_s^T J_s + D^2) sol = J_s^T r, step_s = -sol, candidate
// = x + step_s * scale; model cost change, step norm, candidate cost.
int try_step(sfmx_ba_ctx* c, double radius, bool* valid, double* mcc, double* step_norm, double* ccost) {
    const int K = c->K, P = c->P, O = c->O, C = c->C, npad = c->npad, T = c->T;
    double* S = c->SR.as<double>();
    double* rhs = S + (size_t)npad * npad;
    int* fl = c->failf.as<int>();
    HIPCHK(hipEventRecord(c->ev[0], c->st));
    hipLaunchKernelGGL(ba_lm_d, dim3(nblk(c->n)), dim3(256), 0, c->st, (int)c->n, c->diag.as<double>(), radius,
                       c->D.as<double>());
    HIPCHK(hipMemsetAsync(fl, 0, sizeof(int), c->st));
#define SCHUR(KK)                                                                                                      \
    if (c->ngrp > 0)                                                                                                   \
        hipLaunchKernelGGL(ba_point_blocks_lds<KK>, dim3(c->ngrp), dim3(256), 0, c->st, c->pgrp.as<int>(), P, C,       \
                           c->pt_start.as<int>(), c->obs_cam.as<int>(), c->campos.as<int>(), c->J.as<double>(),        \
                           c->scale.as<double>(), c->D.as<double>(), c->Einv.as<double>(), c->EinvG.as<double>(),      \
                           c->R1.as<double>(), c->R2.as<double>(), c->vzpart.as<double>(), fl);                        \
    if (c->nbig > 0)                                                                                                   \
        hipLaunchKernelGGL(ba_point_blocks<KK>, dim3(nblk(c->nbig)), dim3(256), 0, c->st, P, O, C, c->pt_start.as<int>(), \
                           c->pt_obs.as<int>(), c->obs_cam.as<int>(), c->campos.as<int>(), c->J.as<double>(),          \
                           c->scale.as<double>(), c->D.as<double>(), c->Einv.as<double>(), c->EinvG.as<double>(),      \
                           c->R1.as<double>(), c->R2.as<double>(), c->vzpart.as<double>() + (size_t)c->ngrp * KK * KK, \
                           fl, c->pbig.as<int>(), c->nbig);                                                            \
    if (C > 0)                                                                                                         \
        hipLaunchKernelGGL(ba_cam_blocks<KK>, dim3(C), dim3(256), 0, c->st, C, c->cam_start.as<int>(),                 \
                           c->R2.as<double>(), c->Scc.as<double>(), c->Spi.as<double>(), c->rc.as<double>(),           \
                           c->ipart.as<double>());                                                                     \
    hipLaunchKernelGGL(ba_intr_final<KK>, dim3(KK * KK + KK), dim3(256), 0, c->st, C, c->nvz, c->ipart.as<double>(),   \
                       c->vzpart.as<double>(), c->Sii.as<double>(), c->ri.as<double>());                               \
    if (c->nblocks > 0)                                                                                                \
        hipLaunchKernelGGL(ba_pair_blocks<KK>, dim3(c->nblocks), dim3(256), 0, c->st, c->blk_start.as<int>(),          \
                           c->trip.as<int2>(), c->R1.as<double>(), c->Spp.as<double>())
    if (K == 1) { SCHUR(1); } else if (K == 3) { SCHUR(3); } else { SCHUR(7); }
#undef SCHUR
    HIPCHK(hipMemsetAsync(S, 0, sizeof(double) * ((size_t)npad * npad + npad), c->st));
    if (c->nblocks > 0)
        hipLaunchKernelGGL(ba_assemble_pairs, dim3(c->nblocks), dim3(64), 0, c->st, npad, c->blk_cam.as<int>(),
                           c->Spp.as<double>(), S);
    if (C > 0) hipLaunchKernelGGL(ba_assemble_diag, dim3(C), dim3(64), 0, c->st, npad, c->Scc.as<double>(), S);
    hipLaunchKernelGGL(ba_assemble_rest, dim3(nblk(npad)), dim3(256), 0, c->st, C, K, c->nf, npad, c->Spi.as<double>(),
                       c->Sii.as<double>(), c->rc.as<double>(), c->ri.as<double>(), S, rhs);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev[1], c->st));
    // point-sharded ranks: the reduced camera system and its rhs are sums over ranks
    RC(allreduce(c, S, (int64_t)npad * npad + npad, SFMX_REDUCE_SUM));
    hipLaunchKernelGGL(ba_add_damping, dim3(nblk(c->nf)), dim3(256), 0, c->st, P, c->nf, npad, c->D.as<double>(), S);
    double* W = c->Linv.as<double>();
    double* sol = c->sol.as<double>();
    hipLaunchKernelGGL(chol_first, dim3(1), dim3(256), 0, c->st, S, npad, W, rhs, fl);
    for (int k = 0; k + 1 < T; ++k) {
        const int m = T - k - 1;
        hipLaunchKernelGGL(chol_step, dim3(m * (m + 1) / 2), dim3(256), 0, c->st, S, npad, k, W, rhs, fl);
    }
    for (int k = T - 1; k >= 0; --k)
        hipLaunchKernelGGL(chol_back, dim3(std::max(k, 1)), dim3(256), 0, c->st, S, npad, c->nf, k, rhs, sol + c->ne);
#define BACK(KK)                                                                                                    \
    hipLaunchKernelGGL(ba_backsub<KK>, dim3(nblk(P)), dim3(256), 0, c->st, P, C, c->pt_start.as<int>(),              \
                       c->pt_obs.as<int>(), c->obs_cam.as<int>(), c->R1.as<double>(), c->EinvG.as<double>(), sol + c->ne, sol)
    if (K == 1) { BACK(1); } else if (K == 3) { BACK(3); } else { BACK(7); }
#undef BACK
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev[2], c->st));
    // step, candidate, ||x - candidate||^2 split into the rank-local point part and the replicated rest
    const unsigned ge = nblk(c->ne), gf = nblk(c->nf);
    double* x = c->x.as<double>();
    double* cand = c->cand.as<double>();
    double* stp = c->step.as<double>();
    hipLaunchKernelGGL(ba_step, dim3(ge), dim3(256), 0, c->st, (int)c->ne, sol, c->scale.as<double>(), x, stp, cand,
                       c->partA.as<double>());
    hipLaunchKernelGGL(ba_sum, dim3(1), dim3(256), 0, c->st, c->partA.as<double>(), (int)ge, 1.0, scal(c, 4));
    hipLaunchKernelGGL(ba_step, dim3(gf), dim3(256), 0, c->st, c->nf, sol + c->ne, c->scale.as<double>() + c->ne,
                       x + c->ne, stp + c->ne, cand + c->ne, c->partB.as<double>());
    hipLaunchKernelGGL(ba_sum, dim3(1), dim3(256), 0, c->st, c->partB.as<double>(), (int)gf, 1.0, scal(c, 5));
    const unsigned go = nblk(O);
#define MODEL(KK)                                                                                                 \
    hipLaunchKernelGGL(ba_model<KK>, dim3(go), dim3(256), 0, c->st, P, O, C, c->obs_point.as<int>(),              \
                       c->obs_cam.as<int>(), c->J.as<double>(), c->scale.as<double>(), stp, c->partA.as<double>())
    if (K == 1) { MODEL(1); } else if (K == 3) { MODEL(3); } else { MODEL(7); }
#undef MODEL
    hipLaunchKernelGGL(ba_sum, dim3(1), dim3(256), 0, c->st, c->partA.as<double>(), (int)go, 1.0, scal(c, 6));
    HIPCHK(hipGetLastError());
    // fail flag as a double for the cross-rank max
    {
        int h_fail = 0;
        HIPCHK(hipMemcpyAsync(&h_fail, fl, sizeof(int), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        double fd = h_fail ? 1.0 : 0.0;
        HIPCHK(hipMemcpyAsync(scal(c, 7), &fd, sizeof(double), hipMemcpyHostToDevice, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
    }
    RC(allreduce(c, scal(c, 4), 1, SFMX_REDUCE_SUM));
    RC(allreduce(c, scal(c, 6), 1, SFMX_REDUCE_SUM));
    RC(allreduce(c, scal(c, 7), 1, SFMX_REDUCE_MAX));
    double v[4];
    RC(fetch_scalars(c, 4, 4, v));
    const double sn2 = v[0] + v[1];
    *mcc = -v[2];
    *step_norm = std::sqrt(sn2);
    *valid = v[3] == 0.0 && std::isfinite(sn2) && std::isfinite(v[2]) && *mcc > 0.0;
    *ccost = std::numeric_limits<double>::max();
    if (*valid) {
        double cc;
        RC(eval<false>(c, cand, &cc));
        *ccost = std::isfinite(cc) ? cc : std::numeric_limits<double>::max();
    }
    HIPCHK(hipEventRecord(c->ev[3], c->st));
    HIPCHK(hipEventSynchronize(c->ev[3]));
    float a = 0, b = 0, d = 0;
    HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    HIPCHK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
    HIPCHK(hipEventElapsedTime(&d, c->ev[2], c->ev[3]));
    c->phase_ms[1] += a;
    c->phase_ms[2] += b;
    c->phase_ms[3] += d;
    return SFMX_OK;
}

int relinearize(sfmx_ba_ctx* c, double* cost, double* gmax) {
    HIPCHK(hipEventRecord(c->ev[4], c->st));
    RC(eval<true>(c, c->x.as<double>(), cost));
    RC(columns(c, gmax));
    HIPCHK(hipEventRecord(c->ev[5], c->st));
    HIPCHK(hipEventSynchronize(c->ev[5]));
    float a = 0;
    HIPCHK(hipEventElapsedTime(&a, c->ev[4], c->ev[5]));
    c->phase_ms[0] += a;
    return SFMX_OK;
}

int run_lm(sfmx_ba_ctx* c, int max_iters, sfmx_ba_summary* sum, double* trace, int trace_cap, int* ntrace_out) {
    DeviceGuard dg(c->device);
    const auto t0 = std::chrono::steady_clock::now();
    const sfmx_ba_options& o = c->opt;
    const int maxit = max_iters > 0 ? max_iters : o.max_num_iterations;
    for (double& v : c->phase_ms) v = 0;
    c->scaled = false;   // Ceres computes the Jacobi scale at iteration 0 of each Solve
    double cost, gmax, x_norm;
    RC(relinearize(c, &cost, &gmax));
    RC(split_norm(c, c->x.as<double>(), &x_norm));
    sum->initial_cost = cost;
    double radius = o.initial_trust_region_radius, decrease = 2.0;
    bool successful = true;
    int iteration = 0, succ = 0, unsucc = 0, invalid_total = 0, consec_invalid = 0, ntrace = 0;
    int term = SFMX_BA_NO_CONVERGENCE;
    for (;;) {
        // FinalizeIterationAndCheckIfMinimizerCanContinue (Ceres 1.14 trust_region_minimizer.cc [ext])
        if (successful) ++succ; else ++unsucc;
        if (trace && ntrace < trace_cap) {
            trace[3 * ntrace] = cost; trace[3 * ntrace + 1] = radius; trace[3 * ntrace + 2] = successful ? 1.0 : 0.0;
            ++ntrace;
        }
        if (iteration >= maxit) { term = SFMX_BA_NO_CONVERGENCE; break; }
        if (successful && gmax <= o.gradient_tolerance) { term = SFMX_BA_CONVERGENCE; break; }
        if (radius <= o.min_trust_region_radius) { term = SFMX_BA_CONVERGENCE; break; }
        ++iteration;
        bool valid; double mcc, sn, ccost;
        RC(try_step(c, radius, &valid, &mcc, &sn, &ccost));
        if (!valid) {   // HandleInvalidStep
            ++invalid_total;
            if (++consec_invalid >= o.max_num_consecutive_invalid_steps) { term = SFMX_BA_FAILURE; break; }
            radius /= decrease; decrease *= 2.0;
            successful = false;
            continue;
        }
        consec_invalid = 0;
        if (sn <= o.parameter_tolerance * (x_norm + o.parameter_tolerance)) { term = SFMX_BA_CONVERGENCE; break; }
        if (std::fabs(cost - ccost) <= o.function_tolerance * cost) { term = SFMX_BA_CONVERGENCE; break; }
        const double rel = (cost - ccost) / mcc;
        if (rel > o.min_relative_decrease) {   // HandleSuccessfulStep
            std::swap(c->x, c->cand);
            RC(split_norm(c, c->x.as<double>(), &x_norm));
            RC(relinearize(c, &cost, &gmax));
            radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rel - 1.0, 3));
            radius = std::min(o.max_trust_region_radius, radius);
            decrease = 2.0;
            successful = true;
        } else {                                 // HandleUnsuccessfulStep
            radius /= decrease; decrease *= 2.0;
            successful = false;
        }
    }
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
    if (ntrace_out) *ntrace_out = ntrace;
    return SFMX_OK;
}

int validate(const sfmx_ba_problem* pb) {
    if (!pb) return fail(SFMX_EINVAL, "null problem");
    if (pb->n_points < 0 || pb->n_cams < 0 || pb->n_obs < 0) return fail(SFMX_EINVAL, "negative sizes");
    if (pb->cam_model != SFMX_CAM_SIMPLE && pb->cam_model != SFMX_CAM_SIMPLE_RADIAL && pb->cam_model != SFMX_CAM_DISTORTION)
        return fail(SFMX_EINVAL, "cam_model must be SFMX_CAM_SIMPLE, _SIMPLE_RADIAL or _DISTORTION");
    if ((pb->n_points && !pb->points) || (pb->n_cams && !pb->poses) || !pb->intr ||
        (pb->n_obs && (!pb->obs_point || !pb->obs_cam || !pb->obs_xy)))
        return fail(SFMX_EINVAL, "null problem array");
    for (int o = 0; o < pb->n_obs; ++o)
        if (pb->obs_point[o] < 0 || pb->obs_point[o] >= pb->n_points || pb->obs_cam[o] < 0 || pb->obs_cam[o] >= pb->n_cams)
            return fail(SFMX_EINVAL, "observation index out of range");
    return SFMX_OK;
}

template <class T>
int upload(Buf& b, const std::vector<T>& v, hipStream_t st) {
    RC(b.alloc(sizeof(T) * std::max<size_t>(v.size(), 1)));
    if (!v.empty()) HIPCHK(hipMemcpyAsync(b.p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, st));
    return SFMX_OK;
}

int set_params(sfmx_ba_ctx* c, const sfmx_ba_problem* pb) {
    DeviceGuard dg(c->device);
    double* x = c->x.as<double>();
    std::vector<double> pts(3 * (size_t)c->P);
    for (int q = 0; q < c->P; ++q)
        for (int i = 0; i < 3; ++i) pts[3 * (size_t)q + i] = pb->points[3 * (size_t)c->pperm[q] + i];
    if (c->P) HIPCHK(hipMemcpyAsync(x, pts.data(), sizeof(double) * 3 * c->P, hipMemcpyHostToDevice, c->st));
    if (c->C) HIPCHK(hipMemcpyAsync(x + c->ne, pb->poses, sizeof(double) * 6 * c->C, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(x + c->ne + 6 * (size_t)c->C, pb->intr, sizeof(double) * c->K, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return SFMX_OK;
}

// Locality order (internal only; results are reported in the caller's order):
// points sorted by their sorted camera lists (points seen by the same cameras
// become neighbours, so the per-camera and per-camera-pair gathers of the Schur
// kernels hit contiguous records), observations point-major in that order.
void locality_order(const sfmx_ba_problem* pb, std::vector<int>& pperm, std::vector<int>& operm) {
    const int P = pb->n_points, O = pb->n_obs;
    std::vector<int> start(P + 1, 0), obs(O);
    for (int i = 0; i < O; ++i) start[pb->obs_point[i] + 1]++;
    for (int p = 0; p < P; ++p) start[p + 1] += start[p];
    {
        std::vector<int> f(start.begin(), start.end() - 1);
        for (int i = 0; i < O; ++i) obs[f[pb->obs_point[i]]++] = i;
    }
    std::vector<int> cams(O);   // per point: its cameras, sorted
    for (int p = 0; p < P; ++p) {
        for (int a = start[p]; a < start[p + 1]; ++a) cams[a] = pb->obs_cam[obs[a]];
        std::sort(cams.begin() + start[p], cams.begin() + start[p + 1]);
    }
    pperm.resize(P);
    for (int p = 0; p < P; ++p) pperm[p] = p;
    std::stable_sort(pperm.begin(), pperm.end(), [&](int a, int b) {
        return std::lexicographical_compare(cams.begin() + start[a], cams.begin() + start[a + 1],
                                            cams.begin() + start[b], cams.begin() + start[b + 1]);
    });
    operm.clear();
    operm.reserve(O);
    for (int q = 0; q < P; ++q)
        for (int a = start[pperm[q]]; a < start[pperm[q] + 1]; ++a) operm.push_back(obs[a]);
}

int create(const sfmx_ba_problem* caller, const sfmx_ba_options* opt, sfmx_ba_ctx** out) {
    RC(validate(caller));
    std::vector<int> pperm, operm, ipperm(caller->n_points), rop(caller->n_obs), roc(caller->n_obs);
    std::vector<double> rxy(2 * (size_t)caller->n_obs);
    locality_order(caller, pperm, operm);
    for (int q = 0; q < caller->n_points; ++q) ipperm[pperm[q]] = q;
    for (int q = 0; q < caller->n_obs; ++q) {
        const int o = operm[q];
        rop[q] = ipperm[caller->obs_point[o]];
        roc[q] = caller->obs_cam[o];
        rxy[2 * (size_t)q] = caller->obs_xy[2 * (size_t)o];
        rxy[2 * (size_t)q + 1] = caller->obs_xy[2 * (size_t)o + 1];
    }
    sfmx_ba_problem internal = *caller;
    internal.points = nullptr;   // parameters are uploaded from the caller's arrays by set_params
    internal.obs_point = rop.data();
    internal.obs_cam = roc.data();
    internal.obs_xy = rxy.data();
    const sfmx_ba_problem* pb = &internal;
    sfmx_ba_options o;
    sfmx_ba_default_options(&o);
    if (opt) o = *opt;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(SFMX_EDEVICE, "no HIP device visible");
    if (o.device < 0 || o.device >= ndev) return fail(SFMX_EINVAL, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, o.device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SFMX_EDEVICE, "sfmx BA kernels are built for gfx950 only");
    auto* c = new (std::nothrow) sfmx_ba_ctx();
    if (!c) return fail(SFMX_ENOMEM, "host allocation");
    c->device = o.device;
    c->opt = o;
    c->pperm.swap(pperm);
    c->operm.swap(operm);
    DeviceGuard dg(c->device);
    auto bail = [&](int rc) { delete c; return rc; };
    if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) return bail(fail(SFMX_EDEVICE, "stream"));
    for (auto& e : c->ev) if (hipEventCreate(&e) != hipSuccess) return bail(fail(SFMX_EDEVICE, "event"));
    const int P = pb->n_points, C = pb->n_cams, O = pb->n_obs, K = pb->cam_model;
    c->P = P; c->C = C; c->O = O; c->K = K; c->cx = pb->cx; c->cy = pb->cy;
    c->ne = 3 * (int64_t)P;
    c->nf = 6 * C + K;
    c->n = c->ne + c->nf;
    c->npad = (c->nf + NB - 1) / NB * NB;
    c->T = c->npad / NB;
    // CSR by point and by camera (stable: input order inside each list)
    std::vector<int> pt_start(P + 1, 0), pt_obs(O), cam_start(C + 1, 0), cam_obs(O);
    for (int i = 0; i < O; ++i) { pt_start[pb->obs_point[i] + 1]++; cam_start[pb->obs_cam[i] + 1]++; }
    for (int p = 0; p < P; ++p) pt_start[p + 1] += pt_start[p];
    for (int k = 0; k < C; ++k) cam_start[k + 1] += cam_start[k];
    {
        std::vector<int> fp(pt_start.begin(), pt_start.end() - 1), fc(cam_start.begin(), cam_start.end() - 1);
        for (int i = 0; i < O; ++i) { pt_obs[fp[pb->obs_point[i]]++] = i; cam_obs[fc[pb->obs_cam[i]]++] = i; }
    }
    std::vector<int> campos(O);   // position of each observation in the camera-major order
    for (int a = 0; a < O; ++a) campos[cam_obs[a]] = a;
    // camera-pair blocks of the reduced system: ordered observation pairs of
    // each point with cam(a) <= cam(b), bucketed by (cam(a), cam(b)) (point order inside a bucket)
    std::unordered_map<int64_t, int> bid;
    std::vector<int> blk_cam, cnt;
    for (int p = 0; p < P; ++p)
        for (int a = pt_start[p]; a < pt_start[p + 1]; ++a)
            for (int b = pt_start[p]; b < pt_start[p + 1]; ++b) {
                const int ca = pb->obs_cam[pt_obs[a]], cb = pb->obs_cam[pt_obs[b]];
                if (ca > cb) continue;
                const int64_t key = (int64_t)ca * C + cb;
                auto it = bid.find(key);
                int id;
                if (it == bid.end()) { id = (int)cnt.size(); bid.emplace(key, id); cnt.push_back(0); blk_cam.push_back(ca); blk_cam.push_back(cb); }
                else id = it->second;
                cnt[id]++;
            }
    const int NBLK = (int)cnt.size();
    {   // number blocks in (cam(a), cam(b)) order: neighbouring blocks share points, and
        // ba_pair_blocks maps contiguous block ranges to one XCD (L2 reuse of the R1 records)
        std::vector<std::pair<int64_t, int>> keys;
        keys.reserve(NBLK);
        for (auto& kv : bid) keys.emplace_back(kv.first, kv.second);
        std::sort(keys.begin(), keys.end());
        std::vector<int> cnt2(NBLK), cam2(2 * (size_t)NBLK);
        for (int nb = 0; nb < NBLK; ++nb) {
            const int ob = keys[nb].second;
            cnt2[nb] = cnt[ob];
            cam2[2 * nb] = blk_cam[2 * ob];
            cam2[2 * nb + 1] = blk_cam[2 * ob + 1];
            bid[keys[nb].first] = nb;
        }
        cnt.swap(cnt2);
        blk_cam.swap(cam2);
    }
    std::vector<int> blk_start(NBLK + 1, 0);
    for (int b = 0; b < NBLK; ++b) blk_start[b + 1] = blk_start[b] + cnt[b];
    std::vector<int2> trip(blk_start[NBLK]);
    {
        std::vector<int> fill(blk_start.begin(), blk_start.end() - 1);
        for (int p = 0; p < P; ++p)
            for (int a = pt_start[p]; a < pt_start[p + 1]; ++a)
                for (int b = pt_start[p]; b < pt_start[p + 1]; ++b) {
                    const int oa = pt_obs[a], ob = pt_obs[b];
                    const int ca = pb->obs_cam[oa], cb = pb->obs_cam[ob];
                    if (ca > cb) continue;
                    trip[fill[bid[(int64_t)ca * C + cb]]++] = make_int2(oa, ob);
                }
    }
    c->nblocks = NBLK;
    // point groups for ba_point_blocks_lds: consecutive points, <= PB_MAXP points and
    // <= PB_CAPO observations per group; a point with more observations goes to the
    // point-list fallback (ba_point_blocks)
    std::vector<int> pgrp, pbig;
    const char* pbenv = std::getenv("SFMX_BA_POINT_KERNEL");   // "list": every point via ba_point_blocks (A/B tuning)
    if (pbenv && std::strcmp(pbenv, "list") == 0)
        for (int p = 0; p < P; ++p) pbig.push_back(p);
    for (int p = pbig.empty() ? 0 : P; p < P;) {
        const int cnt = pt_start[p + 1] - pt_start[p];
        if (cnt > PB_CAPO) { pbig.push_back(p); ++p; continue; }
        pgrp.push_back(p);   // group = [pgrp[2g], pgrp[2g+1])
        int np = 0, no = 0;
        while (p < P && np < PB_MAXP && pt_start[p + 1] - pt_start[p] <= PB_CAPO && no + (pt_start[p + 1] - pt_start[p]) <= PB_CAPO) {
            no += pt_start[p + 1] - pt_start[p];
            ++np; ++p;
        }
        pgrp.push_back(p);
    }
    c->ngrp = (int)pgrp.size() / 2;
    c->nbig = (int)pbig.size();
    c->nvz = c->ngrp + (c->nbig ? (int)nblk(c->nbig) : 0);
    std::vector<int> op(pb->obs_point, pb->obs_point + O), oc(pb->obs_cam, pb->obs_cam + O);
    std::vector<double> oxy(pb->obs_xy, pb->obs_xy + 2 * (size_t)O);
    hipStream_t st = c->st;
    int rc;
    if ((rc = upload(c->obs_point, op, st)) || (rc = upload(c->obs_cam, oc, st)) || (rc = upload(c->obs_xy, oxy, st)) ||
        (rc = upload(c->pt_start, pt_start, st)) || (rc = upload(c->pt_obs, pt_obs, st)) ||
        (rc = upload(c->cam_start, cam_start, st)) || (rc = upload(c->cam_obs, cam_obs, st)) ||
        (rc = upload(c->campos, campos, st)) ||
        (rc = upload(c->blk_cam, blk_cam, st)) || (rc = upload(c->blk_start, blk_start, st)) ||
        (rc = upload(c->trip, trip, st)) || (rc = upload(c->pgrp, pgrp, st)) || (rc = upload(c->pbig, pbig, st)))
        return bail(rc);
    const size_t n = c->n, so = std::max(O, 1);
    const int NI = std::max(2 * K, K * (K + 1) / 2 + K);
    struct { Buf* b; size_t bytes; } allocs[] = {
        {&c->x, 8 * n}, {&c->cand, 8 * n}, {&c->scale, 8 * n}, {&c->colsq, 8 * n}, {&c->grad, 8 * n},
        {&c->diag, 8 * n}, {&c->D, 8 * n}, {&c->sol, 8 * n}, {&c->step, 8 * n},
        {&c->J, 8 * so * (20 + 2 * K)}, {&c->partA, 8 * (size_t)nblk(std::max<int64_t>(O, n))},
        {&c->partB, 8 * (size_t)nblk(std::max<int64_t>(O, n))}, {&c->scal, 8 * 16},
        {&c->ipart, 8 * (size_t)std::max(C, 1) * NI}, {&c->Einv, 72 * (size_t)std::max(P, 1)},
        {&c->EinvG, 24 * (size_t)std::max(P, 1)}, {&c->R1, 8 * so * r1s(K)}, {&c->R2, 8 * so * r2s(K)},
        {&c->vzpart, 8 * (size_t)std::max(c->nvz, 1) * K * K}, {&c->Linv, 8 * (size_t)2 * NB * NB},
        {&c->Scc, 288 * (size_t)std::max(C, 1)}, {&c->Spi, 48 * (size_t)K * std::max(C, 1)}, {&c->Sii, 8 * (size_t)K * K},
        {&c->rc, 48 * (size_t)std::max(C, 1)}, {&c->ri, 8 * (size_t)K}, {&c->Spp, 288 * (size_t)std::max(NBLK, 1)},
        {&c->SR, 8 * ((size_t)c->npad * c->npad + c->npad)}, {&c->failf, 64}};
    for (auto& a : allocs) if ((rc = a.b->alloc(a.bytes))) return bail(rc);
    // scale = 1 until (and unless) Jacobi scaling sets it
    {
        std::vector<double> ones(n, 1.0);
        if (hipMemcpyAsync(c->scale.p, ones.data(), 8 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return bail(fail(SFMX_EDEVICE, "upload"));
    }
    if ((rc = set_params(c, caller))) return bail(rc);
    *out = c;
    return SFMX_OK;
}

// ---- Ceres rotation conversions (rotation.h, Ceres 1.14 [ext]) ------------
void rotmat_to_aa(const double* R /*col-major 3x3*/, double* aa) {
    auto r = [&](int i, int j) { return R[i + 3 * j]; };
    double q[4];
    const double trace = r(0, 0) + r(1, 1) + r(2, 2);
    if (trace >= 0.0) {
        double t = std::sqrt(trace + 1.0);
        q[0] = 0.5 * t;
        t = 0.5 / t;
        q[1] = (r(2, 1) - r(1, 2)) * t;
        q[2] = (r(0, 2) - r(2, 0)) * t;
        q[3] = (r(1, 0) - r(0, 1)) * t;
    } else {
        int i = 0;
        if (r(1, 1) > r(0, 0)) i = 1;
        if (r(2, 2) > r(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double t = std::sqrt(r(i, i) - r(j, j) - r(k, k) + 1.0);
        q[i + 1] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (r(k, j) - r(j, k)) * t;
        q[j + 1] = (r(j, i) + r(i, j)) * t;
        q[k + 1] = (r(k, i) + r(i, k)) * t;
    }
    const double s2 = q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    if (s2 > 0.0) {
        const double s = std::sqrt(s2), cth = q[0];
        const double two_theta = 2.0 * ((cth < 0.0) ? std::atan2(-s, -cth) : std::atan2(s, cth));
        const double k = two_theta / s;
        aa[0] = q[1] * k; aa[1] = q[2] * k; aa[2] = q[3] * k;
    } else {
        aa[0] = q[1] * 2.0; aa[1] = q[2] * 2.0; aa[2] = q[3] * 2.0;
    }
}

void aa_to_rotmat(const double* aa, double* R /*col-major*/) {
    auto set = [&](int i, int j, double v) { R[i + 3 * j] = v; };
    const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
    if (theta2 > std::numeric_limits<double>::epsilon()) {
        const double theta = std::sqrt(theta2);
        const double wx = aa[0] / theta, wy = aa[1] / theta, wz = aa[2] / theta;
        const double ct = std::cos(theta), st = std::sin(theta);
        set(0, 0, ct + wx * wx * (1.0 - ct));
        set(1, 0, wz * st + wx * wy * (1.0 - ct));
        set(2, 0, -wy * st + wx * wz * (1.0 - ct));
        set(0, 1, wx * wy * (1.0 - ct) - wz * st);
        set(1, 1, ct + wy * wy * (1.0 - ct));
        set(2, 1, wx * st + wy * wz * (1.0 - ct));
        set(0, 2, wy * st + wx * wz * (1.0 - ct));
        set(1, 2, -wx * st + wy * wz * (1.0 - ct));
        set(2, 2, ct + wz * wz * (1.0 - ct));
    } else {
        set(0, 0, 1.0); set(1, 0, aa[2]); set(2, 0, -aa[1]);
        set(0, 1, -aa[2]); set(1, 1, 1.0); set(2, 1, aa[0]);
        set(0, 2, aa[1]); set(1, 2, -aa[0]); set(2, 2, 1.0);
    }
}

}  // namespace

extern "C" {

int sfmx_ba_default_options(sfmx_ba_options* o) {
    if (!o) return fail(SFMX_EINVAL, "null options");
    o->max_num_iterations = 5000;
    o->max_num_consecutive_invalid_steps = 5;
    o->jacobi_scaling = 1;
    o->device = 0;
    o->function_tolerance = 1e-6;
    o->gradient_tolerance = 1e-10;
    o->parameter_tolerance = 1e-8;
    o->initial_trust_region_radius = 1e4;
    o->max_trust_region_radius = 1e16;
    o->min_trust_region_radius = 1e-32;
    o->min_lm_diagonal = 1e-6;
    o->max_lm_diagonal = 1e32;
    o->min_relative_decrease = 1e-3;
    return SFMX_OK;
}

int sfmx_ba_create(const sfmx_ba_problem* problem, const sfmx_ba_options* opt, sfmx_ba_ctx** out) {
    if (!out) return fail(SFMX_EINVAL, "null out");
    *out = nullptr;
    return create(problem, opt, out);
}

int sfmx_ba_set_allreduce(sfmx_ba_ctx* c, sfmx_allreduce_fn fn, void* user) {
    if (!c) return fail(SFMX_EINVAL, "null context");
    c->ar = fn;
    c->ar_user = user;
    return SFMX_OK;
}

int sfmx_ba_run(sfmx_ba_ctx* c, int32_t max_iterations, sfmx_ba_summary* summary, double* trace, int32_t trace_cap) {
    if (!c || !summary) return fail(SFMX_EINVAL, "null context/summary");
    int nt = 0;
    RC(run_lm(c, max_iterations, summary, trace, trace_cap, &nt));
    return nt;
}

int sfmx_ba_get(sfmx_ba_ctx* c, sfmx_ba_problem* pb) {
    if (!c || !pb) return fail(SFMX_EINVAL, "null context/problem");
    DeviceGuard dg(c->device);
    const double* x = c->x.as<double>();
    std::vector<double> pts(3 * (size_t)c->P);
    if (c->P) HIPCHK(hipMemcpyAsync(pts.data(), x, sizeof(double) * 3 * c->P, hipMemcpyDeviceToHost, c->st));
    if (c->C) HIPCHK(hipMemcpyAsync(pb->poses, x + c->ne, sizeof(double) * 6 * c->C, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemcpyAsync(pb->intr, x + c->ne + 6 * (size_t)c->C, sizeof(double) * c->K, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    for (int q = 0; q < c->P; ++q)
        for (int i = 0; i < 3; ++i) pb->points[3 * (size_t)c->pperm[q] + i] = pts[3 * (size_t)q + i];
    return SFMX_OK;
}

int sfmx_ba_set(sfmx_ba_ctx* c, const sfmx_ba_problem* pb) {
    if (!c || !pb) return fail(SFMX_EINVAL, "null context/problem");
    if (pb->n_points != c->P || pb->n_cams != c->C || pb->cam_model != c->K) return fail(SFMX_EINVAL, "topology mismatch");
    return set_params(c, pb);
}

int sfmx_ba_phase_ms(sfmx_ba_ctx* c, double* ms, int32_t n) {
    if (!c || !ms) return fail(SFMX_EINVAL, "null");
    const int m = std::min<int>(n, 4);
    for (int i = 0; i < m; ++i) ms[i] = c->phase_ms[i];
    return m;
}

int sfmx_ba_destroy(sfmx_ba_ctx* c) {
    delete c;
    return SFMX_OK;
}

int sfmx_ba_solve(sfmx_ba_problem* pb, const sfmx_ba_options* opt, sfmx_ba_summary* summary, double* trace,
                  int32_t trace_cap) {
    if (!summary) return fail(SFMX_EINVAL, "null summary");
    sfmx_ba_ctx* c = nullptr;
    RC(create(pb, opt, &c));
    int nt = 0;
    int rc = run_lm(c, 0, summary, trace, trace_cap, &nt);
    if (!rc) rc = sfmx_ba_get(c, pb);   // write-back (BundleAdjustment.cpp:97-138)
    delete c;
    return rc ? rc : nt;
}

int sfmx_ba_jacobian(const sfmx_ba_problem* pb, int32_t device, double* r, double* Je, double* Jc, double* Ji) {
    sfmx_ba_options o;
    sfmx_ba_default_options(&o);
    o.device = device;
    sfmx_ba_ctx* c = nullptr;
    RC(create(pb, &o, &c));
    int rc = SFMX_OK;
    {
        DeviceGuard dg(c->device);
        double cost;
        rc = eval<true>(c, c->x.as<double>(), &cost);
        if (!rc) {
            const int O = c->O, K = c->K, F = 20 + 2 * K;
            std::vector<double> h((size_t)F * O);
            if (O && (hipMemcpy(h.data(), c->J.p, sizeof(double) * h.size(), hipMemcpyDeviceToHost) != hipSuccess))
                rc = fail(SFMX_EDEVICE, "D2H");
            for (int q = 0; q < O && !rc; ++q) {
                const size_t o = (size_t)c->operm[q];   // caller's observation index
                for (int j = 0; j < 2; ++j) {
                    if (r) r[2 * o + j] = h[(size_t)q * F + j];
                    for (int i = 0; i < 3; ++i) if (Je) Je[6 * o + 3 * j + i] = h[(size_t)q * F + (2 + 3 * j + i)];
                    for (int i = 0; i < 6; ++i) if (Jc) Jc[12 * o + 6 * j + i] = h[(size_t)q * F + (8 + 6 * j + i)];
                    for (int i = 0; i < K; ++i) if (Ji) Ji[2 * (size_t)K * o + K * j + i] = h[(size_t)q * F + (20 + K * j + i)];
                }
            }
        }
    }
    delete c;
    return rc;
}

int sfmx_pose_to_ceres(const double* Rt, double* pose) {
    if (!Rt || !pose) return fail(SFMX_EINVAL, "null");
    // CeresUtils::toCeresPose (CeresUtils.h:119-148): column-major copy of R, then RotationMatrixToAngleAxis
    double R[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i + 3 * j] = Rt[4 * i + j];
    rotmat_to_aa(R, pose);
    for (int i = 0; i < 3; ++i) pose[3 + i] = Rt[4 * i + 3];
    return SFMX_OK;
}

int sfmx_pose_from_ceres(const double* pose, double* Rt) {
    if (!Rt || !pose) return fail(SFMX_EINVAL, "null");
    double R[9];   // CeresUtils::toOpenCvPose (CeresUtils.h:90-117)
    aa_to_rotmat(pose, R);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Rt[4 * i + j] = R[i + 3 * j];
        Rt[4 * i + 3] = pose[3 + i];
    }
    return SFMX_OK;
}

}  // extern "C"
