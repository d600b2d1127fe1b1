// SPDX-License-Identifier: MIT
// sfmx bundle adjustment — host driver behind include/sfmx_ba.h.
//
// Replaces BundleAdjustment::doBundleAdjustment (src/photogrammetrie/common/
// BundleAdjustment.cpp:29-141) + CeresUtils::solve (util/CeresUtils.cpp:38-56):
//   * problem assembly as flat arrays in O(observations), instead of one
//     OpenMpUtils::find_if parallel region per observation (BundleAdjustment.cpp:66-69);
//   * the Ceres 1.14 trust-region / Levenberg-Marquardt loop with DENSE_SCHUR on the
//     host, every numeric step in the HIP kernels of ba_group.hpp / ba_kernels.hpp; one
//     host round trip (8 scalars) per LM step.
// The controller mirrors oracle/ba_oracle.cpp (the CPU restatement) step for step.
//
// Per LM step (try_step), in stream order:
//   ba_gschur -> memset S -> ba_assemble -> [all-reduce S, R, D, r_i] -> ba_add_cam -> chol_factor
//   (the plan's elimination-tree schedule in one launch, ba_plan.hpp / ba_chol.hpp) -> chol_backsolve
//   -> ba_gupdate (+ the candidate cameras) -> ba_glin (the candidate, speculatively: its records are
//   the next linearization if the step is accepted) -> ba_camred -> [all-reduce] -> ba_finalize
//   (-> ba_publish: the scalars through pinned host-coherent memory) -> [all-reduce scalars].
#include "ba_group.hpp"
#include "ba_chol.hpp"
#include "ba_plan.hpp"
#include "diag.hpp"
#include "host_par.hpp"
#include "rccl_dl.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <mutex>
#include <string>
#include <cstdlib>
#include <cstdio>
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
                        std::string(#expr) + " (ba_solver.hip:" + std::to_string(__LINE__) + "): " + hipGetErrorString(e_)); \
    } while (0)
#define RC(expr) do { int rc_ = (expr); if (rc_) return rc_; } while (0)

// Device buffer that keeps its allocation across problems (sfmx_ba_update, the cached context of
// sfmx_ba_solve): alloc(b) reuses the block when it holds b bytes, else reallocates with 25 %
// headroom (a scene grows by a few cameras per BundleAdjustment call, SfM.cpp:235 / :371).
// A Buf with cap == 0 and p set is a view into another Buf's block (UploadSet below): never freed here.
struct Buf {
    void* p = nullptr;
    size_t bytes = 0, cap = 0;
    int alloc(size_t b) {
        b = std::max<size_t>(b, 64);
        if (p && b <= cap) { bytes = b; return SFMX_OK; }
        const size_t want = p && cap ? std::max(b, cap + cap / 2) : b;   // first allocation exact, regrowth with headroom
        if (p && cap) (void)hipFree(p);
        p = nullptr;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) { p = nullptr; cap = bytes = 0; return fail(SFMX_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)); }
        cap = want;
        bytes = b;
        return SFMX_OK;
    }
    void release() { if (p && cap) (void)hipFree(p); p = nullptr; cap = bytes = 0; }
    void set_view(void* q, size_t b) { release(); p = q; bytes = b; }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct HostScratch;                       // the host setup's vectors, kept between calls (below)
void destroy_scratch(HostScratch* h);
inline unsigned nblk(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }
constexpr int MAX_NPAD = 16 * 1024;   // rows of S_cc: the back solve keeps its vector in LDS

}  // namespace

struct sfmx_ba_ctx {
    int device = 0;
    hipStream_t st = nullptr;
    sfmx_ba_options opt{};
    int P = 0, C = 0, O = 0, K = 0;
    double cx = 0, cy = 0;
    // several cameras (sfmx_ba_problem.n_intr >= 1): border column j of x's intrinsics part holds the
    // caller's intr[isrc[j]] (the referenced blocks back to back, then zero padding up to K, -1);
    // per pose its block (pim = model | first column << 4) and principal point (pcc)
    bool multi = false;
    bool loaded = false;            // a problem is loaded (false after a failed update: run / get / set refuse)
    int n_intr = 0, intr_len = 0;   // caller's blocks and the length of its intr array
    std::vector<int> isrc;
    Buf pim, pcc;
    int64_t n = 0, ne = 0;
    int nf = 0, npad = 0, T = 0, RW = 0;
    sfmx_allreduce_fn ar = nullptr;
    void* ar_user = nullptr;
    ncclComm_t comm = nullptr;   // native RCCL (sfmx_ba_set_comm): the collectives go on the solver stream
    // topology: groups, chunks, group cameras, local camera per observation, assembly tasks
    int ngroups = 0, ntasks = 0, nslots = 0, gs_nt = 4;   // gs_nt: ba_gschur specialisation, dp_max / 16
    size_t lds_schur = 0, lds_lin = 0;
    Buf obs_point, obs_cam, obs_xy, pt_start, grp, chk, bat, gcam, obs_lc, obs_row, lcrow, tasks, ents, cref_start, cref;
    Buf obs_xy_b, obs_cam_b, obs_lc_b, obs_row_b, moves;   // the next layout's observation arrays; relayout moves
    Buf topo_arena, plan_arena;   // one block each for the load's topology arrays and the plan's (UploadSet)
    int64_t setup_up_obs = 0;    // observations the last load uploaded (the rest moved on the device)
    // factorization plan of the reduced camera system (one rank: built during the load; sharded: at the
    // first run, from the camera co-visibility of every rank -- the layout of S must be the same on all)
    std::vector<char> adj;       // local camera co-visibility, C x C
    bool planned = false;
    sfmx::ba::FactorPlan plan;
    Buf camrow, padrows, rowmap, leaves, ptasks, psrc, lvl_start, lvl_panels, bs_start, bs_k, Wt, contrib, xi,
        nztiles, packbuf,          // all-reduce of the nonzero lower tiles only (multi-rank)
        border, zbuf, dagctr,      // chol_backsolve: panels root first, z, [ticket, finished, zdone[T]]
        parts, pbuf, lctr,         // chol_level_split: (task, source) parts per level, product slots, arrivals
        ditems, dneed, dctr,       // chol_factor: leaves + every level's parts, their version needs, [ticket, finished, tver]
        dmask,                     // chol_factor: per item, the row masks of its operands (ba_plan.cpp row_masks)
        tpre;                      // per task: the panels swept before its update (r06 pre-sweep, every form)
    bool back_dag = true;          // SFMX_BA_BACK=0: the r02 chol_intr + one-workgroup chol_back
    bool split = true;             // SFMX_BA_SPLIT=0: chol_level (a task's sources in one workgroup)
    std::vector<int> part_start;   // per level: parts[part_start[l] .. part_start[l + 1])
    bool dag = true;               // SFMX_BA_DAG=0: one launch per level (chol_leaves + chol_level[_split])
    bool wide = false;             // SFMX_BA_WIDE=1 (diagnostic): chol_factor_w on NW x NW waves instead of chol_factor
    int n_ditems = 0, n_ver = 0;
    long long dag_timeout = DAG_TIMEOUT;   // in-launch wait bound (wall-clock ticks without progress)
    int dag_fallbacks = 0;                 // steps re-run with the per-level launches after a wait timed out
    int n_nztiles = 0;
    size_t sr_count = 0;         // doubles of SR = S_cc | R | D | r_i
    // state (the *2 buffers hold the candidate's linearization until the step is accepted)
    // Wr / PR: the step kernels' records of a linearization (W_o per observation, E | g | V per
    // point, ba_group.hpp); J: Jacobian rows, for sfmx_ba_jacobian only (allocated there)
    Buf x, cand, scale, colsq, colsq2, grad, grad2, Wr, Wr2, PR, PR2, J, camsum, camsum2, plt, sg, rg, hbig, gpart, gpl,
        scal, SR, sol, failf, partA;
    static constexpr int HS_SLOT = SC_N + LM_N, HS_SEQ = 2 * HS_SLOT, HS_N = HS_SEQ + 3;
    bool scaled = false;
    // the Wr buffer that holds the iteration-0 records, still unscaled (Jacobi scaling on) until the
    // solve's first accepted step: steps on it read them through ba_gschur / ba_gupdate <SCALEJ>
    void* unscaled_wr = nullptr;
    // locality order: internal point p' is caller point pperm[p']; internal
    // observation o' is caller observation operm[o'] (point-major)
    std::vector<int> pperm, operm;
    double phase_ms[4] = {0, 0, 0, 0};
    bool phases = false;         // per-phase events (sfmx_ba_set_phase_timing): ~6 us of GPU time each
    hipEvent_t ev[6] = {};
    double* hs = nullptr;        // pinned host-coherent: 2 slots of [scalars SC_N | LM state LM_N], their
                                 // sequence words (HS_SEQ + slot) and ba_publish's sequence word (HS_SEQ + 2)
    Buf lmst;                    // device LM state (speculative mode, ba_decide)
    Buf camscr;                  // camera sums of a linearization before the all-reduce (scratch)
    bool spec = false;           // SFMX_BA_SPEC=1: device-judged steps, step s + 1 enqueued before s is judged
    int spec_maxit = 0;
    double lm_init[LM_N] = {};   // host source of the initial device LM state (outlives its async copy)
    unsigned seq = 0;
    // uploads go through a pinned staging arena (bump-allocated; the stream is synchronised before
    // it is reused), not pageable memory
    char* stage = nullptr;
    size_t stage_cap = 0, stage_off = 0;
    // host-side setup of the last create / update (include/sfmx_ba.h sfmx_ba_setup_ms): [0] ordering +
    // topology, [1] device allocation, [2] uploads, [3] factorization plan, [4] total (ms), [5] the host
    // ordering / grouping pass alone (ms), [6] buckets redone (a count), [7] validation (ms), [8 .. 15]
    // host_setup's phases (HostScratch::tm), [16] the plan's host computation, [17] the load's final
    // stream wait (ms)
    static constexpr int SETUP_N = 20;   // [18] the parameters' staging + copies, [19] the topology arrays' (ms)
    double setup_ms[SETUP_N] = {};
    std::vector<char> plan_adj;   // the co-visibility the current plan was built from (reused if equal)
    // r05: one rank's plan of a new co-visibility is computed on its own thread while the rest of the
    // load (topology, uploads) runs; ensure_plan takes it when the graph and the mode match
    sfmx::SideThread* plan_th = nullptr;   // (created on first use)
    bool plan_pending = false;
    sfmx::ba::FactorPlan plan_pre;
    std::vector<char> plan_pre_adj;
    int plan_pre_mode = -2;
    std::string plan_form;        // diagnostic library: the form switches the plan was built with
    int plan_K = 0;
    HostScratch* hscr = nullptr;
    ~sfmx_ba_ctx() {
        Buf* all[] = {&topo_arena, &plan_arena, &obs_xy_b, &obs_cam_b, &obs_lc_b, &obs_row_b, &moves, &obs_point, &obs_cam, &obs_xy, &pt_start, &grp, &chk, &bat, &gcam, &obs_lc, &obs_row, &lcrow, &tasks,
                      &ents, &cref_start, &cref, &camrow, &padrows, &rowmap, &leaves, &ptasks, &psrc, &lvl_start,
                      &lvl_panels, &bs_start, &bs_k, &Wt, &contrib, &xi, &nztiles, &packbuf, &border, &zbuf, &dagctr, &parts, &pbuf, &lctr, &ditems, &dneed, &dctr, &dmask, &tpre, &x, &cand, &scale, &colsq, &colsq2, &grad,
                      &grad2, &Wr, &Wr2, &PR, &PR2, &J, &camsum, &camsum2, &plt, &sg, &rg, &hbig, &gpart, &gpl, &scal, &SR, &sol,
                      &failf, &partA, &lmst, &camscr, &pim, &pcc};
        if (plan_th) { plan_th->wait(); delete plan_th; }
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        for (Buf* b : all) b->release();
        for (auto& e : ev) if (e) (void)hipEventDestroy(e);
        if (comm) (void)sfmx::rccl_api().CommDestroy(comm);
        if (st) (void)hipStreamDestroy(st);
        if (hs) (void)hipHostFree(hs);
        if (stage) (void)hipHostFree(stage);
        destroy_scratch(hscr);
        (void)hipSetDevice(prev);
    }
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) { (void)hipGetDevice(&prev); (void)hipSetDevice(d); }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// The solve's collectives: native RCCL on the solver's stream when a communicator is set
// (sfmx_ba_set_comm), else the caller's callback (sfmx_ba_set_allreduce, e.g. gloo in tests).
int allreduce(sfmx_ba_ctx* c, double* buf, int64_t count, int op) {
    if (count <= 0) return SFMX_OK;
    if (c->comm) {
        const sfmx::RcclApi& r = sfmx::rccl_api();
        const ncclResult_t e = r.AllReduce(buf, buf, (size_t)count, ncclFloat64, op == SFMX_REDUCE_SUM ? ncclSum : ncclMax,
                                           c->comm, c->st);
        if (e != ncclSuccess) return fail(SFMX_EDEVICE, std::string("ncclAllReduce: ") + r.GetErrorString(e));
        return SFMX_OK;
    }
    if (!c->ar) return SFMX_OK;
    if (c->ar(buf, count, op, c->ar_user, (void*)c->st) != 0) return fail(SFMX_EDEVICE, "all-reduce callback failed");
    return SFMX_OK;
}

// bytes of pinned staging for one upload; the arena restarts (after a stream sync) when full
void* stage_bytes(sfmx_ba_ctx* c, size_t n) {
    n = (n + 255) & ~(size_t)255;
    if (c->stage_off + n > c->stage_cap) {
        if (hipStreamSynchronize(c->st) != hipSuccess) return nullptr;
        c->stage_off = 0;
        if (n > c->stage_cap) {
            if (c->stage) (void)hipHostFree(c->stage);
            c->stage = nullptr;
            c->stage_cap = std::max(n, c->stage_cap * 2);
            if (hipHostMalloc(reinterpret_cast<void**>(&c->stage), c->stage_cap, hipHostMallocDefault) != hipSuccess) {
                c->stage_cap = 0;
                return nullptr;
            }
        }
    }
    void* p = c->stage + c->stage_off;
    c->stage_off += n;
    return p;
}

// the arena sized for a whole call's uploads at once (else a full arena waits for the DMAs in flight)
int stage_reserve(sfmx_ba_ctx* c, size_t n) {
    if (c->stage_off + n <= c->stage_cap) return SFMX_OK;
    HIPCHK(hipStreamSynchronize(c->st));
    c->stage_off = 0;
    if (n > c->stage_cap) {
        if (c->stage) (void)hipHostFree(c->stage);
        c->stage = nullptr;
        c->stage_cap = n + n / 4;
        if (hipHostMalloc(reinterpret_cast<void**>(&c->stage), c->stage_cap, hipHostMallocDefault) != hipSuccess) {
            c->stage_cap = 0;
            return fail(SFMX_ENOMEM, "pinned staging buffer");
        }
    }
    return SFMX_OK;
}

// Several host arrays to the device in ONE copy (r05: every hipMemcpyAsync costs ~5-10 us of host
// time, and a load made ~25 of them): each array at a 256-B aligned offset of one device block
// (`arena`, regrown like any Buf), its Buf a view of that range.  add() keeps a pointer (the array
// must live until flush) or, with copy = true, a copy.
struct UploadSet {
    struct Part { Buf* dst; const void* src; size_t bytes; std::vector<char> own; };
    std::vector<Part> parts;
    template <class V>
    void add(Buf& dst, const V& v, bool copy = false) {
        Part pt{&dst, v.data(), sizeof(v[0]) * v.size(), {}};
        if (copy) {
            pt.own.assign(reinterpret_cast<const char*>(v.data()), reinterpret_cast<const char*>(v.data()) + pt.bytes);
            pt.src = pt.own.data();
        }
        parts.push_back(std::move(pt));
    }
    int flush(sfmx_ba_ctx* c, Buf& arena) {
        if (parts.empty()) return SFMX_OK;
        auto r = [](size_t b) { return (std::max<size_t>(b, 1) + 255) & ~(size_t)255; };
        std::vector<size_t> off(parts.size() + 1, 0);
        for (size_t i = 0; i < parts.size(); ++i) off[i + 1] = off[i] + r(parts[i].bytes);
        RC(arena.alloc(off.back()));
        char* h = static_cast<char*>(stage_bytes(c, off.back()));
        if (!h) return fail(SFMX_ENOMEM, "pinned staging buffer");
        // the copies into pinned memory in 256 KiB pieces on the worker pool
        std::vector<std::pair<int, size_t>> pieces;
        for (size_t i = 0; i < parts.size(); ++i)
            for (size_t b = 0; b < parts[i].bytes; b += (size_t)1 << 18) pieces.emplace_back((int)i, b);
        sfmx::parallel_items((int)pieces.size(), [&](int k) {
            const Part& pt = parts[pieces[k].first];
            const size_t b0 = pieces[k].second, n = std::min(pt.bytes - b0, (size_t)1 << 18);
            std::memcpy(h + off[pieces[k].first] + b0, static_cast<const char*>(pt.src) + b0, n);
        });
        HIPCHK(hipMemcpyAsync(arena.p, h, off.back(), hipMemcpyHostToDevice, c->st));
        for (size_t i = 0; i < parts.size(); ++i) parts[i].dst->set_view(arena.as<char>() + off[i], std::max<size_t>(parts[i].bytes, 64));
        parts.clear();
        return SFMX_OK;
    }
};

bool multirank(const sfmx_ba_ctx* c) { return c->ar != nullptr || c->comm != nullptr; }
double* scal(sfmx_ba_ctx* c, int i) { return c->scal.as<double>() + i; }
int* gate(sfmx_ba_ctx* c) { return c->failf.as<int>() + 1; }   // the step gate word (ba_kernels.hpp step_gated)

int fetch_scalars(sfmx_ba_ctx* c, int i0, int cnt, double* out) {
    HIPCHK(hipMemcpyAsync(out, scal(c, i0), sizeof(double) * cnt, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return SFMX_OK;
}

// The LM step's scalars: ba_publish writes them to pinned memory behind everything queued so far
// and the host spins on the sequence word (a stream error or a drained stream without the word
// ends the wait).
// published: ba_finalize already published sequence number `published` (one rank, no phase mark)
int poll_scalars(sfmx_ba_ctx* c, double* out, hipEvent_t mark, unsigned published = 0) {
    const unsigned want = published ? published : ++c->seq;
    unsigned* hseq = reinterpret_cast<unsigned*>(c->hs + sfmx_ba_ctx::HS_SEQ + 2);
    if (!published) {
        if (mark) HIPCHK(hipEventRecord(mark, c->st));
        hipLaunchKernelGGL(ba_publish, dim3(1), dim3(64), 0, c->st, scal(c, 0), (int)SC_N, c->hs, hseq, want,
                           c->failf.as<int>());
        HIPCHK(hipGetLastError());
    }
    for (unsigned spins = 1;; ++spins) {
        if (__atomic_load_n(hseq, __ATOMIC_ACQUIRE) == want) break;
        if ((spins & 255) == 0) {
            const hipError_t e = hipStreamQuery(c->st);
            if (e != hipSuccess && e != hipErrorNotReady) return fail(SFMX_EDEVICE, std::string("LM step: ") + hipGetErrorString(e));
            if (e == hipSuccess && __atomic_load_n(hseq, __ATOMIC_ACQUIRE) != want)
                return fail(SFMX_EINTERNAL, "LM step: stream drained without the scalar handoff");
        }
        __builtin_ia32_pause();
    }
    std::memcpy(out, c->hs, sizeof(double) * SC_N);
    return SFMX_OK;
}

// Speculative mode: wait for ba_decide's publication with sequence number q (slot q & 1) -> out[HS_SLOT].
int wait_slot(sfmx_ba_ctx* c, unsigned q, double* out) {
    unsigned* hseq = reinterpret_cast<unsigned*>(c->hs + sfmx_ba_ctx::HS_SEQ + (q & 1));
    for (unsigned spins = 1;; ++spins) {
        if (__atomic_load_n(hseq, __ATOMIC_ACQUIRE) == q) break;
        if ((spins & 255) == 0) {
            const hipError_t e = hipStreamQuery(c->st);
            if (e != hipSuccess && e != hipErrorNotReady) return fail(SFMX_EDEVICE, std::string("LM step: ") + hipGetErrorString(e));
            if (e == hipSuccess && __atomic_load_n(hseq, __ATOMIC_ACQUIRE) != q)
                return fail(SFMX_EINTERNAL, "LM step: stream drained without the step's publication");
        }
        __builtin_ia32_pause();
    }
    std::memcpy(out, c->hs + (q & 1) * sfmx_ba_ctx::HS_SLOT, sizeof(double) * sfmx_ba_ctx::HS_SLOT);
    return SFMX_OK;
}

// 1/2 sum ||r||^2 at parameters xp with the Jacobian into c->partA-sized J (sfmx_ba_jacobian only).
int eval_jacobian(sfmx_ba_ctx* c, const double* xp, double* cost_out) {
    const unsigned g = nblk(c->O);
    RC(c->J.alloc(8 * (size_t)std::max(c->O, 1) * jst(c->K)));
    const double* pts = xp;
    const double* poses = xp + c->ne;
    const double* intr = poses + 6 * (size_t)c->C;
#define LIN(KK) hipLaunchKernelGGL((ba_linearize<KK, true>), dim3(g), dim3(256), 0, c->st, c->O, c->obs_point.as<int>(), \
                                   c->obs_cam.as<int>(), c->obs_xy.as<double>(), c->cx, c->cy, pts, poses, intr,         \
                                   c->J.as<double>(), c->partA.as<double>(), c->multi ? c->pim.as<int>() : nullptr,      \
                                   c->multi ? c->pcc.as<double2>() : nullptr)
    if (c->K == 1) LIN(1); else if (c->K == 3) LIN(3); else LIN(7);
#undef LIN
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(ba_sum, dim3(1), dim3(256), 0, c->st, c->partA.as<double>(), (int)g, 0.5, scal(c, 0));
    RC(fetch_scalars(c, 0, 1, cost_out));
    return SFMX_OK;
}

// Linearization at xp (x or the candidate) into (Jo, colsq_o, grad_o, camsum_o) and the LM scalars
// into scal (cand_mode: the step's model / step-norm partials are already in gpl): -> out[SC_N].
template <int K>
int lin_at(sfmx_ba_ctx* c, const double* xp, double* Wo, double* PRo, double* colsq_o, double* grad_o,
           double* camsum_o, bool cand_mode, double* out) {
    if (c->ngroups > 0) {
#define GLIN(MULTI) hipLaunchKernelGGL((ba_glin<K, MULTI>), dim3(c->ngroups), dim3(256), c->lds_lin, c->st, c->grp.as<Grp>(), \
                           c->chk.as<Chunk>(), c->lcrow.as<int>(), c->obs_lc.as<short>(), c->obs_row.as<short>(),         \
                           c->obs_point.as<int>(), c->obs_cam.as<int>(),                                                   \
                           c->obs_xy.as<double>(), c->pt_start.as<int>(), c->cx, c->cy, c->P, c->C, xp,                    \
                           c->scaled ? c->scale.as<double>() : nullptr, Wo, PRo, colsq_o, grad_o, c->gpart.as<double>(),   \
                           c->gpl.as<double>(), gate(c), c->pim.as<int>(), c->pcc.as<double2>())
        if (c->multi) GLIN(true); else GLIN(false);
#undef GLIN
    }
    // multi-rank speculative steps all-reduce a scratch copy of the camera sums: a skipped step's
    // all-reduce then touches no state (ba_finalize copies them behind the step gate)
    const int ncs = c->C * ncp(K) + K * (K + 1) / 2 + K;
    double* cs_red = (multirank(c) && c->spec) ? c->camscr.as<double>() : camsum_o;
    if (c->C) hipLaunchKernelGGL(ba_camred<K>, dim3(c->C), dim3(CRED_THREADS), 0, c->st, c->C, c->nslots, c->cref_start.as<int>(),
                       c->cref.as<int>(), c->gpart.as<double>(), cs_red, gate(c));
    HIPCHK(hipGetLastError());
    // multi-rank: the group sums ride in the camera-sum all-reduce (cs_red[ncs .. ncs + 4), the
    // rank's point max |grad| at cs_red[ncs + 4] outside it): 3 collectives per LM step, not 4
    double* pre = multirank(c) ? cs_red + ncs : nullptr;
    if (pre)
        hipLaunchKernelGGL(ba_group_sums, dim3(1), dim3(1024), 0, c->st, c->ngroups, c->gpl.as<double>(), pre, gate(c));
    RC(allreduce(c, cs_red, ncs + (pre ? 4 : 0), SFMX_REDUCE_SUM));
    // one rank, host-judged, no phase mark: ba_finalize publishes the scalars itself (one launch fewer)
    const bool fold = out && !multirank(c) && !(c->phases && cand_mode);
    const unsigned fold_seq = fold ? ++c->seq : 0;
    hipLaunchKernelGGL(ba_finalize<K>, dim3(1), dim3(1024), 0, c->st, c->ngroups, c->P, c->C, cs_red,
                       c->gpl.as<double>(), xp + c->ne, c->x.as<double>() + c->ne, cand_mode ? 1 : 0, c->failf.as<int>(),
                       colsq_o, grad_o, scal(c, 0), camsum_o, cs_red == camsum_o ? 0 : ncs, pre,
                       fold ? c->hs : nullptr, reinterpret_cast<unsigned*>(c->hs + sfmx_ba_ctx::HS_SEQ + 2), fold_seq,
                       c->camsum.as<double>(), c->sol.as<double>() + c->ne, c->scale.as<double>() + c->ne);
    HIPCHK(hipGetLastError());
    RC(allreduce(c, scal(c, SC_GMAX), 2, SFMX_REDUCE_MAX));
    if (!out) return SFMX_OK;   // speculative step: ba_decide judges and publishes
    RC(poll_scalars(c, out, c->phases && cand_mode ? c->ev[3] : nullptr, fold ? fold_seq : 0));
    return SFMX_OK;
}

// One LM step at `radius`: Schur solve of (J_s^T J_s + D^2) sol = J_s^T r, step_s = -sol,
// candidate = x + step_s * scale, its cost, Jacobian and scalars (speculative linearization).
// The level-scheduled solve of the bordered reduced system (ba_chol.hpp) -> sol (natural order).
template <int RW>
int solve_reduced(sfmx_ba_ctx* c, double* sol_f) {
    const sfmx::ba::FactorPlan& pl = c->plan;
    const int npad = c->npad;
    double* S = c->SR.as<double>();
    double* R = S + (size_t)npad * npad;
    double* Dm = R + (size_t)npad * RW;
    double* ri = Dm + (RW - 1) * (RW - 1);
    int* fl = c->failf.as<int>();
    // the wide form within 128 VGPRs: k = 1, 3 (RW = 8 would spill: k = 7 keeps chol_factor)
    constexpr bool WIDE_OK = RW <= 4;
    if (WIDE_OK && c->dag && c->split && c->wide) {
        if constexpr (WIDE_OK)
            hipLaunchKernelGGL(chol_factor_w<RW>, dim3((unsigned)c->n_ditems), dim3(NTW), 0, c->st, S, npad, R,
                               c->ptasks.as<int4>(), c->ditems.as<int4>(), c->dneed.as<int4>(), c->psrc.as<int>(),
                               c->Wt.as<double>(), c->contrib.as<double>(), fl, c->pbuf.as<double>(), c->lctr.as<int>(),
                               c->dctr.as<int>(), c->n_ditems, c->n_ver, c->dag_timeout);
    } else if (c->dag && c->split) {
        hipLaunchKernelGGL(chol_factor<RW>, dim3((unsigned)c->n_ditems), dim3(NTH), 0, c->st, S, npad, R,
                           c->ptasks.as<int4>(), c->ditems.as<int4>(), c->dneed.as<int4>(), c->psrc.as<int>(),
                           c->Wt.as<double>(), c->contrib.as<double>(), fl, c->pbuf.as<double>(), c->lctr.as<int>(),
                           c->dctr.as<int>(), c->n_ditems, c->n_ver, c->dag_timeout, c->dmask.as<int4>());
    } else {
    hipLaunchKernelGGL(chol_leaves<RW>, dim3((unsigned)pl.leaves.size()), dim3(NTH), 0, c->st, S, npad, R,
                       c->leaves.as<int>(), c->Wt.as<double>(), c->contrib.as<double>(), fl);
    for (int l = 0; l < pl.height; ++l) {
        const int t0 = pl.task_start[l], nt = pl.task_start[l + 1] - t0;
        if (c->split) {
            const int p0 = c->part_start[l], np = c->part_start[l + 1] - p0;
            hipLaunchKernelGGL(chol_level_split<RW>, dim3(np), dim3(NTH), 0, c->st, S, npad, R, c->ptasks.as<int4>(),
                               c->parts.as<int4>() + p0, c->psrc.as<int>(), c->Wt.as<double>(), c->contrib.as<double>(),
                               fl, c->pbuf.as<double>(), c->lctr.as<int>(), c->tpre.as<int>());
        } else {
            hipLaunchKernelGGL(chol_level<RW>, dim3(nt), dim3(NTH), 0, c->st, S, npad, R, c->ptasks.as<int4>() + t0,
                               c->psrc.as<int>(), pl.ninv[l], c->Wt.as<double>(), c->contrib.as<double>(), fl,
                               c->tpre.as<int>() + t0);
        }
    }
    }
    if (c->back_dag) {
        hipLaunchKernelGGL(chol_backsolve<RW>, dim3(c->T), dim3(NTH), 0, c->st, S, npad, R, Dm, ri,
                           c->contrib.as<double>(), c->T, c->border.as<int>(), c->bs_start.as<int>(), c->bs_k.as<int>(),
                           c->rowmap.as<int>(), c->zbuf.as<double>(), sol_f, sol_f + 6 * (size_t)c->C,
                           c->dagctr.as<int>(), fl, c->dag_timeout);
    } else {
        hipLaunchKernelGGL(chol_intr<RW - 1>, dim3(1), dim3(64), 0, c->st, Dm, ri, c->contrib.as<double>(), c->T,
                           c->xi.as<double>(), sol_f + 6 * (size_t)c->C, fl);
        hipLaunchKernelGGL(chol_back<RW>, dim3(1), dim3(1024), sizeof(double) * npad, c->st, S, npad, R,
                           c->xi.as<double>(), pl.height, c->lvl_start.as<int>(), c->lvl_panels.as<int>(),
                           c->bs_start.as<int>(), c->bs_k.as<int>(), c->rowmap.as<int>(), sol_f, gate(c));
    }
    HIPCHK(hipGetLastError());
    return SFMX_OK;
}

constexpr unsigned GUPDATE_LDS = 33 * 1024;   // + 6.1 KB static: 4 x 39 KB fit 160 KiB, 5 do not

// One LM step at `radius`: Schur solve of (J_s^T J_s + D^2) sol = J_s^T r, step_s = -sol,
// candidate = x + step_s * scale, its cost, Jacobian and scalars (speculative linearization).
// spec: speculative mode (the device LM state supplies the radius; ba_decide judges the step and
// publishes with sequence number spec_seq); otherwise the host reads the scalars and judges.
template <int K>
int try_step(sfmx_ba_ctx* c, double radius, bool* valid, double* mcc, double* step_norm, double* ccost,
             double* cgmax, double* cxnorm, bool spec = false, unsigned spec_seq = 0) {
    constexpr int RW = K + 1;
    const double* lmr = spec ? c->lmst.as<double>() : nullptr;
    const int C = c->C, npad = c->npad;
    double* S = c->SR.as<double>();
    double* R = S + (size_t)npad * npad;
    double* Dm = R + (size_t)npad * RW;
    double* ri = Dm + K * K;
    int* fl = c->failf.as<int>();
    const sfmx_ba_options& o = c->opt;
    // the failure flag is zero here: cleared by the run's start and by every scalar handoff (ba_publish)
    if (c->phases) HIPCHK(hipEventRecord(c->ev[0], c->st));
    const bool sj = c->unscaled_wr && c->Wr.p == c->unscaled_wr;   // a step on the unscaled iteration-0 records
    const long long sr_tail = (long long)(c->sr_count - (size_t)npad * npad);
    {   // (r06: ba_gschur's workgroups past the groups zero S's nonzero tiles and its tail; no S memset)
#define GSCHUR(NTV) if (sj) GSCHUR2(NTV, true); else GSCHUR2(NTV, false)
#define GSCHUR2(NTV, SJ) hipLaunchKernelGGL((ba_gschur<K, NTV, SJ>), dim3(c->ngroups + c->n_nztiles + 1), dim3(256), c->lds_schur, c->st, \
                           c->grp.as<Grp>(), c->bat.as<Batch>(), c->gcam.as<int>(), c->obs_lc.as<short>(),             \
                           c->obs_point.as<int>(), c->obs_cam.as<int>(), c->pt_start.as<int>(), c->Wr.as<double>(),     \
                           c->PR.as<double>(), c->scale.as<double>(), c->colsq.as<double>(), o.min_lm_diagonal,         \
                           o.max_lm_diagonal, radius,                                                                   \
                           c->P, C, c->plt.as<double>(), c->sg.as<double>(), c->rg.as<double>(), c->hbig.as<double>(), fl, lmr, \
                           c->ngroups, S, npad, c->nztiles.as<int2>(), c->n_nztiles, sr_tail, c->rowmap.as<int>())
        switch (c->gs_nt) { case 1: GSCHUR(1); break; case 2: GSCHUR(2); break; case 3: GSCHUR(3); break; default: GSCHUR(4); }
#undef GSCHUR2
#undef GSCHUR
    }
    // one rank: ba_assemble adds ba_add_cam's camera terms to its outputs itself (r06: one launch fewer);
    // point-sharded ranks add them after the all-reduce (they are replicated, not sharded)
    // diagnostic library: SFMX_BA_FUSE = the terms ba_assemble adds (bit 0 camera blocks, 1 camera B rows
    // and gradient, 2 intrinsics); the rest stay with ba_add_cam
    const char* nf_env = SFMX_DIAG_ENV("SFMX_BA_FUSE");
    const int fuse_mask = multirank(c) ? 0 : nf_env ? (std::atoi(nf_env) & 7) : 7;
    const bool fuse_cam = fuse_mask == 7;
    hipLaunchKernelGGL(ba_assemble, dim3(c->ntasks), dim3(ASM_THREADS), 0, c->st, c->tasks.as<ATask>(), c->ents.as<AEnt>(),
                       c->sg.as<double>(), c->hbig.as<double>(), c->rg.as<double>(), K, c->camrow.as<int>(), npad, S,
                       R, Dm, ri, gate(c), fuse_mask, c->P, C, c->camsum.as<double>(), c->scale.as<double>(),
                       c->colsq.as<double>(), o.min_lm_diagonal, o.max_lm_diagonal, radius, lmr);
    HIPCHK(hipGetLastError());
    if (c->phases) HIPCHK(hipEventRecord(c->ev[1], c->st));
    // point-sharded ranks: the group part of the reduced camera system and its rhs are sums over
    // ranks; only the structurally nonzero lower tiles (+ R, D, r_i) travel
    if (multirank(c)) {
        const int tail = (int)(c->sr_count - (size_t)npad * npad);
        hipLaunchKernelGGL(chol_pack, dim3(c->n_nztiles + 1), dim3(256), 0, c->st, S, npad, c->nztiles.as<int2>(),
                           c->n_nztiles, tail, c->packbuf.as<double>(), 0, gate(c));
        RC(allreduce(c, c->packbuf.as<double>(), (int64_t)c->n_nztiles * NB * NB + tail, SFMX_REDUCE_SUM));
        hipLaunchKernelGGL(chol_pack, dim3(c->n_nztiles + 1), dim3(256), 0, c->st, S, npad, c->nztiles.as<int2>(),
                           c->n_nztiles, tail, c->packbuf.as<double>(), 1, gate(c));
    }
    if (!fuse_cam)
    hipLaunchKernelGGL(ba_add_cam<K>, dim3(C + 1), dim3(64), 0, c->st, c->P, C, npad, c->camrow.as<int>(),
                       c->padrows.as<int>(), (int)c->plan.padrows.size(), c->camsum.as<double>(),
                       c->scale.as<double>(), c->colsq.as<double>(), o.min_lm_diagonal, o.max_lm_diagonal, radius, S,
                       R, Dm, ri, gate(c), lmr, fuse_mask);
    double* sol = c->sol.as<double>();
    RC(solve_reduced<RW>(c, sol + c->ne));
    if (c->phases) HIPCHK(hipEventRecord(c->ev[2], c->st));
    // the point update, and in workgroups past the groups the candidate cameras / intrinsics
    // An unused dynamic LDS request of GUPDATE_LDS holds it at 4 workgroups (4 waves per SIMD) per CU:
    // 52.8 us against 57-58 at the 5 its VGPRs allow, 64 at 6 and 61 at 3 (r04u..y)
#define GUPD(SJ) hipLaunchKernelGGL((ba_gupdate<K, SJ>), dim3(c->ngroups + nblk(c->nf)), dim3(256), GUPDATE_LDS, c->st, \
                       c->grp.as<Grp>(), c->chk.as<Chunk>(), c->obs_cam.as<int>(), c->obs_point.as<int>(),             \
                       c->pt_start.as<int>(), c->Wr.as<double>(), c->PR.as<double>(), c->scale.as<double>(),           \
                       c->plt.as<double>(), sol + c->ne, c->P, C, c->x.as<double>(), c->cand.as<double>(),               \
                       c->gpl.as<double>(), gate(c), c->ngroups, (int)c->nf)
    if (sj) GUPD(true); else GUPD(false);
#undef GUPD
    HIPCHK(hipGetLastError());
    double v[SC_N];
    RC(lin_at<K>(c, c->cand.as<double>(), c->Wr2.as<double>(), c->PR2.as<double>(), c->colsq2.as<double>(), c->grad2.as<double>(),
                 c->camsum2.as<double>(), true, spec ? nullptr : v));
    if (spec) {
        const sfmx_ba_options& op = c->opt;
        LmOpt lo{op.parameter_tolerance, op.function_tolerance, op.min_relative_decrease, op.max_trust_region_radius,
                 op.gradient_tolerance, op.min_trust_region_radius, c->spec_maxit, op.max_num_consecutive_invalid_steps,
                 SFMX_BA_CONVERGENCE, SFMX_BA_NO_CONVERGENCE, SFMX_BA_FAILURE};
        const int slot = spec_seq & 1;
        unsigned* hseq = reinterpret_cast<unsigned*>(c->hs + sfmx_ba_ctx::HS_SEQ + slot);
        hipLaunchKernelGGL(ba_decide, dim3(1), dim3(64), 0, c->st, scal(c, 0), c->lmst.as<double>(), c->failf.as<int>(),
                           lo, c->hs + slot * sfmx_ba_ctx::HS_SLOT, hseq, spec_seq);
        HIPCHK(hipGetLastError());
        return SFMX_OK;
    }
    if (v[SC_FAIL] >= 2.0) {
        // an in-launch dependency wait saw no progress for dag_timeout ticks (e.g. a preempted
        // queue): the step's solve is void, nothing of the state was touched (the step writes only
        // candidate buffers), so re-run it with the per-level launches, which have no waits
        const int fb = (int)v[SC_FAIL];
        if (c->dag || c->back_dag) {
            c->dag = false;
            c->back_dag = false;
            ++c->dag_fallbacks;
            return try_step<K>(c, radius, valid, mcc, step_norm, ccost, cgmax, cxnorm);
        }
        return fail(SFMX_EINTERNAL, std::string("BA solve: a dependency wait of the in-launch ") +
                                        ((fb & FAIL_FACTOR_WAIT) ? "factorization (chol_factor)" : "back solve (chol_backsolve)") +
                                        " timed out");
    }
    const double sn2 = v[SC_STEPN] + v[SC_STEPN_F];
    *mcc = -v[SC_MODEL];
    *step_norm = std::sqrt(sn2);
    *valid = v[SC_FAIL] == 0.0 && std::isfinite(sn2) && std::isfinite(v[SC_MODEL]) && *mcc > 0.0;
    *ccost = std::numeric_limits<double>::max();
    if (*valid) *ccost = std::isfinite(v[SC_COST]) ? v[SC_COST] : std::numeric_limits<double>::max();
    *cgmax = v[SC_GMAX];
    *cxnorm = std::sqrt(v[SC_XN] + v[SC_XN_F]);
    if (c->phases) {
        float a = 0, b = 0, d = 0;
        HIPCHK(hipEventSynchronize(c->ev[3]));
        HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
        HIPCHK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
        HIPCHK(hipEventElapsedTime(&d, c->ev[2], c->ev[3]));
        c->phase_ms[1] += a;
        c->phase_ms[2] += b;
        c->phase_ms[3] += d;
    }
    return SFMX_OK;
}

// The factorization plan, rebuilt when the co-visibility changes (one rank: during the load, beside its
// copies; sharded: at the first run, when the collectives are known -- setting them drops a plan): the
int plan_mode() {   // SFMX_BA_ORDER (diagnostic library): auto | natural | nd | nd1 | nd2 | nd4
    int mode = -1;
    if (const char* e = SFMX_DIAG_ENV("SFMX_BA_ORDER")) {
        const std::string m(e);
        mode = m == "natural" ? 0 : m == "nd" ? 1 : m == "nd1" ? 2 : m == "nd2" ? 3 : m == "nd4" ? 4 : -1;
    }
    return mode;
}

// camera co-visibility summed over ranks (every rank builds the same plan), the
// ordering and level schedule (SFMX_BA_ORDER: auto | natural | nd | nd1 | nd2 | nd4), the device
// copies of the schedule, and S / W / the Schur terms sized by it.
int ensure_plan(sfmx_ba_ctx* c) {
#ifdef SFMX_DIAG
    // the diagnostic library's form switches are read when a plan is built: a cached context (the
    // per-device one of sfmx_ba_solve) re-plans when they change, so a test that switches forms
    // between solves really runs each form
    std::string form;
    for (const char* k : {"SFMX_BA_ORDER", "SFMX_BA_BACK", "SFMX_BA_SPEC", "SFMX_BA_DAG", "SFMX_BA_DAG_TIMEOUT", "SFMX_BA_WIDE",
                          "SFMX_BA_SPLIT"}) {
        const char* v = SFMX_DIAG_ENV(k);
        form += std::string(k) + "=" + (v ? v : "") + ";";
    }
    if (c->planned && form != c->plan_form) c->planned = false;
    c->plan_form = form;
#endif
    if (c->planned) return SFMX_OK;
    const auto t_plan = std::chrono::steady_clock::now();
    const int C = c->C;
    std::vector<char> adj = c->adj;
    if (multirank(c) && C > 1) {   // global co-visibility: sum of the ranks' upper triangles
        std::vector<double> h((size_t)C * (C - 1) / 2);
        for (int a = 0, e = 0; a < C; ++a)
            for (int b = a + 1; b < C; ++b, ++e) h[e] = adj[(size_t)a * C + b] ? 1.0 : 0.0;
        Buf& d = c->SR;   // scratch until S is sized below
        RC(d.alloc(sizeof(double) * h.size()));
        HIPCHK(hipMemcpyAsync(d.p, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice, c->st));
        RC(allreduce(c, d.as<double>(), (int64_t)h.size(), SFMX_REDUCE_SUM));
        HIPCHK(hipMemcpyAsync(h.data(), d.p, sizeof(double) * h.size(), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        for (int a = 0, e = 0; a < C; ++a)
            for (int b = a + 1; b < C; ++b, ++e) adj[(size_t)a * C + b] = adj[(size_t)b * C + a] = h[e] > 0.0;
    }
    const int mode = plan_mode();
    sfmx::ba::FactorPlan& pl = c->plan;
    const auto t_make = std::chrono::steady_clock::now();
    bool pre = false;
    if (c->plan_pending) {   // the load's plan, computed beside it (same graph and mode: the same plan)
        c->plan_th->wait();
        c->plan_pending = false;
        if (!multirank(c) && c->plan_pre_mode == mode && c->plan_pre_adj == adj) {
            std::swap(pl, c->plan_pre);
            pre = true;
        }
        c->plan_pre_mode = -2;
    }
    if (!pre) sfmx::ba::make_plan(C, adj, mode, pl);
    if (pl.npad > MAX_NPAD) sfmx::ba::make_plan(C, adj, 0, pl);   // padding past the back solve's LDS
    c->npad = pl.npad;
    c->T = pl.T;
    const int RW = c->RW, K = c->K;
    c->sr_count = (size_t)pl.npad * pl.npad + (size_t)pl.npad * RW + (size_t)K * K + K;
    std::vector<int4> tk(pl.tasks.size());
    for (size_t i = 0; i < tk.size(); ++i) tk[i] = make_int4(pl.tasks[i].a, pl.tasks[i].b, pl.tasks[i].s0, pl.tasks[i].s1);
    hipStream_t st = c->st;
    UploadSet up;   // every schedule array in one copy at the end (no launch reads them before)
    up.add(c->camrow, pl.camrow); up.add(c->padrows, pl.padrows); up.add(c->rowmap, pl.rowmap);
    up.add(c->leaves, pl.leaves); up.add(c->ptasks, tk); up.add(c->psrc, pl.src); up.add(c->lvl_start, pl.lvl_start);
    up.add(c->lvl_panels, pl.lvl_panels); up.add(c->bs_start, pl.bs_start); up.add(c->bs_k, pl.bs_k);
    RC(c->SR.alloc(sizeof(double) * c->sr_count));
    {   // nonzero lower tiles (diagonal included): the compact all-reduce payload
        std::vector<int2> nzt;
        for (int a = 0; a < pl.T; ++a)
            for (int b = 0; b <= a; ++b)
                if (pl.nz[(size_t)a * pl.T + b]) nzt.push_back(make_int2(a, b));
        c->n_nztiles = (int)nzt.size();
        up.add(c->nztiles, nzt, true);
        RC(c->packbuf.alloc(sizeof(double) * ((size_t)c->n_nztiles * NB * NB + (c->sr_count - (size_t)pl.npad * pl.npad))));
    }
    RC(c->Wt.alloc(sizeof(double) * (size_t)pl.T * NB * NB));
    RC(c->contrib.alloc(sizeof(double) * (size_t)pl.T * K * RW));
    RC(c->xi.alloc(sizeof(double) * K));
    {   // chol_backsolve: panels root first (level descending), so a workgroup only waits on earlier tickets
        std::vector<int> order;
        for (int l = pl.height; l >= 0; --l)
            for (int t = pl.lvl_start[l]; t < pl.lvl_start[l + 1]; ++t) order.push_back(pl.lvl_panels[t]);
        up.add(c->border, order, true);
        RC(c->zbuf.alloc(sizeof(double) * (size_t)pl.npad));
        RC(c->dagctr.alloc(sizeof(int) * (size_t)((pl.T + 2 + 3) / 4 * 4)));
        HIPCHK(hipMemsetAsync(c->dagctr.p, 0, c->dagctr.bytes, st));
        const char* e = SFMX_DIAG_ENV("SFMX_BA_BACK");
        c->back_dag = !(e && e[0] == '0');
        e = SFMX_DIAG_ENV("SFMX_BA_SPEC");   // opt-in: measured no faster (host turnaround)
        c->spec = e && e[0] == '1';
    }
    {   // chol_level_split: per level, the parts of the inverting tasks first (the plan's task order)
        std::vector<int4> parts;
        c->part_start.assign(1, 0);
        int max_slots = 1;
        for (int l = 0; l < pl.height; ++l) {
            int slot = 0;
            for (int t = pl.task_start[l]; t < pl.task_start[l + 1]; ++t) {
                const int n = pl.tasks[t].s1 - pl.tasks[t].s0, inv = (t - pl.task_start[l]) < pl.ninv[l];
                if (n == 1) { parts.push_back(make_int4(t, pl.tasks[t].s0, 0, 1 | inv << 16)); continue; }
                for (int j = 0; j < n; ++j) parts.push_back(make_int4(t, pl.tasks[t].s0 + j, slot + j, n | inv << 16));
                slot += n;
            }
            max_slots = std::max(max_slots, slot);
            c->part_start.push_back((int)parts.size());
        }
        up.add(c->parts, parts, true);
        // chol_factor: the leaves, then every level's parts in the same order, product slots unique over
        // the launch; need = the versions (finished tasks, leaf inverse included) of A_ak, A_bk, (k, k)
        // and of A_ab before the task.  A plan whose source tile is not final at its use (never built
        // by ba_plan) keeps the per-level launches.
        const int T = pl.T, nver = T * (T + 1) / 2;
        auto vid = [](int a, int b) { return a * (a + 1) / 2 + b; };
        std::vector<int> vfin(nver, 0), vcnt(nver, 0);
        // an inverse (leaf or inverting task) adds 2: once when W_k is stored, once at its end (R rows)
        for (int k : pl.leaves) vfin[vid(k, k)] += 2;
        for (int l = 0; l < pl.height; ++l)
            for (int t = pl.task_start[l]; t < pl.task_start[l + 1]; ++t)
                vfin[vid(pl.tasks[t].a, pl.tasks[t].b)] += 1 + ((t - pl.task_start[l]) < pl.ninv[l] ? 1 : 0);
        std::vector<int4> items, need, imask;
        const std::vector<sfmx::ba::RowMask>& smask = pl.src_mask;   // (made with the plan)
        const std::vector<int>& padp = pl.pad_panels;
        // r06: per task, the panels an inverting one-source task sweeps before its update (the ones
        // outside A_ak's row strips and not padding); every factorization form uses the same order
        std::vector<int> tpre(std::max<size_t>(pl.tasks.size(), 1), 0);
        for (int l = 0; l < pl.height; ++l)
            for (int t = pl.task_start[l]; t < pl.task_start[l + 1]; ++t) {
                const auto& tk = pl.tasks[t];
                const bool inv = (t - pl.task_start[l]) < pl.ninv[l];
                if (inv && tk.a == tk.b && tk.s1 - tk.s0 == 1)
                    tpre[t] = ~smask[tk.s0].ra & ((1 << NW) - 1) & ~padp[tk.a];
            }
        up.add(c->tpre, tpre, true);
        for (int k : pl.leaves) {
            items.push_back(make_int4(k, -1, 0, 0));
            need.push_back(make_int4(0, 0, 0, 0));
            imask.push_back(make_int4(padp[k] << 12, 0, 0, 0));
            vcnt[vid(k, k)] = 2;
        }
        int dslots = 0;
        bool dag_ok = (size_t)c->sr_count * 8 < (1u << 31) && (size_t)T * NB * NB * 8 < (1u << 31);   // 32-bit buffer offsets
        for (int l = 0; l < pl.height; ++l) {
            for (int t = pl.task_start[l]; t < pl.task_start[l + 1]; ++t) {
                const auto& tk = pl.tasks[t];
                const int n = tk.s1 - tk.s0, inv = (t - pl.task_start[l]) < pl.ninv[l];
                for (int j = 0; j < n; ++j) {
                    const int k = pl.src[tk.s0 + j];
                    dag_ok = dag_ok && k < tk.b && vcnt[vid(tk.a, k)] == vfin[vid(tk.a, k)] &&
                             vcnt[vid(tk.b, k)] == vfin[vid(tk.b, k)] && vcnt[vid(k, k)] == vfin[vid(k, k)];
                    items.push_back(make_int4(t, tk.s0 + j, n == 1 ? 0 : dslots + j, n | inv << 16));
                    {   // G's column tiles: all for a diagonal task (G^T is stored for the back solve), else
                        // the tiles holding A_bk's nonzero columns (the only ones G A_bk^T reads)
                        const sfmx::ba::RowMask& rm = smask[tk.s0 + j];
                        int gc = 0;
                        for (int c = 0; c < NW; ++c) gc |= ((rm.kb >> (4 * c)) & 15 ? 1 : 0) << c;
                        if (tk.a == tk.b) gc = (1 << NW) - 1;
                        const int pre = tpre[t];
                        imask.push_back(make_int4(rm.ra | rm.rb << 4 | gc << 8 | (inv ? padp[tk.a] << 12 : 0) | pre << 16,
                                                  rm.ka, rm.kb, 0));
                    }
                    need.push_back(make_int4(vfin[vid(tk.a, k)], tk.a == tk.b ? 0 : vfin[vid(tk.b, k)], vfin[vid(k, k)],
                                             vcnt[vid(tk.a, tk.b)]));
                }
                if (n > 1) dslots += n;
            }
            for (int t = pl.task_start[l]; t < pl.task_start[l + 1]; ++t)
                vcnt[vid(pl.tasks[t].a, pl.tasks[t].b)] += 1 + ((t - pl.task_start[l]) < pl.ninv[l] ? 1 : 0);
        }
        c->n_ditems = (int)items.size();
        c->n_ver = nver;
        up.add(c->ditems, items, true);
        up.add(c->dneed, need, true);
        up.add(c->dmask, imask, true);
        RC(c->dctr.alloc(sizeof(int) * (size_t)((nver + 2 + 3) / 4 * 4)));
        HIPCHK(hipMemsetAsync(c->dctr.p, 0, c->dctr.bytes, st));
        const char* ed = SFMX_DIAG_ENV("SFMX_BA_DAG");
        c->dag = dag_ok && !(ed && ed[0] == '0');
        if (const char* et = SFMX_DIAG_ENV("SFMX_BA_DAG_TIMEOUT")) c->dag_timeout = std::atoll(et);   // recovery test
        max_slots = std::max(max_slots, dslots);
        const int tpo = std::max(1, NTH / (NB * RW)), opt = NB * RW / (NTH / tpo);
        const size_t slot = std::max<size_t>((size_t)(4 * NW + opt) * NTH, (size_t)4 * NTW + (size_t)opt * NTH);   // chol_factor | _w
        RC(c->pbuf.alloc(sizeof(double) * (size_t)max_slots * slot));
        // chol_factor_w (SFMX_BA_WIDE=1, diagnostic build only): measured no faster (r04c / r04d: the 16-wave
        // diagonal inverse's barriers cost what the quarter-length products save; C5 0.627-0.631 vs
        // 0.613-0.616 ms per iteration for the r03 library, profiles/r04d_ab.txt)
        const char* ew = SFMX_DIAG_ENV("SFMX_BA_WIDE");
        c->wide = ew && ew[0] == '1';
        // [arrivals per task | chol_factor: per task, parts whose product / y terms are stored, at nitems +
        // task / 2 nitems + task]
        RC(c->lctr.alloc(sizeof(int) * (size_t)((pl.tasks.size() + 2 * (size_t)c->n_ditems + 4) / 4 * 4)));
        HIPCHK(hipMemsetAsync(c->lctr.p, 0, c->lctr.bytes, st));
        const char* e = SFMX_DIAG_ENV("SFMX_BA_SPLIT");
        c->split = !(e && e[0] == '0');
    }
    hipError_t e = hipSuccess;
#define BACKATTR(RWV) e = hipFuncSetAttribute((const void*)chol_back<RWV>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                              (int)(sizeof(double) * pl.npad))
    if (RW == 2) BACKATTR(2); else if (RW == 4) BACKATTR(4); else BACKATTR(8);
#undef BACKATTR
    if (e != hipSuccess) return fail(SFMX_EDEVICE, std::string("LDS attribute: ") + hipGetErrorString(e));
    RC(up.flush(c, c->plan_arena));
    const auto t_wait = std::chrono::steady_clock::now();
    c->setup_ms[16] = std::chrono::duration<double, std::milli>(t_wait - t_make).count();
    HIPCHK(hipStreamSynchronize(st));
    c->setup_ms[17] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wait).count();
    c->planned = true;
    c->plan_adj = c->adj;
    c->plan_K = c->K;
    const double pms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_plan).count();
    c->setup_ms[3] = pms;
    c->setup_ms[4] += pms;
    return SFMX_OK;
}

template <int K>
int run_lm_k(sfmx_ba_ctx* c, int max_iters, sfmx_ba_summary* sum, double* trace, int trace_cap, int* ntrace_out) {
    DeviceGuard dg(c->device);
    RC(ensure_plan(c));
    const auto t0 = std::chrono::steady_clock::now();
    const sfmx_ba_options& o = c->opt;
    const int maxit = max_iters > 0 ? max_iters : o.max_num_iterations;
    for (double& v : c->phase_ms) v = 0;
    c->scaled = false;   // Ceres computes the Jacobi scale at iteration 0 of each Solve
    HIPCHK(hipEventRecord(c->ev[4], c->st));
    HIPCHK(hipMemsetAsync(c->failf.p, 0, sizeof(int), c->st));
    hipLaunchKernelGGL(ba_open_gate, dim3(1), dim3(64), 0, c->st, c->failf.as<int>());
    double v[SC_N];
    RC(lin_at<K>(c, c->x.as<double>(), c->Wr.as<double>(), c->PR.as<double>(), c->colsq.as<double>(), c->grad.as<double>(),
                 c->camsum.as<double>(), false, v));
    if (o.jacobi_scaling) {
        hipLaunchKernelGGL(ba_scale, dim3(nblk(c->n)), dim3(256), 0, c->st, (int)c->n, c->colsq.as<double>(),
                           c->scale.as<double>());
    }
    // the iteration-0 records were written unscaled: the steps on them scale what they read
    c->unscaled_wr = o.jacobi_scaling ? c->Wr.p : nullptr;
    c->scaled = true;
    HIPCHK(hipEventRecord(c->ev[5], c->st));
    HIPCHK(hipEventSynchronize(c->ev[5]));
    {
        float a = 0;
        HIPCHK(hipEventElapsedTime(&a, c->ev[4], c->ev[5]));
        c->phase_ms[0] += a;
    }
    double cost = v[SC_COST], gmax = v[SC_GMAX], x_norm = std::sqrt(v[SC_XN] + v[SC_XN_F]);
    sum->initial_cost = cost;
    double radius = o.initial_trust_region_radius, decrease = 2.0;
    bool successful = true;
    int iteration = 0, succ = 0, unsucc = 0, invalid_total = 0, consec_invalid = 0, ntrace = 0;
    int term = SFMX_BA_NO_CONVERGENCE;
    if (c->spec && !c->phases) {
        // Speculative LM: the device judges every step (ba_decide, the loop below restated) and the
        // host enqueues step s + 1 on the accepted buffers before it reads step s's outcome, so the GPU
        // never waits for the host; a rejected step's successor is skipped by the step gate and
        // enqueued again on the unchanged buffers.  The first iteration's top is the host's.
        ++succ;
        if (trace && ntrace < trace_cap) { trace[0] = cost; trace[1] = radius; trace[2] = 1.0; ++ntrace; }
        if (iteration >= maxit) term = SFMX_BA_NO_CONVERGENCE;
        else if (gmax <= o.gradient_tolerance) term = SFMX_BA_CONVERGENCE;
        else if (radius <= o.min_trust_region_radius) term = SFMX_BA_CONVERGENCE;
        else {
            ++iteration;
            c->spec_maxit = maxit;
            double* li = c->lm_init;
            for (int i = 0; i < LM_N; ++i) li[i] = 0.0;
            li[LM_COST] = cost; li[LM_GMAX] = gmax; li[LM_XNORM] = x_norm; li[LM_RADIUS] = radius; li[LM_DECREASE] = 2.0;
            li[LM_ITER] = iteration; li[LM_SUCC] = succ; li[LM_SUCCESSFUL] = 1.0; li[LM_TERM] = LM_RUNNING;
            HIPCHK(hipMemcpyAsync(c->lmst.p, li, sizeof(double) * LM_N, hipMemcpyHostToDevice, c->st));
            auto swap_state = [c]() {
                std::swap(c->x, c->cand);
                std::swap(c->Wr, c->Wr2);
                std::swap(c->PR, c->PR2);
                std::swap(c->colsq, c->colsq2);
                std::swap(c->grad, c->grad2);
                std::swap(c->camsum, c->camsum2);
            };
            bool vd; double d0, d1, d2, d3, d4;
            unsigned q = ++c->seq;
            RC(try_step<K>(c, radius, &vd, &d0, &d1, &d2, &d3, &d4, true, q));
            double L[sfmx_ba_ctx::HS_SLOT];
            for (;;) {
                swap_state();   // provisional: the next step runs on the accepted step's buffers
                unsigned q2 = ++c->seq;
                RC(try_step<K>(c, radius, &vd, &d0, &d1, &d2, &d3, &d4, true, q2));
                RC(wait_slot(c, q, L));
                const double* lm = L + SC_N;
                if (lm[LM_ERROR] != 0.0) {
                    (void)hipStreamSynchronize(c->st);
                    return fail(SFMX_EINTERNAL, "BA solve: a dependency wait of the in-launch factorization / back "
                                                "solve timed out (speculative mode has no per-level fallback)");
                }
                const bool acc = lm[LM_ACCEPTED] != 0.0;
                if (!acc) swap_state();
                else c->unscaled_wr = nullptr;   // (the iteration-0 buffer is candidate storage from here)
                if (lm[LM_TRACE] != 0.0 && trace && ntrace < trace_cap) {
                    trace[3 * ntrace] = lm[LM_COST]; trace[3 * ntrace + 1] = lm[LM_RADIUS];
                    trace[3 * ntrace + 2] = lm[LM_SUCCESSFUL]; ++ntrace;
                }
                if (lm[LM_TERM] != LM_RUNNING) {   // the successor is gated off
                    term = (int)lm[LM_TERM];
                    break;
                }
                if (!acc) {   // the successor was skipped: the same step again, on the unchanged buffers
                    hipLaunchKernelGGL(ba_open_gate, dim3(1), dim3(64), 0, c->st, c->failf.as<int>());
                    q2 = ++c->seq;
                    RC(try_step<K>(c, radius, &vd, &d0, &d1, &d2, &d3, &d4, true, q2));
                }
                q = q2;
            }
            HIPCHK(hipStreamSynchronize(c->st));   // the skipped successor drains
            const double* lm = L + SC_N;
            cost = lm[LM_COST]; gmax = lm[LM_GMAX]; radius = lm[LM_RADIUS];
            succ = (int)lm[LM_SUCC]; unsucc = (int)lm[LM_UNSUCC]; invalid_total = (int)lm[LM_INVALID];
        }
    } else
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
        bool valid; double mcc, sn, ccost, cgmax, cxn;
        RC(try_step<K>(c, radius, &valid, &mcc, &sn, &ccost, &cgmax, &cxn));
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
        if (rel > o.min_relative_decrease) {   // HandleSuccessfulStep: the candidate's linearization is current
            c->unscaled_wr = nullptr;   // (the iteration-0 buffer is candidate storage from here)
            std::swap(c->x, c->cand);
            std::swap(c->Wr, c->Wr2);
            std::swap(c->PR, c->PR2);
            std::swap(c->colsq, c->colsq2);
            std::swap(c->grad, c->grad2);
            std::swap(c->camsum, c->camsum2);
            cost = ccost;
            gmax = cgmax;
            x_norm = cxn;
            radius = radius / std::max(1.0 / 3.0, 1.0 - lm_cube(2.0 * rel - 1.0));   // == ba_decide's bits
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

int run_lm(sfmx_ba_ctx* c, int max_iters, sfmx_ba_summary* sum, double* trace, int trace_cap, int* ntrace_out) {
    if (c->K == 1) return run_lm_k<1>(c, max_iters, sum, trace, trace_cap, ntrace_out);
    if (c->K == 3) return run_lm_k<3>(c, max_iters, sum, trace, trace_cap, ntrace_out);
    return run_lm_k<7>(c, max_iters, sum, trace, trace_cap, ntrace_out);
}

bool valid_model(int m) { return m == SFMX_CAM_SIMPLE || m == SFMX_CAM_SIMPLE_RADIAL || m == SFMX_CAM_DISTORTION; }

int validate(const sfmx_ba_problem* pb) {
    if (!pb) return fail(SFMX_EINVAL, "null problem");
    if (pb->n_points < 0 || pb->n_cams < 0 || pb->n_obs < 0 || pb->n_intr < 0) return fail(SFMX_EINVAL, "negative sizes");
    if (pb->n_intr == 0 && !valid_model(pb->cam_model))
        return fail(SFMX_EINVAL, "cam_model must be SFMX_CAM_SIMPLE, _SIMPLE_RADIAL or _DISTORTION");
    if (pb->n_intr > 0) {
        if (!pb->intr_model || (pb->n_cams && !pb->pose_intr) || !pb->intr_center)
            return fail(SFMX_EINVAL, "n_intr > 0 needs intr_model, pose_intr and intr_center");
        for (int m = 0; m < pb->n_intr; ++m)
            if (!valid_model(pb->intr_model[m]))
                return fail(SFMX_EINVAL, "intr_model entries must be SFMX_CAM_SIMPLE, _SIMPLE_RADIAL or _DISTORTION");
        for (int c = 0; c < pb->n_cams; ++c)
            if (pb->pose_intr[c] < 0 || pb->pose_intr[c] >= pb->n_intr)
                return fail(SFMX_EINVAL, "pose_intr entry out of range");
    }
    if ((pb->n_points && !pb->points) || (pb->n_cams && !pb->poses) || !pb->intr ||
        (pb->n_obs && (!pb->obs_point || !pb->obs_cam || !pb->obs_xy)))
        return fail(SFMX_EINVAL, "null problem array");
    std::atomic<bool> bad{false};   // O(observations) on every call: on the worker pool
    sfmx::parallel_ranges(pb->n_obs, pb->n_obs >= 65536 ? 16 : 1, [&](int64_t o0, int64_t o1) {
        const int P = pb->n_points, C = pb->n_cams;
        bool b = false;
        for (int64_t o = o0; o < o1; ++o)
            b |= (unsigned)pb->obs_point[o] >= (unsigned)P || (unsigned)pb->obs_cam[o] >= (unsigned)C;
        if (b) bad = true;
    });
    if (bad) return fail(SFMX_EINVAL, "observation index out of range");
    return SFMX_OK;
}

int set_params(sfmx_ba_ctx* c, const sfmx_ba_problem* pb, bool sync = true) {
    DeviceGuard dg(c->device);
    double* x = c->x.as<double>();
    // x = [points 3P | poses 6C | intrinsics border K]: staged back to back, one copy (r05)
    const size_t n = 3 * (size_t)c->P + 6 * (size_t)c->C + (size_t)c->K;
    double* h = static_cast<double*>(stage_bytes(c, sizeof(double) * std::max<size_t>(n, 1)));
    if (!h) return fail(SFMX_ENOMEM, "pinned staging buffer");
    sfmx::parallel_ranges(c->P, c->P >= 16384 ? 16 : 1, [&](int64_t q0, int64_t q1) {
        for (int64_t q = q0; q < q1; ++q)
            for (int i = 0; i < 3; ++i) h[3 * (size_t)q + i] = pb->points[3 * (size_t)c->pperm[q] + i];
    });
    if (c->C) std::memcpy(h + 3 * (size_t)c->P, pb->poses, sizeof(double) * 6 * c->C);
    double* iv = h + 3 * (size_t)c->P + 6 * (size_t)c->C;   // the border: referenced blocks, zero padding
    for (int j = 0; j < c->K; ++j) iv[j] = c->isrc[j] >= 0 ? pb->intr[c->isrc[j]] : 0.0;
    if (n) HIPCHK(hipMemcpyAsync(x, h, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
    if (sync) HIPCHK(hipStreamSynchronize(c->st));
    return SFMX_OK;
}

// Locality order (internal only; results are reported in the caller's order): points sorted by
// their sorted camera lists (points seen by the same cameras become neighbours, so a point group
// spans few cameras), observations point-major in that order.  The sort key is the list's first
// cameras, as many as fit 64 bits at ceil(log2(C + 2)) bits each, at most 6 (lexicographic, a
// shorter list first), ties keep the caller's order.  Its most significant field is the point's
// smallest camera, so the order is the concatenation of camera BUCKETS (points whose smallest camera
// lies in [BUCKET_CAMS b, BUCKET_CAMS (b + 1)); points without observations in bucket 0, first), each
// sorted on its own: a bucket is ordered and grouped independently and kept between calls, and an
// update (sfmx_ba_update, the SfM loop's grown scene) redoes only the buckets whose points changed
// (HostScratch below).
// 4 (r04; 8 before): an SfM step's new camera dirties its own bucket and the ring's closing one, so the
// points re-ordered and re-grouped per update halve (C5: ~2 x 4000 instead of ~2 x 8000), for a few more
// partial groups at bucket edges
constexpr int BUCKET_CAMS = 4;

// The caller's observations as a point-major view: obs of point p are view positions
// [start[p], start[p + 1]); position i is caller observation i (point-major input, pm) or vobs[i].
struct View {
    std::vector<int> start, vobs;
    bool pm = true;
    int obs(int64_t i) const { return pm ? (int)i : vobs[i]; }
};
void make_view(const sfmx_ba_problem* pb, View& v) {
    const int P = pb->n_points, O = pb->n_obs;
    constexpr int PIECES = 64;   // fixed ranges (host_par.hpp): the same result on every host
    v.start.resize(P + 1);
    std::atomic<bool> pm{true};
    // the reference adds residuals point by point (BundleAdjustment.cpp:50-91).  Two passes: the
    // order check over every range (each range compares across its left boundary, so all ranges
    // monotone = the whole array monotone), then, only for a point-major problem, the start fill, where
    // every start is written by exactly one range.  (r05 fused them: on shuffled input the fill then
    // wrote overlapping start ranges from several threads, O(O * P) work and a data race)
    const int* op = pb->obs_point;
    sfmx::parallel_ranges((int64_t)O + 1, PIECES, [&](int64_t i0, int64_t i1) {
        for (int64_t i = std::max<int64_t>(i0, 1); i < std::min<int64_t>(i1, O); ++i)
            if (op[i - 1] > op[i]) { pm = false; return; }
    });
    if (pm)
        sfmx::parallel_ranges((int64_t)O + 1, PIECES, [&](int64_t i0, int64_t i1) {
            for (int64_t i = i0; i < i1; ++i) {   // points (op[i - 1], op[i]] start at i
                const int lo = i == 0 ? -1 : op[i - 1], hi = i == O ? P - 1 : op[i];
                for (int p = lo + 1; p <= hi; ++p) v.start[p] = (int)i;
            }
        });
    v.pm = pm;
    if (v.pm) {
        v.start[P] = O;
        v.vobs.clear();
    } else {
        std::fill(v.start.begin(), v.start.end(), 0);
        for (int i = 0; i < O; ++i) v.start[pb->obs_point[i] + 1]++;
        for (int p = 0; p < P; ++p) v.start[p + 1] += v.start[p];
        std::vector<int> f(v.start.begin(), v.start.end() - 1);
        v.vobs.resize(O);
        for (int i = 0; i < O; ++i) v.vobs[f[pb->obs_point[i]]++] = i;
    }
}
struct KeyBits { int kb, nk; };
KeyBits key_bits(int C) {   // bits per camera (c + 1, 0 = none) and cameras per 64-bit key
    int kb = 1;
    while ((1ll << kb) < (long long)C + 2) ++kb;
    return KeyBits{kb, std::min(6, 64 / kb)};
}
// the point's sort key and its smallest camera (-1: no observation)
uint64_t point_key(const sfmx_ba_problem* pb, const View& v, int p, KeyBits kb, int* minc) {
    uint32_t lo[6] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u};   // the nk smallest cameras, sorted
    for (int a = v.start[p]; a < v.start[p + 1]; ++a) {
        uint32_t c = (uint32_t)pb->obs_cam[v.obs(a)];
        for (int j = 0; j < kb.nk; ++j)
            if (c < lo[j]) std::swap(c, lo[j]);
    }
    uint64_t k = 0;
    for (int j = 0; j < kb.nk; ++j) k = (k << kb.kb) | (lo[j] == ~0u ? 0u : lo[j] + 1);
    *minc = lo[0] == ~0u ? -1 : (int)lo[0];
    return k;
}
int bucket_of(int minc) { return minc < 0 ? 0 : minc / BUCKET_CAMS; }

// Stable LSD radix sort of (key, index) records on the key's low `bits` bits, 8 bits a pass, passes
// whose digit is the same for every record skipped: the order std::sort gives (key, index) records
// whose indices ascend on entry (r04: std::sort took ~80 ns per point of the ring-closing bucket).
void radix_sort_keys(std::pair<uint64_t, int>* kp, size_t n, int bits) {
    if (n < 2) return;
    thread_local std::vector<std::pair<uint64_t, int>> tmp;
    tmp.resize(n);
    std::pair<uint64_t, int>*src = kp, *dst = tmp.data();
    for (int sh = 0; sh < bits; sh += 8) {
        uint32_t cnt[257] = {};
        for (size_t i = 0; i < n; ++i) cnt[((src[i].first >> sh) & 255) + 1]++;
        bool one = false;
        for (int d = 1; d <= 256; ++d) if (cnt[d] == n) one = true;
        if (one) continue;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (size_t i = 0; i < n; ++i) dst[cnt[(src[i].first >> sh) & 255]++] = src[i];
        std::swap(src, dst);
    }
    if (src != kp) std::copy(src, src + n, kp);
}

// Point groups, chunks, local cameras, assembly task lists and camera slot lists (see ba_group.hpp).
struct TopoSeg;
struct PairRef { uint64_t key; int g, la, lb; };   // finish_topology: one (camera a, camera b) block of a group
// A vector whose resize() leaves new elements of trivial types uninitialised (r05: the merged topology
// is resized and then filled in parallel; value-initialising ~3 MB of assembly entries first was a
// serial memset on every load)
template <class T, class A = std::allocator<T>>
struct uninit_alloc : A {
    template <class U> struct rebind { using other = uninit_alloc<U, typename std::allocator_traits<A>::template rebind_alloc<U>>; };
    using A::A;
    template <class U> void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) { ::new (static_cast<void*>(p)) U; }
    template <class U, class... Args> void construct(U* p, Args&&... args) {
        std::allocator_traits<A>::construct(static_cast<A&>(*this), p, std::forward<Args>(args)...);
    }
};
template <class T> using uvec = std::vector<T, uninit_alloc<T>>;

struct Topology {   // kept with the context: its vectors keep their capacity between calls
    std::vector<PairRef> pr, pr_out;   // finish_topology's scratch (kept: no per-call allocation)
    std::vector<int> pr_cnt, slot_g;
    // the camera co-visibility of the problem's points: bit a C + b set when some point is observed by
    // cameras a and b (a != b).  S_cc's pattern and the factorization plan come from it, not from the
    // point groups' camera unions (a group's dense block holds exact zeros for the pairs none of its
    // points connects: on the C5 ring the unions add ~150 such pairs, the elimination tree gets one level
    // more and 82 instead of 66 nonzero tiles, r04)
    std::vector<uint64_t> covis;
    uvec<Grp> grp;
    uvec<Chunk> chk;
    uvec<Batch> bat;
    uvec<int> gcam, lcrow;
    std::vector<int> cref_start, cref;
    std::vector<short> obs_lc, obs_row;
    uvec<ATask> tasks;
    uvec<AEnt> ents;
    long long sg_total = 0, h_total = 0;
    int rg_total = 0, dp_max = 16;
    void clear() {
        grp.clear(); chk.clear(); bat.clear(); gcam.clear(); cref_start.clear(); cref.clear(); lcrow.clear();
        tasks.clear(); ents.clear();
        sg_total = h_total = 0; rg_total = 0; dp_max = 16;
    }
};

// One segment of the greedy point-group scan: points [s0, s1) (groups never span segments);
// offsets in the group records are local to the segment until the merge.
struct TopoSeg {
    std::vector<Grp> grp;
    std::vector<Chunk> chk;
    std::vector<Batch> bat;
    std::vector<int> gcam, lcrow;
    long long sg_total = 0, h_total = 0;
    int rg_total = 0, dp_max = 16;
    void clear() { grp.clear(); chk.clear(); bat.clear(); gcam.clear(); lcrow.clear(); sg_total = h_total = 0; rg_total = 0; dp_max = 16; }
};

// (r05: the per-point sort / union on small stack arrays and the local-camera lookups through a
// per-thread camera -> slot table instead of binary searches: the same groups, ~3x less host time)
void topo_segment(int s0, int s1, int K, int gpts, int C, const std::vector<int>& pt_start, const int* obs_cam,
                  short* obs_lc, short* obs_row, TopoSeg& tp) {
    thread_local std::vector<int> lcm;   // camera -> its slot in the group being added (set before every use)
    if ((int)lcm.size() < C) lcm.resize(C);
    std::vector<int> bigc;               // a big point's cameras (any count)
    int cur[UMAX + WB_OBS], uni[UMAX + WB_OBS], pc[WB_OBS];
    int ncur = 0;
    int cnt[UMAX], fill[UMAX];
    tp.clear();
    int g_p0 = s0, g_obs = 0;
    auto add_group = [&](int p0, int p1, const int* cams, int u, bool big) {
        Grp G{};
        G.o0 = pt_start[p0]; G.o1 = pt_start[p1]; G.p0 = p0; G.p1 = p1;
        G.u = u;
        G.cam_off = (int)tp.gcam.size();
        G.big = big ? 1 : 0;
        const int dim = 6 * G.u + K;
        G.rg_off = tp.rg_total;
        tp.rg_total += dim;
        G.ch0 = (int)tp.chk.size();
        G.nch = 0;
        G.b0 = (int)tp.bat.size();
        G.nb = 0;
        for (int i = 0; i < u; ++i) lcm[cams[i]] = i;
        if (big) {
            G.h_off = tp.h_total;
            tp.h_total += (long long)dim * 3;
            G.sg_off = 0;
        } else {
            G.sg_off = tp.sg_total;
            tp.sg_total += (long long)dim * dim;
            G.h_off = 0;
            tp.dp_max = std::max(tp.dp_max, (dim + 15) & ~15);
            // ba_gschur wave batches: whole points, <= WB_OBS observations, <= WB_PTS points
            for (int q = p0; q < p1;) {
                Batch b{pt_start[q], pt_start[q], q, q};
                while (q < p1 && pt_start[q + 1] - b.o0 <= WB_OBS && q - b.p0 < WB_PTS) ++q;
                b.o1 = pt_start[q];
                b.p1 = q;
                tp.bat.push_back(b);
                ++G.nb;
            }
            // chunks of whole points, <= GCH observations; feature rows sorted by local camera
            // (observation order inside a camera), each camera's rows zero-padded to a multiple of 4
            int q = p0;
            while (q < p1) {
                Chunk ch{pt_start[q], pt_start[q], q - p0, q - p0, (int)tp.lcrow.size(), 0, 0, 0};
                while (q < p1 && pt_start[q + 1] - ch.o0 <= GCH) { ++q; }
                ch.o1 = pt_start[q]; ch.q1 = q - p0;
                for (int lc = 0; lc < u; ++lc) cnt[lc] = 0;
                for (int o = ch.o0; o < ch.o1; ++o) cnt[lcm[obs_cam[o]]]++;
                int row = 0;
                for (int lc = 0; lc < u; ++lc) {
                    tp.lcrow.push_back(row);
                    fill[lc] = row;
                    row += (2 * cnt[lc] + 3) & ~3;
                }
                tp.lcrow.push_back(row);
                ch.nrows = row;
                for (int o = ch.o0; o < ch.o1; ++o) {
                    const int lc = lcm[obs_cam[o]];
                    obs_row[o] = (short)fill[lc];
                    fill[lc] += 2;
                }
                tp.chk.push_back(ch);
                ++G.nch;
            }
        }
        tp.gcam.insert(tp.gcam.end(), cams, cams + u);
        for (int o = G.o0; o < G.o1; ++o) obs_lc[o] = (short)lcm[obs_cam[o]];
        tp.grp.push_back(G);
    };
    for (int p = s0; p < s1; ++p) {
        const int m = pt_start[p + 1] - pt_start[p];
        const int* oc = obs_cam + pt_start[p];
        bool big = m > WB_OBS, dup = false;
        int npc = 0;
        if (!big) {   // insertion sort of the point's cameras, duplicates dropped (and noted)
            for (int i = 0; i < m; ++i) {
                const int c = oc[i];
                int j = npc;
                while (j > 0 && pc[j - 1] > c) --j;
                if (j > 0 && pc[j - 1] == c) { dup = true; continue; }
                for (int k = npc; k > j; --k) pc[k] = pc[k - 1];
                pc[j] = c;
                ++npc;
            }
            big = dup || 6 * npc + K > GDPMAX;
        }
        if (big) {
            bigc.assign(oc, oc + m);
            std::sort(bigc.begin(), bigc.end());
            bigc.erase(std::unique(bigc.begin(), bigc.end()), bigc.end());
            if (p > g_p0) add_group(g_p0, p, cur, ncur, false);
            add_group(p, p + 1, bigc.data(), (int)bigc.size(), true);
            g_p0 = p + 1; g_obs = 0; ncur = 0;
            continue;
        }
        int nu = 0;   // cur U pc (both sorted, unique)
        for (int a = 0, b = 0; a < ncur || b < npc;) {
            if (b == npc || (a < ncur && cur[a] < pc[b])) uni[nu++] = cur[a++];
            else if (a == ncur || pc[b] < cur[a]) uni[nu++] = pc[b++];
            else { uni[nu++] = cur[a++]; ++b; }
        }
        if (p > g_p0 && (g_obs + m > GOBS || p - g_p0 + 1 > gpts || 6 * nu + K > GDPMAX)) {
            add_group(g_p0, p, cur, ncur, false);
            g_p0 = p; g_obs = 0;
            std::copy(pc, pc + npc, cur);
            ncur = npc;
        } else {
            std::copy(uni, uni + nu, cur);
            ncur = nu;
        }
        g_obs += m;
    }
    if (s1 > g_p0) add_group(g_p0, s1, cur, ncur, false);
}

// Points in segments of SEG_PTS (a fixed size: the same groups on every host), scanned in
// parallel (host_par.hpp), merged in segment order; then the camera slots and assembly tasks.
// 2048 (r04; 8192 before): an update that redoes two camera buckets of ~8000 points scans 8 segments
// on the worker pool instead of 2 (the scan is ~0.3 us per point), for ~1 % more (partial) groups.
constexpr int SEG_PTS = 2048;

// Points per group: the group kernels (ba_glin, ba_gschur, ba_gupdate) run one workgroup per group
// and their workgroups take about the same time, so a launch costs ceil(groups / slots) rounds
// (slots = workgroups resident at once, from the device's occupancy of ba_glin).  C5 with 128-point
// groups is 1564 groups on 512 slots: a fourth round for 28 workgroups.  The cap is the smallest
// group size (a multiple of 8) that keeps the rounds of full-size groups (estimated on SEG_PTS
// segments): there, 104 points -> ~1930 groups in 4 rounds.  Camera limits can still cut groups earlier.
// Only problems of several rounds are re-sized, and never below GPTS / 2 points: a problem of one
// round keeps full-size groups (the regime every small-problem parity test was pinned in).
int group_points(int P, int slots) {
    if (P <= 0 || slots <= 0) return GPTS;
    auto groups = [P](int cap) {
        int64_t g = 0;
        for (int s0 = 0; s0 < P; s0 += SEG_PTS) g += (std::min(P - s0, SEG_PTS) + cap - 1) / cap;
        return g;
    };
    const int64_t rounds = (groups(GPTS) + slots - 1) / slots;
    if (rounds < 2) return GPTS;
    // caps in steps of 8 points: a growing scene (sfmx_ba_update) keeps its cap, so its unchanged
    // buckets keep their groups, until the step no longer fits the rounds
    for (int cap = (int)((std::max<int64_t>(GPTS / 2, P / (rounds * slots)) + 7) / 8 * 8); cap < GPTS; cap += 8)
        if (groups(cap) <= rounds * slots) return cap;
    return GPTS;
}

// The camera slots and assembly tasks of the merged groups (tp.grp / gcam in internal order).
bool covisible(const Topology& tp, int C, int a, int b) {
    const size_t bit = (size_t)a * C + b;
    return (tp.covis[bit >> 6] >> (bit & 63)) & 1;
}
// (r05: in parallel.  The pose-pair tasks are cut by camera ranges: piece t owns the pairs whose first
// camera lies in [C t / TP, C (t + 1) / TP), scans every group in order for them (a group's cameras are
// sorted, so they are one run of its local cameras), sorts them stably by pair and builds its tasks and
// entries; the pieces are concatenated in camera order.  The same tasks and entries as one serial pass.)
constexpr int TOPO_PIECES = 16;
struct TaskPiece {
    std::vector<PairRef> pr;
    uvec<PairRef> out;
    std::vector<int> cnt;
    std::vector<ATask> tasks;
    std::vector<AEnt> ents;
};
void finish_topology(int C, int K, Topology& tp) {
    thread_local std::vector<TaskPiece> pcs_tl;   // the caller thread's pieces, kept between calls (the
    std::vector<TaskPiece>& pcs = pcs_tl;          // workers below reach them through this reference)
    pcs.resize(TOPO_PIECES);
    const int ng = (int)tp.grp.size();
    // camera slots: per camera, its (group, local camera) slots in group order
    std::vector<int>& slot_g = tp.slot_g;
    slot_g.resize(tp.gcam.size());
    tp.cref_start.assign(C + 1, 0);
    for (int g = 0; g < ng; ++g)
        for (int lc = 0; lc < tp.grp[g].u; ++lc) slot_g[tp.grp[g].cam_off + lc] = g;
    for (int cm : tp.gcam) tp.cref_start[cm + 1]++;
    for (int c = 0; c < C; ++c) tp.cref_start[c + 1] += tp.cref_start[c];
    tp.cref.assign(tp.cref_start[C], 0);
    {
        std::vector<int> f(tp.cref_start.begin(), tp.cref_start.end() - 1);
        for (int sl = 0; sl < (int)tp.gcam.size(); ++sl) tp.cref[f[tp.gcam[sl]]++] = sl;
    }
    auto ent = [&](int g, int la, int lb) {   // contribution of group g at local rows 6la / 6lb
        const Grp& G = tp.grp[g];
        const int dim = 6 * G.u + K;
        AEnt e{};
        e.dim = dim;
        e.big = G.big;
        e.rg = G.rg_off + 6 * la;
        if (G.big) { e.b0 = G.h_off + 3LL * (6 * la); e.b1 = G.h_off + 3LL * (6 * lb); }
        else { e.b0 = G.sg_off + (long long)(6 * la) * dim + 6 * lb; e.b1 = 0; }
        return e;
    };
    // assembly tasks: pose blocks (a <= b) with their (group, la, lb) lists in group order, then
    // pose-intrinsics blocks per camera, then the intrinsics block
    sfmx::parallel_items(TOPO_PIECES, [&](int t) {
        TaskPiece& P = pcs[t];
        const int a0 = (int)((int64_t)C * t / TOPO_PIECES), a1 = (int)((int64_t)C * (t + 1) / TOPO_PIECES);
        P.pr.clear(); P.tasks.clear(); P.ents.clear();
        if (a1 <= a0) return;
        for (int g = 0; g < ng; ++g) {   // (key (a, b), group order)
            const Grp& G = tp.grp[g];
            const int* cams = tp.gcam.data() + G.cam_off;
            for (int la = 0; la < G.u; ++la) {
                if (cams[la] < a0) continue;
                if (cams[la] >= a1) break;
                for (int lb = la; lb < G.u; ++lb)
                    P.pr.push_back(PairRef{((uint64_t)(uint32_t)cams[la] << 32) | (uint32_t)cams[lb], g, la, lb});
            }
        }
        // stable counting sort on the pair index (a - a0) C + b
        auto idx = [C, a0](const PairRef& x) { return (size_t)((int)(x.key >> 32) - a0) * C + (size_t)(x.key & 0xffffffffu); };
        const size_t span = (size_t)(a1 - a0) * C;
        if (span <= ((size_t)1 << 20) || span <= 4 * P.pr.size()) {   // dense counting sort (C5: 13 x 200 slots)
            P.cnt.assign(span + 1, 0);
            for (const PairRef& x : P.pr) P.cnt[idx(x) + 1]++;
            for (size_t i = 1; i < P.cnt.size(); ++i) P.cnt[i] += P.cnt[i - 1];
            P.out.resize(P.pr.size());
            for (const PairRef& x : P.pr) P.out[P.cnt[idx(x)]++] = x;
        } else {   // large C with few pairs per slot: the same stable order without C^2 counters
            P.out.assign(P.pr.begin(), P.pr.end());
            std::stable_sort(P.out.begin(), P.out.end(), [](const PairRef& x, const PairRef& y) { return x.key < y.key; });
        }
        const uvec<PairRef>& pr = P.out;
        for (size_t i = 0; i < pr.size();) {
            ATask tk{0, (int)(pr[i].key >> 32), (int)(pr[i].key & 0xffffffffu), (int)P.ents.size(), 0, 0, 0, 0};
            size_t j = i;
            while (j < pr.size() && pr[j].key == pr[i].key) ++j;
            if (tk.a == tk.b || covisible(tp, C, tk.a, tk.b)) {   // a pair no point connects: exact zeros, no task
                for (size_t q = i; q < j; ++q) P.ents.push_back(ent(pr[q].g, pr[q].la, pr[q].lb));
                tk.l1 = (int)P.ents.size();
                P.tasks.push_back(tk);
            }
            i = j;
        }
    });
    // concatenated in camera order; then the per-camera and intrinsics tasks
    std::vector<size_t> eoff(TOPO_PIECES + 1, 0), toff(TOPO_PIECES + 1, 0);
    for (int t = 0; t < TOPO_PIECES; ++t) {
        eoff[t + 1] = eoff[t] + pcs[t].ents.size();
        toff[t + 1] = toff[t] + pcs[t].tasks.size();
    }
    const size_t ne_pose = eoff[TOPO_PIECES], nt_pose = toff[TOPO_PIECES];
    const size_t ne_cam = tp.cref.size(), ne = ne_pose + ne_cam + (size_t)ng;
    // r06: a type-1 task for every camera and an (empty) diagonal pose task for every camera no group
    // holds: ba_assemble adds the camera terms of ba_add_cam to its outputs (one rank), so every camera
    // row block needs a task (its D^2 damping even without observations)
    const size_t nt_cam = (size_t)C;
    size_t n_orph = 0;
    for (int cm = 0; cm < C; ++cm) n_orph += tp.cref_start[cm + 1] == tp.cref_start[cm];
    tp.ents.resize(ne);
    tp.tasks.resize(nt_pose + nt_cam + n_orph + (size_t)(K * K + K));
    sfmx::parallel_items(TOPO_PIECES + 2, [&](int t) {
        if (t < TOPO_PIECES) {
            const TaskPiece& P = pcs[t];
            std::copy(P.ents.begin(), P.ents.end(), tp.ents.begin() + eoff[t]);
            for (size_t i = 0; i < P.tasks.size(); ++i) {
                ATask tk = P.tasks[i];
                tk.l0 += (int)eoff[t];
                tk.l1 += (int)eoff[t];
                tp.tasks[toff[t] + i] = tk;
            }
        } else if (t == TOPO_PIECES) {   // pose-intrinsics blocks per camera (column block: the intrinsics rows)
            size_t e = ne_pose, k = nt_pose;
            for (int cm = 0; cm < C; ++cm) {
                ATask tk{1, cm, 0, (int)e, 0, 0, 0, 0};
                for (int q = tp.cref_start[cm]; q < tp.cref_start[cm + 1]; ++q) {
                    const int sl = tp.cref[q], g = slot_g[sl];
                    tp.ents[e++] = ent(g, sl - tp.grp[g].cam_off, tp.grp[g].u);
                }
                tk.l1 = (int)e;
                tp.tasks[k++] = tk;
            }
            for (int cm = 0; cm < C; ++cm)   // cameras without observations: their diagonal block
                if (tp.cref_start[cm + 1] == tp.cref_start[cm]) tp.tasks[k++] = ATask{0, cm, cm, 0, 0, 0, 0, 0};
        } else {   // the intrinsics block and rhs: one task per output, every group
            const int l0 = (int)(ne_pose + ne_cam);
            for (int g = 0; g < ng; ++g) tp.ents[l0 + g] = ent(g, tp.grp[g].u, tp.grp[g].u);
            for (int x = 0; x < K * K + K; ++x) tp.tasks[nt_pose + nt_cam + n_orph + x] = ATask{2, 0, x, l0, (int)ne, 0, 0, 0};
        }
    });
}

// Every index the group kernels derive from the topology, checked against the limits and buffer
// sizes they assume (ba_glin: GROWS feature rows, GCH observations, GPTS point threads, UMAX
// cameras; ba_gschur: WB_OBS / WB_PTS batches, the lane map, dp <= GDPMAX; ba_gupdate: one thread
// per point of a chunk; ba_assemble / ba_camred: entry and slot ranges inside sg / hbig / rg /
// gpart).  Run by the diagnostic library on every load and by the CPU tests on random problems
// (tests/test_ba_host.py); "" when everything holds, else the first violation.
[[maybe_unused]] std::string check_topology(int P, int C, int O, int K, const std::vector<int>& pt_start, const int* obs_cam,
                                            const Topology& tp) {
    auto bad = [](const std::string& m) { return m; };
    auto S = [](long long v) { return std::to_string(v); };
    if ((int)pt_start.size() != P + 1 || pt_start[0] != 0 || pt_start[P] != O) return bad("pt_start does not span the observations");
    if ((int)tp.obs_lc.size() != O || (int)tp.obs_row.size() != O) return bad("obs_lc / obs_row size");
    int next_p = 0;
    for (size_t g = 0; g < tp.grp.size(); ++g) {
        const Grp& G = tp.grp[g];
        const std::string at = "group " + S((long long)g) + ": ";
        if (G.p0 != next_p || G.p1 <= G.p0 || G.p1 > P) return bad(at + "points not contiguous");
        next_p = G.p1;
        if (G.o0 != pt_start[G.p0] || G.o1 != pt_start[G.p1]) return bad(at + "observation range");
        if (G.u < 0 || G.cam_off < 0 || G.cam_off + G.u > (int)tp.gcam.size()) return bad(at + "camera slots");
        for (int lc = 0; lc < G.u; ++lc) {
            const int cm = tp.gcam[G.cam_off + lc];
            if (cm < 0 || cm >= C || (lc > 0 && tp.gcam[G.cam_off + lc - 1] >= cm)) return bad(at + "cameras not sorted / out of range");
        }
        const long long dim = 6LL * G.u + K;
        if (G.rg_off < 0 || G.rg_off + dim > tp.rg_total) return bad(at + "rhs block outside rg");
        for (int o = G.o0; o < G.o1; ++o) {
            const int lc = tp.obs_lc[o];
            if (lc < 0 || lc >= G.u || tp.gcam[G.cam_off + lc] != obs_cam[o]) return bad(at + "obs_lc of observation " + S(o));
        }
        if (G.big) {
            if (G.p1 != G.p0 + 1) return bad(at + "big group of several points");
            if (G.h_off < 0 || G.h_off + 3 * dim > tp.h_total) return bad(at + "H outside hbig");
            continue;
        }
        if (G.p1 - G.p0 > GPTS || G.o1 - G.o0 > GOBS) return bad(at + "more points / observations than a workgroup holds");
        if (G.u > UMAX || dim > GDPMAX) return bad(at + "camera union too wide for ba_gschur / ba_glin");
        if (G.sg_off < 0 || G.sg_off + dim * dim > tp.sg_total) return bad(at + "block outside sg");
        if (((dim + 15) & ~15) > tp.dp_max) return bad(at + "dp above the launch's dp_max");
        // chunks: whole points in order, <= GCH observations, feature rows per camera
        int q = G.p0;
        if (G.nch < 1 || G.ch0 < 0 || G.ch0 + G.nch > (int)tp.chk.size()) return bad(at + "chunk range");
        for (int c = 0; c < G.nch; ++c) {
            const Chunk& ch = tp.chk[G.ch0 + c];
            const std::string cat = at + "chunk " + S(c) + ": ";
            if (ch.q0 != q - G.p0 || ch.q1 < ch.q0 || G.p0 + ch.q1 > G.p1) return bad(cat + "point slots");
            if (ch.o0 != pt_start[G.p0 + ch.q0] || ch.o1 != pt_start[G.p0 + ch.q1]) return bad(cat + "observation range");
            if (ch.o1 - ch.o0 > GCH || ch.q1 > GCH) return bad(cat + "more than GCH observations / point threads");
            if (ch.lc0 < 0 || ch.lc0 + G.u + 1 > (int)tp.lcrow.size()) return bad(cat + "lcrow range");
            if (tp.lcrow[ch.lc0] != 0 || tp.lcrow[ch.lc0 + G.u] != ch.nrows || ch.nrows > GROWS) return bad(cat + "feature rows");
            std::vector<int> used(G.u, 0);
            for (int lc = 0; lc < G.u; ++lc) {
                const int r0 = tp.lcrow[ch.lc0 + lc], r1 = tp.lcrow[ch.lc0 + lc + 1];
                if (r1 < r0 || ((r1 - r0) & 3)) return bad(cat + "camera rows not a multiple of 4");
            }
            for (int o = ch.o0; o < ch.o1; ++o) {
                const int lc = tp.obs_lc[o], row = tp.obs_row[o];
                const int r0 = tp.lcrow[ch.lc0 + lc], r1 = tp.lcrow[ch.lc0 + lc + 1];
                if (row < r0 || row + 2 > r1 || ((row - r0) & 1)) return bad(cat + "feature row of observation " + S(o));
                if (row - r0 != 2 * used[lc]) return bad(cat + "feature rows not in observation order");
                ++used[lc];
            }
            for (int lc = 0; lc < G.u; ++lc) {
                const int r0 = tp.lcrow[ch.lc0 + lc], r1 = tp.lcrow[ch.lc0 + lc + 1];
                if (((2 * used[lc] + 3) & ~3) != r1 - r0) return bad(cat + "camera row padding");
            }
            q = G.p0 + ch.q1;
        }
        if (q != G.p1) return bad(at + "chunks do not cover the points");
        // ba_gschur wave batches: whole points, <= WB_OBS observations, <= WB_PTS points
        q = G.p0;
        if (G.nb < 1 || G.b0 < 0 || G.b0 + G.nb > (int)tp.bat.size()) return bad(at + "batch range");
        for (int b = 0; b < G.nb; ++b) {
            const Batch& B = tp.bat[G.b0 + b];
            if (B.p0 != q || B.p1 < B.p0 || B.p1 > G.p1 || B.p1 - B.p0 > WB_PTS) return bad(at + "batch points");
            if (B.o0 != pt_start[B.p0] || B.o1 != pt_start[B.p1] || B.o1 - B.o0 > WB_OBS) return bad(at + "batch observations");
            for (int p = B.p0; p < B.p1; ++p) {   // the lane map holds one lane per (point, camera)
                char seen[UMAX] = {};
                for (int o = pt_start[p]; o < pt_start[p + 1]; ++o) {
                    if (seen[tp.obs_lc[o]]) return bad(at + "two observations of one point in one camera (not big)");
                    seen[tp.obs_lc[o]] = 1;
                }
            }
            q = B.p1;
        }
        if (q != G.p1) return bad(at + "batches do not cover the points");
    }
    if (next_p != P) return bad("groups do not cover the points");
    // camera slot lists
    if ((int)tp.cref_start.size() != C + 1 || tp.cref_start[C] != (int)tp.gcam.size() || (int)tp.cref.size() != (int)tp.gcam.size())
        return bad("camera slot lists");
    for (int cm = 0; cm < C; ++cm)
        for (int e = tp.cref_start[cm]; e < tp.cref_start[cm + 1]; ++e)
            if (tp.cref[e] < 0 || tp.cref[e] >= (int)tp.gcam.size() || tp.gcam[tp.cref[e]] != cm) return bad("slot of camera " + S(cm));
    // assembly: every entry's reads inside its group's block
    for (size_t t = 0; t < tp.tasks.size(); ++t) {
        const ATask& T = tp.tasks[t];
        if (T.l0 < 0 || T.l1 < T.l0 || T.l1 > (int)tp.ents.size()) return bad("task " + S((long long)t) + ": entry range");
        if (T.type == 0 && (T.a < 0 || T.b < T.a || T.b >= C)) return bad("task " + S((long long)t) + ": pose pair");
        if (T.type == 1 && (T.a < 0 || T.a >= C)) return bad("task " + S((long long)t) + ": camera");
        if (T.type == 2 && (T.b < 0 || T.b >= K * K + K)) return bad("task " + S((long long)t) + ": intrinsics output");
        if (T.type < 0 || T.type > 2) return bad("task type");
        const int rows = T.type == 2 ? K : 6, cols = T.type == 0 ? 6 : K;
        for (int e = T.l0; e < T.l1; ++e) {
            const AEnt& E = tp.ents[e];
            if (E.dim < K || (E.dim - K) % 6) return bad("entry " + S(e) + ": dim");
            if (E.rg < 0 || E.rg + rows > tp.rg_total) return bad("entry " + S(e) + ": rhs outside rg");
            if (E.big) {
                if (E.b0 < 0 || E.b0 + 3LL * rows > tp.h_total || E.b1 < 0 || E.b1 + 3LL * cols > tp.h_total)
                    return bad("entry " + S(e) + ": H rows outside hbig");
            } else if (E.b0 < 0 || E.b0 + (long long)(rows - 1) * E.dim + cols > tp.sg_total) {
                return bad("entry " + S(e) + ": block outside sg");
            }
        }
    }
    return "";
}

// Everything problem-dependent of a context: the locality order, the point groups, the device
// copies of the topology and the state buffers (reused when they are large enough), the
// parameters.  The factorization plan is kept when the camera co-visibility and the border are
// unchanged (ensure_plan), else rebuilt at the next run.  Used by create and by sfmx_ba_update
// (the reference's BundleAdjustment call after every registered camera, SfM.cpp:235 / :371).
// A camera bucket's ordered points and point groups, kept between calls.  Offsets are local to the
// bucket (points, observations) and to each sub-segment (groups never span SEG_PTS points).
struct Bucket {
    std::vector<int> pts;           // caller points in the internal order
    std::vector<int> cpts, rank;    // the same points in caller order; rank[j] = internal position of cpts[j]
    std::vector<int> lpt;           // bucket-local pt_start (pts.size() + 1)
    std::vector<int> roc;           // per internal observation: its camera
    std::vector<short> lc, row;     // obs_lc / obs_row (ba_group.hpp)
    std::vector<uint32_t> cpairs;   // the camera pairs (a << 16 | b, a < b) some point of the bucket connects
    std::vector<std::pair<uint64_t, int>> kp, kp2;   // ordering scratch: (key, caller position) per piece
                                                     // sorted, then merged
    std::vector<int> m;                         // observations per point (caller order)
    std::vector<std::vector<uint32_t>> pcp;     // co-visible pairs per piece of OPIECE internal points
    std::vector<int> sub;           // sub-segment starts in points (+ the end)
    std::vector<TopoSeg> topo;      // per sub-segment, offsets local to the bucket / sub-segment
    int no = 0;                     // observations
    int64_t io0 = -1;               // its observations' offset in the device arrays of the last load (-1: none)
    int64_t io0_new = 0;            // and in the layout being built
    int ip0 = 0;                    // its first internal point
    bool dirty = true;
};
// Caller-order copy of one block of SHB caller points: what an update compares to find changed points.
constexpr int SHB = 1024;   // (r05: 4096 before; finer work items for the compare and the shadow copies)
struct Shadow {
    std::vector<int> cnt, oc;       // observations per point; their cameras
    std::vector<double> xy;         // their pixels
    bool valid = false;
};
struct HostScratch {
    bool valid = false;             // the caches describe the last successfully loaded problem
    int P = 0, K = 0, kb = 0, gpts = 0;
    std::vector<int> pbucket;       // caller point -> bucket
    std::vector<Bucket> bk;
    std::vector<Shadow> sh;
    View view;
    Topology tp;                    // the merged topology of the last load
    std::vector<int> pt_start;      // internal pt_start of the last load
    std::vector<int> iperm;         // caller point -> internal point (the inverse of pperm)
    int n_dirty = 0;                // buckets redone by the last load
    double tm[9] = {};              // host_setup phases (ms): view, compare, bucket lists, order + groups, layout, merge, tasks,
                                    // shadows; [8] the ordering part of [3] (keys, sort, co-visible pairs)
};
void destroy_scratch(HostScratch* h) { delete h; }

// The host half of a load: the locality order and point groups of `pb`, redoing only the buckets
// whose points changed since the last load described by hs (incremental: an unchanged point-major
// problem prefix, the same K, key width and group size), then merged: tp (every group kernel's
// topology), pperm (internal -> caller point), operm (internal -> caller observation), pt_start.  A
// fresh load (incremental = false) runs every bucket through the same code, so both give the same
// layout bit for bit (tests/test_ba_host.py).  hs.valid stays false until the caller confirms
// the device half (load_problem).
void build_operm(const HostScratch& hs, int O, std::vector<int>& operm);
void host_setup(const sfmx_ba_problem* pb, int K, int gpts, bool incremental, HostScratch& hs, std::vector<int>& pperm,
                std::vector<int>* operm, const std::function<void(const std::vector<uint64_t>&)>& on_covis = nullptr) {
    const int P = pb->n_points, C = pb->n_cams, O = pb->n_obs;
    using clk = std::chrono::steady_clock;
    auto tick = [t = clk::now()](double& slot) mutable {
        const auto n = clk::now();
        slot = std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
    };
    View& v = hs.view;
    make_view(pb, v);
    tick(hs.tm[0]);
    const KeyBits kb = key_bits(C);
    const int nbk = std::max(1, (C + BUCKET_CAMS - 1) / BUCKET_CAMS);
    incremental = incremental && hs.valid && v.pm && hs.K == K && hs.kb == kb.kb && hs.gpts == gpts;
    const int Pold = incremental ? hs.P : 0;
    hs.valid = false;
    if ((int)hs.bk.size() < nbk) hs.bk.resize(nbk);
    for (int b = 0; b < (int)hs.bk.size(); ++b) hs.bk[b].dirty = !incremental || b >= nbk;
    hs.pbucket.resize(std::max(P, Pold));
    // changed points: per caller block, compare with the shadow; a changed point dirties its old
    // and its new bucket
    const int nblk_old = (Pold + SHB - 1) / SHB, nblk = (P + SHB - 1) / SHB;
    hs.sh.resize(std::max(nblk, nblk_old));
    std::vector<char> dirty(hs.bk.size(), incremental ? 0 : 1), bchanged(hs.sh.size(), 1);
    std::mutex mu;
    sfmx::parallel_items((int)hs.sh.size(), [&](int k) {
        const int p0 = k * SHB, p1 = std::min(P, p0 + SHB), q1 = std::min(Pold, p0 + SHB);
        Shadow& S = hs.sh[k];
        std::vector<int> mark;   // buckets this block dirties
        if (incremental && S.valid && p1 == q1) {
            const int o0 = p0 < P ? v.start[p0] : O, o1 = p1 > p0 ? v.start[p1] : o0;
            bool same = (int)S.oc.size() == o1 - o0;
            for (int p = p0; same && p < p1; ++p) same = S.cnt[p - p0] == v.start[p + 1] - v.start[p];
            same = same && std::memcmp(S.oc.data(), pb->obs_cam + o0, sizeof(int) * (size_t)(o1 - o0)) == 0 &&
                   std::memcmp(S.xy.data(), pb->obs_xy + 2 * (size_t)o0, 16 * (size_t)(o1 - o0)) == 0;
            if (same) { bchanged[k] = 0; return; }
        }
        // point by point (old contents from the shadow when it is valid)
        std::vector<int> soff;
        if (S.valid) {
            soff.assign(S.cnt.size() + 1, 0);
            for (size_t i = 0; i < S.cnt.size(); ++i) soff[i + 1] = soff[i] + S.cnt[i];
        }
        for (int p = p0; p < std::max(p1, incremental ? q1 : p1); ++p) {
            const bool now = p < P, before = incremental && S.valid && p < q1;
            bool same = now && before;
            if (same) {
                const int i = p - p0, n = v.start[p + 1] - v.start[p];
                same = S.cnt[i] == n && std::memcmp(S.oc.data() + soff[i], pb->obs_cam + v.start[p], sizeof(int) * n) == 0 &&
                       std::memcmp(S.xy.data() + 2 * (size_t)soff[i], pb->obs_xy + 2 * (size_t)v.start[p], 16 * (size_t)n) == 0;
            }
            if (same) continue;
            if (incremental && p < Pold) mark.push_back(hs.pbucket[p]);
            if (now) {
                int minc;
                point_key(pb, v, p, kb, &minc);
                hs.pbucket[p] = bucket_of(minc);
                mark.push_back(hs.pbucket[p]);
            }
        }
        if (!mark.empty()) {
            std::lock_guard<std::mutex> lk(mu);
            for (int b : mark) dirty[b] = 1;
        }
    });
    for (size_t b = 0; b < hs.bk.size(); ++b) hs.bk[b].dirty = hs.bk[b].dirty || dirty[b];
    hs.pbucket.resize(P);
    tick(hs.tm[1]);
    // the dirty buckets' points, in caller order (ties of the sort keep it)
    {   // (fixed caller ranges on the worker pool, concatenated in range order)
        constexpr int LP = 32;
        std::vector<int> slot(hs.bk.size(), -1), dl;
        for (int b = 0; b < nbk; ++b)
            if (hs.bk[b].dirty) { slot[b] = (int)dl.size(); dl.push_back(b); hs.bk[b].pts.clear(); }
        const int nd = (int)dl.size();
        std::vector<std::vector<int>> part((size_t)LP * nd);
        if (nd > 0) {
            sfmx::parallel_items(LP, [&](int r) {
                const int p0 = (int)((int64_t)P * r / LP), p1 = (int)((int64_t)P * (r + 1) / LP);
                for (int p = p0; p < p1; ++p) {
                    const int sl = slot[hs.pbucket[p]];
                    if (sl >= 0) part[(size_t)r * nd + sl].push_back(p);
                }
            });
            sfmx::parallel_items(nd, [&](int k) {
                Bucket& B = hs.bk[dl[k]];
                size_t n = 0;
                for (int r = 0; r < LP; ++r) n += part[(size_t)r * nd + k].size();
                B.pts.reserve(n);
                for (int r = 0; r < LP; ++r) B.pts.insert(B.pts.end(), part[(size_t)r * nd + k].begin(), part[(size_t)r * nd + k].end());
            });
        }
    }
    tick(hs.tm[2]);
    // order + groups of every dirty bucket, in parallel
    std::vector<int> todo;
    for (int b = 0; b < nbk; ++b) if (hs.bk[b].dirty) todo.push_back(b);
    hs.n_dirty = (int)todo.size();
    // (1) per dirty bucket: keys, order, observation lists, co-visible pairs, sub-segments, in pieces of
    // OPIECE points on the worker pool (r05: the ring-closing bucket holds ~9000 points, one thread per
    // bucket made it the critical path); (2) every sub-segment's groups
    constexpr int OPIECE = 1024;
    std::vector<std::pair<int, int>> pieces;   // (bucket, first point)
    for (int b : todo) {
        Bucket& B = hs.bk[b];
        const int np = (int)B.pts.size();
        // the caller's arrays are read in caller order only (ascending addresses; r03 read them in the
        // sorted order, a cache miss per point on a bucket spread over the whole problem)
        B.cpts.swap(B.pts);
        B.pts.resize(np);
        B.kp.resize(np);
        B.m.resize(np);
        for (int q = 0; q < np; q += OPIECE) pieces.emplace_back(b, q);
    }
    sfmx::parallel_items((int)pieces.size(), [&](int t) {   // keys and observation counts
        Bucket& B = hs.bk[pieces[t].first];
        const int j0 = pieces[t].second, j1 = std::min((int)B.cpts.size(), j0 + OPIECE);
        for (int j = j0; j < j1; ++j) {
            int minc;
            const int p = B.cpts[j];
            B.kp[j] = {point_key(pb, v, p, kb, &minc), j};
            B.m[j] = v.start[p + 1] - v.start[p];
        }
        radix_sort_keys(B.kp.data() + j0, (size_t)(j1 - j0), kb.kb * kb.nk);   // the piece, stably
    });
    sfmx::parallel_items((int)todo.size(), [&](int t) {   // the order (stable radix sort of the keys)
        Bucket& B = hs.bk[todo[t]];
        const int np = (int)B.pts.size();
        {   // (key, caller order): the pieces' sorted runs merged pairwise, bottom-up (std::merge takes the
            // first run's element on ties, so the result is the stable order of the key)
            B.kp2.resize(np);
            auto by_key = [](const std::pair<uint64_t, int>& x, const std::pair<uint64_t, int>& y) { return x.first < y.first; };
            std::vector<std::pair<uint64_t, int>>*src = &B.kp, *dst = &B.kp2;
            for (int w = OPIECE; w < np; w *= 2) {
                for (int i = 0; i < np; i += 2 * w) {
                    const int m = std::min(np, i + w), e = std::min(np, i + 2 * w);
                    std::merge(src->begin() + i, src->begin() + m, src->begin() + m, src->begin() + e, dst->begin() + i, by_key);
                }
                std::swap(src, dst);
            }
            if (src != &B.kp2) std::copy(src->begin(), src->end(), B.kp2.begin());
        }
        const std::vector<std::pair<uint64_t, int>>& kps = B.kp2;
        B.lpt.assign(np + 1, 0);
        B.rank.resize(np);
        for (int i = 0; i < np; ++i) {
            const int j = kps[i].second;
            B.pts[i] = B.cpts[j];
            B.rank[j] = i;
            B.lpt[i + 1] = B.lpt[i] + B.m[j];
        }
        B.no = B.lpt[np];
        B.roc.resize(B.no);
        B.lc.assign(B.no, 0);
        B.row.assign(B.no, 0);
        B.sub.clear();
        for (int q = 0; q < np; q += SEG_PTS) B.sub.push_back(q);
        B.sub.push_back(np);
        B.topo.resize(B.sub.size() - 1);
        B.pcp.resize((np + OPIECE - 1) / OPIECE);
    });
    const size_t cwords = ((size_t)C * C + 63) / 64;
    sfmx::parallel_items((int)pieces.size(), [&](int t) {   // observation cameras (then the pieces' co-visible pairs)
        Bucket& B = hs.bk[pieces[t].first];
        const int j0 = pieces[t].second, j1 = std::min((int)B.cpts.size(), j0 + OPIECE);
        for (int j = j0; j < j1; ++j) {   // (caller order: ascending addresses)
            const int p = B.cpts[j];
            for (int a = v.start[p], k = B.lpt[B.rank[j]]; a < v.start[p + 1]; ++a, ++k) B.roc[k] = pb->obs_cam[v.obs(a)];
        }
    });
    sfmx::parallel_items((int)pieces.size(), [&](int t) {
        Bucket& B = hs.bk[pieces[t].first];
        const int j0 = pieces[t].second, j1 = std::min((int)B.cpts.size(), j0 + OPIECE);
        // the piece's internal points [j0, j1): pairs deduplicated through a per-thread bit table
        thread_local std::vector<uint64_t> mark;
        if (mark.size() < cwords) mark.assign(cwords, 0);
        std::vector<uint32_t>& out = B.pcp[j0 / OPIECE];
        out.clear();
        for (int i = j0; i < j1; ++i)
            for (int x = B.lpt[i]; x < B.lpt[i + 1]; ++x)
                for (int y = x + 1; y < B.lpt[i + 1]; ++y) {
                    const int a = std::min(B.roc[x], B.roc[y]), b = std::max(B.roc[x], B.roc[y]);
                    if (a == b) continue;
                    const size_t bit = (size_t)a * C + b;
                    if ((mark[bit >> 6] >> (bit & 63)) & 1) continue;
                    mark[bit >> 6] |= 1ull << (bit & 63);
                    out.push_back((uint32_t)a << 16 | (uint32_t)b);
                }
        for (uint32_t q : out) {   // leave the table clear for the thread's next piece
            const size_t bit = (size_t)(q >> 16) * C + (q & 0xffff);
            mark[bit >> 6] &= ~(1ull << (bit & 63));
        }
    });
    sfmx::parallel_items((int)todo.size(), [&](int t) {   // the bucket's pairs: the pieces' lists, deduplicated
        Bucket& B = hs.bk[todo[t]];
        thread_local std::vector<uint64_t> mark;
        if (mark.size() < cwords) mark.assign(cwords, 0);
        B.cpairs.clear();
        for (const auto& pc : B.pcp)
            for (uint32_t q : pc) {
                const size_t bit = (size_t)(q >> 16) * C + (q & 0xffff);
                if ((mark[bit >> 6] >> (bit & 63)) & 1) continue;
                mark[bit >> 6] |= 1ull << (bit & 63);
                B.cpairs.push_back(q);
            }
        for (uint32_t q : B.cpairs) {
            const size_t bit = (size_t)(q >> 16) * C + (q & 0xffff);
            mark[bit >> 6] &= ~(1ull << (bit & 63));
        }
    });
    {
        double t1;
        auto t = tick;
        t(t1);
        hs.tm[8] = t1;
    }
    std::vector<std::pair<int, int>> segs;   // (bucket, sub-segment)
    for (int b : todo)
        for (int j = 0; j + 1 < (int)hs.bk[b].sub.size(); ++j) segs.emplace_back(b, j);
    sfmx::parallel_items((int)segs.size(), [&](int t) {   // disjoint observation ranges of lc / row
        Bucket& B = hs.bk[segs[t].first];
        const int j = segs[t].second;
        topo_segment(B.sub[j], B.sub[j + 1], K, gpts, C, B.lpt, B.roc.data(), B.lc.data(), B.row.data(), B.topo[j]);
    });
    hs.bk.resize(nbk);
    tick(hs.tm[3]);
    // layout: buckets in order
    int ip = 0;
    int64_t io = 0;
    for (Bucket& B : hs.bk) { B.ip0 = ip; B.io0_new = io; ip += (int)B.pts.size(); io += B.no; }
    // pperm, pt_start: per bucket, in parallel (operm only when asked: the solve never reads it)
    pperm.resize(P);
    hs.iperm.resize(P);
    std::vector<int>& pts = hs.pt_start;
    pts.resize(P + 1);
    pts[P] = O;
    sfmx::parallel_items(nbk, [&](int b) {
        const Bucket& B = hs.bk[b];
        const int np = (int)B.pts.size();
        for (int i = 0; i < np; ++i) {
            pperm[B.ip0 + i] = B.pts[i];
            hs.iperm[B.pts[i]] = B.ip0 + i;
            pts[B.ip0 + i] = (int)(B.io0_new + B.lpt[i]);
        }
    });
    if (operm) build_operm(hs, O, *operm);
    tick(hs.tm[4]);
    // merge the groups: bucket / sub-segment offsets -> internal ones
    Topology& tp = hs.tp;
    tp.clear();
    {   // every segment's offsets first (serial, one entry per segment), then the copies on the worker pool
        struct SegOff { const Bucket* B; const TopoSeg* g; size_t grp, chk, bat, gcam, lcrow; long long sg, h; int rg; };
        std::vector<SegOff> so;
        SegOff o{nullptr, nullptr, 0, 0, 0, 0, 0, 0, 0, 0};
        for (const Bucket& B : hs.bk)
            for (size_t j = 0; j < B.topo.size(); ++j) {
                const TopoSeg& g = B.topo[j];
                o.B = &B; o.g = &g;
                so.push_back(o);
                o.grp += g.grp.size(); o.chk += g.chk.size(); o.bat += g.bat.size(); o.gcam += g.gcam.size();
                o.lcrow += g.lcrow.size(); o.sg += g.sg_total; o.h += g.h_total; o.rg += g.rg_total;
                tp.dp_max = std::max(tp.dp_max, g.dp_max);
            }
        tp.grp.resize(o.grp); tp.chk.resize(o.chk); tp.bat.resize(o.bat); tp.gcam.resize(o.gcam); tp.lcrow.resize(o.lcrow);
        tp.sg_total = o.sg; tp.h_total = o.h; tp.rg_total = o.rg;
        sfmx::parallel_items((int)so.size(), [&](int k) {
            const SegOff& s0 = so[k];
            const TopoSeg& g = *s0.g;
            const int dp = s0.B->ip0, dobs = (int)s0.B->io0_new;
            const int cam0 = (int)s0.gcam, ch0 = (int)s0.chk, b0 = (int)s0.bat, l0 = (int)s0.lcrow;
            for (size_t i = 0; i < g.grp.size(); ++i) {
                Grp G = g.grp[i];
                G.o0 += dobs; G.o1 += dobs; G.p0 += dp; G.p1 += dp;
                G.cam_off += cam0; G.ch0 += ch0; G.b0 += b0; G.rg_off += s0.rg;
                if (G.big) G.h_off += s0.h; else G.sg_off += s0.sg;
                tp.grp[s0.grp + i] = G;
            }
            for (size_t i = 0; i < g.chk.size(); ++i) {
                Chunk ch = g.chk[i];
                ch.o0 += dobs; ch.o1 += dobs; ch.lc0 += l0;
                tp.chk[s0.chk + i] = ch;
            }
            for (size_t i = 0; i < g.bat.size(); ++i) {
                Batch bt = g.bat[i];
                bt.o0 += dobs; bt.o1 += dobs; bt.p0 += dp; bt.p1 += dp;
                tp.bat[s0.bat + i] = bt;
            }
            std::copy(g.gcam.begin(), g.gcam.end(), tp.gcam.begin() + s0.gcam);
            std::copy(g.lcrow.begin(), g.lcrow.end(), tp.lcrow.begin() + s0.lcrow);
        });
    }
    tick(hs.tm[5]);
    {   // the problem's co-visibility: the union of the buckets' pairs (kept ones included)
        tp.covis.assign(((size_t)C * C + 63) / 64, 0);
        for (const Bucket& B : hs.bk)
            for (uint32_t q : B.cpairs) {
                const size_t a = q >> 16, b = q & 0xffff, b1 = a * C + b, b2 = b * C + a;
                tp.covis[b1 >> 6] |= 1ull << (b1 & 63);
                tp.covis[b2 >> 6] |= 1ull << (b2 & 63);
            }
    }
    if (on_covis) on_covis(tp.covis);   // (load_problem: the plan of this graph starts here, on its own thread)
    finish_topology(C, K, tp);
    tick(hs.tm[6]);
    // shadows of the changed blocks (point-major problems only: the next update compares slices)
    sfmx::parallel_items(nblk, [&](int k) {
        Shadow& S = hs.sh[k];
        if (!bchanged[k] && S.valid) return;
        S.valid = v.pm;
        if (!v.pm) return;
        const int p0 = k * SHB, p1 = std::min(P, p0 + SHB), o0 = v.start[p0], o1 = v.start[p1];
        S.cnt.resize(p1 - p0);
        for (int p = p0; p < p1; ++p) S.cnt[p - p0] = v.start[p + 1] - v.start[p];
        S.oc.assign(pb->obs_cam + o0, pb->obs_cam + o1);
        S.xy.assign(pb->obs_xy + 2 * (size_t)o0, pb->obs_xy + 2 * (size_t)o1);
    });
    hs.sh.resize(nblk);
    hs.P = P; hs.K = K; hs.kb = kb.kb; hs.gpts = gpts;
    tick(hs.tm[7]);
}

// internal -> caller observation of the layout hs describes (the buckets' io0_new offsets and the view
// of the problem it was built from): sfmx_ba_jacobian and the layout checks only
void build_operm(const HostScratch& hs, int O, std::vector<int>& operm) {
    operm.resize(O);
    const View& v = hs.view;
    sfmx::parallel_items((int)hs.bk.size(), [&](int b) {   // in caller order (see phase 1)
        const Bucket& B = hs.bk[b];
        for (size_t j = 0; j < B.cpts.size(); ++j) {
            const int p = B.cpts[j], i = B.rank[j];
            for (int a = v.start[p], k = (int)B.io0_new + B.lpt[i]; a < v.start[p + 1]; ++a, ++k) operm[k] = v.obs(a);
        }
    });
}

// The global observation arrays of the merged layout (diagnostics / checks): obs_cam, obs_lc, obs_row.
[[maybe_unused]] void gather_obs(const HostScratch& hs, int O, std::vector<int>& roc, std::vector<short>& lc, std::vector<short>& row) {
    roc.resize(O); lc.resize(O); row.resize(O);
    for (const Bucket& B : hs.bk) {
        std::copy(B.roc.begin(), B.roc.end(), roc.begin() + B.io0_new);
        std::copy(B.lc.begin(), B.lc.end(), lc.begin() + B.io0_new);
        std::copy(B.row.begin(), B.row.end(), row.begin() + B.io0_new);
    }
}

// ba_glin workgroups resident at once on this device (its occupancy at the launch's LDS size times
// the CUs); 0 when unknown (then full-size groups)
int group_slots(sfmx_ba_ctx* c, int K) {
    if (const char* e = SFMX_DIAG_ENV("SFMX_BA_SLOTS")) return std::atoi(e);   // A/B: 0 = full-size groups
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) return 0;
    const size_t lds = glin_lds(K);
    const void* f = K == 1 ? (const void*)ba_glin<1, false> : K == 3 ? (const void*)ba_glin<3, false> : (const void*)ba_glin<7, false>;
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 256, lds) != hipSuccess || nb <= 0) return 0;
    return nb * prop.multiProcessorCount;
}

// The intrinsics border of a problem (no context state touched): one camera -> its block; several
// cameras -> the blocks some POSE names (pose_intr), in block order, back to back.  Poses and cameras
// are replicated on every rank of a point-sharded solve, so every rank derives the same border (K,
// single / multi kernels, column layout) and the collectives agree in size and meaning (ADVICE r03:
// a border from the rank's own observations could differ between ranks).  A camera only unobserved
// poses name gets zero Jacobian columns (its step is 0); the reference's scenes have no such pose.
struct IntrLayout {
    int K = 0, intr_len = 0;
    bool multi = false;
    double cx = 0, cy = 0;
    std::vector<int> isrc, pim;
    std::vector<double2> pcc;
};
int intr_layout(const sfmx_ba_problem* pb, IntrLayout& L) {
    const int C = pb->n_cams;
    L = IntrLayout{};
    L.cx = pb->cx; L.cy = pb->cy;
    if (pb->n_intr == 0) {
        L.K = L.intr_len = pb->cam_model;
        for (int j = 0; j < L.K; ++j) L.isrc.push_back(j);
        return SFMX_OK;
    }
    const int M = pb->n_intr;
    std::vector<int> used(M, 0), first(M, -1), off(M + 1, 0);
    for (int m = 0; m < M; ++m) off[m + 1] = off[m] + pb->intr_model[m];
    L.intr_len = off[M];
    for (int cm = 0; cm < C; ++cm) used[pb->pose_intr[cm]] = 1;
    int kb = 0, nused = 0;
    for (int m = 0; m < M; ++m)
        if (used[m]) {
            ++nused;
            first[m] = kb;
            for (int i = 0; i < pb->intr_model[m]; ++i) L.isrc.push_back(off[m] + i);
            kb += pb->intr_model[m];
        }
    if (nused <= 1) {   // one referenced camera: the single-block kernels with its block and centre
        const int m = (int)(std::find(used.begin(), used.end(), 1) - used.begin());
        L.K = m < M ? pb->intr_model[m] : pb->intr_model[0];
        if (m == M) for (int i = 0; i < L.K; ++i) L.isrc.push_back(i);
        L.cx = pb->intr_center[2 * (m < M ? m : 0)];
        L.cy = pb->intr_center[2 * (m < M ? m : 0) + 1];
        return SFMX_OK;
    }
    if (kb > SFMX_BA_MAX_INTR)
        return fail(SFMX_ECAPACITY, "the referenced cameras hold " + std::to_string(kb) +
                                        " intrinsics parameters; at most SFMX_BA_MAX_INTR = 7 are supported");
    L.multi = true;
    L.K = kb <= 1 ? 1 : kb <= 3 ? 3 : 7;   // the kernels' border widths; padding columns stay 0
    while ((int)L.isrc.size() < L.K) L.isrc.push_back(-1);
    L.pim.assign(std::max(C, 1), 1);
    L.pcc.assign(std::max(C, 1), double2{0.0, 0.0});
    for (int cm = 0; cm < C; ++cm) {
        const int m = pb->pose_intr[cm];
        L.pim[cm] = pb->intr_model[m] | (first[m] << 4);
        L.pcc[cm] = double2{pb->intr_center[2 * m], pb->intr_center[2 * m + 1]};
    }
    return SFMX_OK;
}

// every check that can refuse a problem runs before any context state changes; a failure
// after that point (allocation, upload) leaves the context marked unloaded, and run / get / set
// refuse it (SFMX_ESTATE) until an update succeeds.
int load_problem(sfmx_ba_ctx* c, const sfmx_ba_problem* caller, double validate_ms = 0.0) {
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
    DeviceGuard dg(c->device);
    if (6 * (int64_t)caller->n_cams > MAX_NPAD)
        return fail(SFMX_EINVAL, "too many cameras for the reduced camera system (6C > 16384)");
    IntrLayout L;
    RC(intr_layout(caller, L));
    if (!c->hscr) c->hscr = new (std::nothrow) HostScratch();
    if (!c->hscr) return fail(SFMX_ENOMEM, "host allocation");
    HostScratch& hs = *c->hscr;
    const int P = caller->n_points, C = caller->n_cams, O = caller->n_obs, K = L.K;
    // the previous load's device layout is reusable only if it completed
    const bool incremental = c->loaded && hs.valid;
    c->loaded = false;
    const int slots = group_slots(c, K);
    int gpts = group_points(P, slots);
    if (c->opt.max_group_points > 0) gpts = std::min(gpts, std::min(GPTS, (int)c->opt.max_group_points));
#ifdef SFMX_DIAG
    if (const char* e = SFMX_DIAG_ENV("SFMX_BA_GPTS")) gpts = std::max(1, std::min(GPTS, std::atoi(e)));   // tiny-group tests
    const bool force_fresh = SFMX_DIAG_ENV("SFMX_BA_FRESH") != nullptr;   // A/B: every load rebuilds every bucket
#else
    const bool force_fresh = false;
#endif
    if (c->plan_pending) { c->plan_th->wait(); c->plan_pending = false; }   // (a failed earlier load's)
    // the co-visibility as soon as the ordering has it: S_cc's pattern (the pose-pair tasks are exactly
    // its edges) and, on one rank, the plan of a new graph computed beside the rest of the load
    auto on_covis = [c, C](const std::vector<uint64_t>& covis) {
        c->adj.assign((size_t)C * C, 0);
        for (int a = 0; a < C; ++a)
            for (int b = 0; b < C; ++b) {
                const size_t bit = (size_t)a * C + b;
                if (a != b && ((covis[bit >> 6] >> (bit & 63)) & 1)) c->adj[bit] = 1;
            }
        if (multirank(c) || (c->planned && c->adj == c->plan_adj)) return;
        c->plan_pre_adj = c->adj;
        c->plan_pre_mode = plan_mode();
        if (!c->plan_th) c->plan_th = new sfmx::SideThread();
        c->plan_pending = true;
        c->plan_th->submit([c, C] { sfmx::ba::make_plan(C, c->plan_pre_adj, c->plan_pre_mode, c->plan_pre); });
    };
    host_setup(caller, K, gpts, incremental && !force_fresh, hs, c->pperm, nullptr, on_covis);
    c->operm.clear();
    Topology& tp = hs.tp;
    const std::vector<int>& pt_start = hs.pt_start;
    c->setup_ms[5] = ms_since(t_start);
    c->setup_ms[7] = validate_ms;
    for (int i = 0; i < 8; ++i) c->setup_ms[8 + i] = hs.tm[i];
    c->setup_ms[16] = c->setup_ms[17] = 0.0;
    auto bail = [](int rc) { return rc; };
    // per-problem state starts over
    c->scaled = false;
    c->unscaled_wr = nullptr;
    HIPCHK(hipStreamSynchronize(c->st));   // (a failed earlier load may have left copies from the arena in flight)
    c->stage_off = 0;
    c->P = P; c->C = C; c->O = O;
    c->K = K; c->intr_len = L.intr_len; c->multi = L.multi; c->cx = L.cx; c->cy = L.cy;
    c->n_intr = caller->n_intr;
    c->isrc.swap(L.isrc);
    std::vector<int>& pim_h = L.pim;
    std::vector<double2>& pcc_h = L.pcc;
    if (c->plan_K != K) c->planned = false;   // the border sizes S, W and the Schur terms
    c->ne = 3 * (int64_t)P;
    c->nf = 6 * C + K;
    c->n = c->ne + c->nf;
    c->RW = K + 1;
#ifdef SFMX_DIAG
    if (SFMX_DIAG_ENV("SFMX_BA_TRACE"))
        fprintf(stderr, "sfmx ba: P %d slots %d points/group %d groups %zu dp_max %d buckets %zu redone %d\n", P, slots, gpts,
                tp.grp.size(), tp.dp_max, hs.bk.size(), hs.n_dirty);
    {   // the diagnostic library checks every topology it uploads
        std::vector<int> roc;
        gather_obs(hs, O, roc, tp.obs_lc, tp.obs_row);
        const std::string why = check_topology(P, C, O, K, pt_start, roc.data(), tp);
        if (!why.empty()) return bail(fail(SFMX_EINTERNAL, "BA topology check: " + why));
    }
#endif
    c->setup_ms[6] = hs.n_dirty;   // buckets redone (the ordering's and the groups' ms are [5] and [0])
    // local camera co-visibility (the pose blocks this rank's points create): c->adj, from on_covis
    // a plan is reused only when this graph is the one it was built from; ranks of a sharded solve
    // rebuild on every update (the plan needs the co-visibility all-reduced over all of them)
    if (c->adj != c->plan_adj || multirank(c)) c->planned = false;
    c->setup_ms[0] = ms_since(t_start);
    c->ngroups = (int)tp.grp.size();
    c->ntasks = (int)tp.tasks.size();
    c->nslots = (int)tp.gcam.size();
    {
        const size_t wreg = K == 1 ? gs_wreg(1, tp.dp_max) : K == 3 ? gs_wreg(3, tp.dp_max) : gs_wreg(7, tp.dp_max);
        size_t nb_max = 0;   // batch descriptors of one group in LDS (2 doubles each)
        for (const Grp& G : tp.grp) nb_max = std::max<size_t>(nb_max, G.nb);
        c->gs_nt = std::min(4, std::max(1, tp.dp_max / 16));
        c->lds_schur = sizeof(double) * std::max<size_t>({4 * wreg + 2 * nb_max, (size_t)tp.dp_max * (tp.dp_max + 1) + tp.dp_max,
                                                          (size_t)gs_comb(c->gs_nt), 16});
    }
    c->lds_lin = glin_lds(K);
    {
        hipError_t e = hipSuccess;
#define LDSATTR(KK)                                                                                                  \
        for (const void* f : {(const void*)ba_gschur<KK, 1, false>, (const void*)ba_gschur<KK, 2, false>,              \
                              (const void*)ba_gschur<KK, 3, false>, (const void*)ba_gschur<KK, 4, false>,             \
                              (const void*)ba_gschur<KK, 1, true>, (const void*)ba_gschur<KK, 2, true>,               \
                              (const void*)ba_gschur<KK, 3, true>, (const void*)ba_gschur<KK, 4, true>})              \
            if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds_schur); \
        for (const void* f : {(const void*)ba_glin<KK, false>, (const void*)ba_glin<KK, true>})                    \
            if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds_lin);
        if (K == 1) { LDSATTR(1); } else if (K == 3) { LDSATTR(3); } else { LDSATTR(7); }
#undef LDSATTR
        if (e != hipSuccess) return bail(fail(SFMX_EDEVICE, std::string("LDS attribute: ") + hipGetErrorString(e)));
    }
    hipStream_t st = c->st;
    int rc;
    const auto t_up = clk::now();
    // Observation arrays (pixels, cameras, local camera, feature row) in the new layout, written into
    // the second set of buffers and then swapped in: an unchanged bucket moves on the device
    // (ba_relayout, 24 B per observation), a redone one is uploaded from the host.
    std::vector<ObsMove> moves;
    int64_t up_obs = 0;
    for (const Bucket& B : hs.bk) {
        if (!B.dirty && B.io0 >= 0) {
            for (int64_t k = 0; k < B.no; k += RELAYOUT_CHUNK)
                moves.push_back(ObsMove{B.io0 + k, B.io0_new + k, (int)std::min<int64_t>(RELAYOUT_CHUNK, B.no - k), 0});
        } else {
            up_obs += B.no;
        }
    }
    {   // every staged upload of this call (256-B rounded parts): one arena, no mid-call waits
        auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
        size_t total = r(sizeof(ObsMove) * moves.size()) + r(4 * (size_t)(P + 1)) + r(sizeof(Grp) * tp.grp.size()) +
                       r(sizeof(Chunk) * tp.chk.size()) + r(sizeof(Batch) * tp.bat.size()) + r(4 * tp.gcam.size()) +
                       r(4 * tp.lcrow.size()) + r(sizeof(ATask) * tp.tasks.size()) + r(sizeof(AEnt) * tp.ents.size()) +
                       r(4 * tp.cref_start.size()) + r(4 * tp.cref.size()) + r(4 * pim_h.size()) +
                       r(sizeof(double2) * pcc_h.size()) + r(24 * (size_t)P + 48 * (size_t)C + 8 * (size_t)K) + 4096;
        for (const Bucket& B : hs.bk)
            if (B.dirty || B.io0 < 0) total += r(16 * (size_t)B.no) + r(4 * (size_t)B.no) + 2 * r(2 * (size_t)B.no);
        RC(stage_reserve(c, total));
    }
    const size_t so = std::max<size_t>(O, 1);
    if ((rc = c->obs_xy_b.alloc(16 * so)) || (rc = c->obs_cam_b.alloc(4 * so)) || (rc = c->obs_lc_b.alloc(2 * so)) ||
        (rc = c->obs_row_b.alloc(2 * so)))
        return bail(rc);
    if (!moves.empty()) {
        ObsMove* h = static_cast<ObsMove*>(stage_bytes(c, sizeof(ObsMove) * moves.size()));
        if (!h) return bail(fail(SFMX_ENOMEM, "pinned staging buffer"));
        std::memcpy(h, moves.data(), sizeof(ObsMove) * moves.size());
        RC(c->moves.alloc(sizeof(ObsMove) * moves.size()));
        HIPCHK(hipMemcpyAsync(c->moves.p, h, sizeof(ObsMove) * moves.size(), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(ba_relayout, dim3((unsigned)moves.size()), dim3(256), 0, st, c->moves.as<ObsMove>(),
                           c->obs_xy.as<double2>(), c->obs_cam.as<int>(), c->obs_lc.as<short>(), c->obs_row.as<short>(),
                           c->obs_xy_b.as<double2>(), c->obs_cam_b.as<int>(), c->obs_lc_b.as<short>(), c->obs_row_b.as<short>());
        HIPCHK(hipGetLastError());
    }
    {   // the redone buckets: pixels gathered from the caller's array while copied into pinned staging
        const double2* xy = reinterpret_cast<const double2*>(caller->obs_xy);
        const View& v = hs.view;
        for (const Bucket& B : hs.bk) {
            if ((!B.dirty && B.io0 >= 0) || B.no == 0) continue;
            double2* h = static_cast<double2*>(stage_bytes(c, 16 * (size_t)B.no));
            int* hc = static_cast<int*>(stage_bytes(c, 4 * (size_t)B.no));
            short* hl = static_cast<short*>(stage_bytes(c, 2 * (size_t)B.no));
            short* hr = static_cast<short*>(stage_bytes(c, 2 * (size_t)B.no));
            if (!h || !hc || !hl || !hr) return bail(fail(SFMX_ENOMEM, "pinned staging buffer"));
            const int64_t o0 = B.io0_new;
            const int np = (int)B.cpts.size();
            sfmx::parallel_ranges(np, B.no >= 8192 ? 16 : 1, [&](int64_t j0, int64_t j1) {   // caller order
                for (int64_t j = j0; j < j1; ++j) {
                    const int p = B.cpts[j];
                    for (int a = v.start[p], k = B.lpt[B.rank[j]]; a < v.start[p + 1]; ++a, ++k) h[k] = xy[v.obs(a)];
                }
            });
            std::memcpy(hc, B.roc.data(), 4 * (size_t)B.no);
            std::memcpy(hl, B.lc.data(), 2 * (size_t)B.no);
            std::memcpy(hr, B.row.data(), 2 * (size_t)B.no);
            HIPCHK(hipMemcpyAsync(c->obs_xy_b.as<double2>() + o0, h, 16 * (size_t)B.no, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(c->obs_cam_b.as<int>() + o0, hc, 4 * (size_t)B.no, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(c->obs_lc_b.as<short>() + o0, hl, 2 * (size_t)B.no, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(c->obs_row_b.as<short>() + o0, hr, 2 * (size_t)B.no, hipMemcpyHostToDevice, st));
        }
    }
    std::swap(c->obs_xy, c->obs_xy_b);
    std::swap(c->obs_cam, c->obs_cam_b);
    std::swap(c->obs_lc, c->obs_lc_b);
    std::swap(c->obs_row, c->obs_row_b);
    c->setup_up_obs = up_obs;
    // the observations' points from the point-major CSR on the device (no upload of rop)
    RC(c->obs_point.alloc(4 * so));
    UploadSet up;   // the layout's CSR and topology arrays in one copy
    up.add(c->pt_start, pt_start);
    up.add(c->grp, tp.grp); up.add(c->chk, tp.chk); up.add(c->bat, tp.bat); up.add(c->gcam, tp.gcam);
    up.add(c->lcrow, tp.lcrow); up.add(c->tasks, tp.tasks); up.add(c->ents, tp.ents); up.add(c->cref_start, tp.cref_start);
    up.add(c->cref, tp.cref); up.add(c->pim, pim_h); up.add(c->pcc, pcc_h);
    const auto t_topo = clk::now();
    if ((rc = up.flush(c, c->topo_arena))) return bail(rc);
    c->setup_ms[19] = ms_since(t_topo);
    if (P && O) {
        hipLaunchKernelGGL(ba_obs_point, dim3(nblk(P)), dim3(256), 0, st, P, c->pt_start.as<int>(), c->obs_point.as<int>());
        HIPCHK(hipGetLastError());
    }

    const size_t n = c->n;
    const size_t ncams = (size_t)C * ncp(K) + K * (K + 1) / 2 + K;
    struct { Buf* b; size_t bytes; } allocs[] = {
        {&c->x, 8 * n}, {&c->cand, 8 * n}, {&c->scale, 8 * n}, {&c->colsq, 8 * n}, {&c->colsq2, 8 * n},
        {&c->grad, 8 * n}, {&c->grad2, 8 * n}, {&c->sol, 8 * n},
        {&c->Wr, 8 * so * WST}, {&c->Wr2, 8 * so * WST}, {&c->PR, 8 * (size_t)std::max(P, 1) * npr(K)},
        {&c->PR2, 8 * (size_t)std::max(P, 1) * npr(K)}, {&c->camsum, 8 * (ncams + 5)}, {&c->camsum2, 8 * (ncams + 5)},
        {&c->plt, 72 * (size_t)std::max(P, 1)}, {&c->sg, 8 * (size_t)std::max<long long>(tp.sg_total, 1)},
        {&c->rg, 8 * (size_t)std::max(tp.rg_total, 1)}, {&c->hbig, 8 * (size_t)std::max<long long>(tp.h_total, 1)},
        {&c->gpart, 8 * (size_t)std::max(c->nslots, 1) * ncp(K)}, {&c->gpl, 8 * (size_t)std::max(c->ngroups, 1) * GP_N},
        {&c->scal, 8 * SC_N}, {&c->failf, 64}, {&c->lmst, 8 * LM_N}, {&c->camscr, 8 * (ncams + 5)},
        {&c->partA, 8 * (size_t)nblk(std::max<int64_t>(O, n))}};
    const double up_ms = ms_since(t_up);
    const auto t_al = clk::now();
    for (auto& a : allocs) if ((rc = a.b->alloc(a.bytes))) return bail(rc);
    c->setup_ms[1] = ms_since(t_al);
    const auto t_up2 = clk::now();
    HIPCHK(hipMemsetAsync(c->gpl.p, 0, c->gpl.bytes, st));
    // scale = 1 until (and unless) Jacobi scaling sets it
    hipLaunchKernelGGL(ba_fill, dim3(nblk((int64_t)n)), dim3(256), 0, st, (int64_t)n, 1.0, c->scale.as<double>());
    HIPCHK(hipGetLastError());
    // one rank: the factorization plan of the new co-visibility is built (host) while this call's copies
    // and relayout run, and its own uploads end with the stream synchronisation; ranks of a sharded
    // solve plan at run (the plan's co-visibility all-reduce needs every rank)
    const bool plan_now = !multirank(c);
    const auto t_par = clk::now();
    if ((rc = set_params(c, caller, !plan_now))) return bail(rc);
    c->setup_ms[18] = ms_since(t_par);
    c->setup_ms[2] = up_ms + ms_since(t_up2);
    c->setup_ms[3] = 0.0;
    c->setup_ms[4] = ms_since(t_start);
    if (plan_now && (rc = ensure_plan(c))) {   // (adds its time to setup_ms[3] / [4])
        (void)hipStreamSynchronize(st);         // the copies from the staging arena end before it is reused
        return bail(rc);
    }
    {
        const auto t_wait = clk::now();
        HIPCHK(hipStreamSynchronize(st));   // (an unchanged plan returns at once: the copies end here)
        c->setup_ms[17] += ms_since(t_wait);
    }
    for (Bucket& B : hs.bk) { B.io0 = B.io0_new; B.dirty = false; }
    hs.valid = true;
    c->loaded = true;
    return SFMX_OK;
}

int init_ctx(sfmx_ba_ctx* c, const sfmx_ba_options* opt) {
    sfmx_ba_options o;
    sfmx_ba_default_options(&o);
    if (opt) o = *opt;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(SFMX_EDEVICE, "no HIP device visible");
    if (o.device < 0 || o.device >= ndev) return fail(SFMX_EINVAL, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, o.device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SFMX_EDEVICE, "sfmx BA kernels are built for gfx950 only");
    c->device = o.device;
    c->opt = o;
    DeviceGuard dg(c->device);
    if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) return fail(SFMX_EDEVICE, "stream");
    for (auto& e : c->ev) if (hipEventCreate(&e) != hipSuccess) return fail(SFMX_EDEVICE, "event");
    if (hipHostMalloc(reinterpret_cast<void**>(&c->hs), sizeof(double) * sfmx_ba_ctx::HS_N,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return fail(SFMX_ENOMEM, "pinned scalar buffer");
    std::memset(c->hs, 0, sizeof(double) * sfmx_ba_ctx::HS_N);
    return SFMX_OK;
}

int create(const sfmx_ba_problem* caller, const sfmx_ba_options* opt, sfmx_ba_ctx** out) {
    const auto t0 = std::chrono::steady_clock::now();
    RC(validate(caller));
    const double vms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    auto* c = new (std::nothrow) sfmx_ba_ctx();
    if (!c) return fail(SFMX_ENOMEM, "host allocation");
    int rc = init_ctx(c, opt);
    if (!rc) rc = load_problem(c, caller, vms);
    if (rc) { delete c; return rc; }
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
    o->max_group_points = 0;
    o->_reserved_opt = 0;
    return SFMX_OK;
}

int sfmx_ba_create(const sfmx_ba_problem* problem, const sfmx_ba_options* opt, sfmx_ba_ctx** out) {
    if (!out) return fail(SFMX_EINVAL, "null out");
    *out = nullptr;
    return create(problem, opt, out);
}

int sfmx_ba_comm_unique_id(void* id) {
    if (!id) return fail(SFMX_EINVAL, "null id");
    const sfmx::RcclApi& r = sfmx::rccl_api();
    if (!r.ok) return fail(SFMX_EDEVICE, "RCCL (librccl.so.1) not loadable");
    const ncclResult_t e = r.GetUniqueId(static_cast<ncclUniqueId*>(id));
    if (e != ncclSuccess) return fail(SFMX_EDEVICE, std::string("ncclGetUniqueId: ") + r.GetErrorString(e));
    return SFMX_OK;
}

int sfmx_ba_set_comm(sfmx_ba_ctx* c, const void* id, int32_t nranks, int32_t rank) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(SFMX_EINVAL, "bad communicator arguments");
    const sfmx::RcclApi& r = sfmx::rccl_api();
    if (!r.ok) return fail(SFMX_EDEVICE, "RCCL (librccl.so.1) not loadable");
    DeviceGuard dg(c->device);
    if (c->comm) { (void)r.CommDestroy(c->comm); c->comm = nullptr; }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    ncclComm_t comm = nullptr;
    const ncclResult_t e = r.CommInitRank(&comm, nranks, uid, rank);
    if (e != ncclSuccess) return fail(SFMX_EDEVICE, std::string("ncclCommInitRank: ") + r.GetErrorString(e));
    c->comm = comm;
    c->planned = false;   // the plan needs the co-visibility of every rank
    return SFMX_OK;
}

int sfmx_ba_set_allreduce(sfmx_ba_ctx* c, sfmx_allreduce_fn fn, void* user) {
    if (!c) return fail(SFMX_EINVAL, "null context");
    c->ar = fn;
    c->ar_user = user;
    c->planned = false;   // the plan needs the co-visibility of every rank (a one-rank load planned on its own)
    return SFMX_OK;
}

int sfmx_ba_run(sfmx_ba_ctx* c, int32_t max_iterations, sfmx_ba_summary* summary, double* trace, int32_t trace_cap) {
    if (!c || !summary) return fail(SFMX_EINVAL, "null context/summary");
    if (!c->loaded) return fail(SFMX_ESTATE, "no problem loaded (the last update failed)");
    int nt = 0;
    RC(run_lm(c, max_iterations, summary, trace, trace_cap, &nt));
    return nt;
}

int sfmx_ba_get(sfmx_ba_ctx* c, sfmx_ba_problem* pb) {
    if (!c || !pb) return fail(SFMX_EINVAL, "null context/problem");
    if (!c->loaded) return fail(SFMX_ESTATE, "no problem loaded (the last update failed)");
    DeviceGuard dg(c->device);
    const double* x = c->x.as<double>();
    c->stage_off = 0;   // nothing staged is in flight: every upload was synchronised
    // x = [points | poses | border] in one copy; the points scattered into the caller's order (r05d:
    // one copy and one wait beat four pieces scattered as they land: 0.31 vs 0.40 ms at C5)
    const size_t n = 3 * (size_t)c->P + 6 * (size_t)c->C + (size_t)c->K;
    double* h = static_cast<double*>(stage_bytes(c, sizeof(double) * std::max<size_t>(n, 1)));
    if (!h) return fail(SFMX_ENOMEM, "pinned staging buffer");
    if (n) HIPCHK(hipMemcpyAsync(h, x, sizeof(double) * n, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (!c->hscr || (int)c->hscr->iperm.size() != c->P) return fail(SFMX_EINTERNAL, "BA get: no layout of the loaded problem");
    const int* ip = c->hscr->iperm.data();   // caller -> internal: the caller's array written in order
    sfmx::parallel_ranges(c->P, c->P >= 16384 ? 16 : 1, [&](int64_t p0, int64_t p1) {   // write-back in caller order
        for (int64_t p = p0; p < p1; ++p)
            for (int i = 0; i < 3; ++i) pb->points[3 * (size_t)p + i] = h[3 * (size_t)ip[p] + i];
    });
    if (c->C) std::memcpy(pb->poses, h + c->ne, sizeof(double) * 6 * c->C);
    const double* iv = h + c->ne + 6 * (size_t)c->C;
    for (int j = 0; j < c->K; ++j) if (c->isrc[j] >= 0) pb->intr[c->isrc[j]] = iv[j];   // unreferenced cameras: untouched
    return SFMX_OK;
}

int sfmx_ba_set(sfmx_ba_ctx* c, const sfmx_ba_problem* pb) {
    if (!c || !pb) return fail(SFMX_EINVAL, "null context/problem");
    if (!c->loaded) return fail(SFMX_ESTATE, "no problem loaded (the last update failed)");
    if (pb->n_points != c->P || pb->n_cams != c->C || pb->n_intr != c->n_intr || (c->n_intr == 0 && pb->cam_model != c->K))
        return fail(SFMX_EINVAL, "topology mismatch");
    return set_params(c, pb);
}

int sfmx_ba_set_phase_timing(sfmx_ba_ctx* c, int32_t on) {
    if (!c) return fail(SFMX_EINVAL, "null context");
    c->phases = on != 0;
    return SFMX_OK;
}

int sfmx_ba_phase_ms(sfmx_ba_ctx* c, double* ms, int32_t n) {
    if (!c || !ms) return fail(SFMX_EINVAL, "null");
    const int m = std::min<int>(n, 5);
    for (int i = 0; i < m && i < 4; ++i) ms[i] = c->phase_ms[i];
    if (m > 4) ms[4] = c->dag_fallbacks;
    return m;
}

int sfmx_ba_destroy(sfmx_ba_ctx* c) {
    delete c;
    return SFMX_OK;
}

int sfmx_ba_update(sfmx_ba_ctx* c, const sfmx_ba_problem* pb) {
    if (!c) return fail(SFMX_EINVAL, "null context");
    const auto t0 = std::chrono::steady_clock::now();
    RC(validate(pb));
    return load_problem(c, pb, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

int sfmx_ba_setup_ms(sfmx_ba_ctx* c, double* ms, int32_t n) {
    if (!c || !ms) return fail(SFMX_EINVAL, "null");
    const int m = std::min<int>(n, sfmx_ba_ctx::SETUP_N);
    for (int i = 0; i < m; ++i) ms[i] = c->setup_ms[i];
    return m;
}

// sfmx_ba_solve keeps one context per device between calls (the reference solves a growing scene
// after every registered camera, SfM.cpp:235 / :371): stream, events, pinned memory and device
// buffers are reused, the plan too while the co-visibility holds.  Plain pointers, no static
// destructor (the HIP runtime may be gone at process exit); sfmx_ba_release_cache frees them.
namespace {
std::mutex g_solve_mu;
sfmx_ba_ctx* g_solve_ctx[64] = {};
}

int sfmx_ba_release_cache(void) {
    std::lock_guard<std::mutex> lk(g_solve_mu);
    for (auto& c : g_solve_ctx) { delete c; c = nullptr; }
    return SFMX_OK;
}

int sfmx_ba_solve(sfmx_ba_problem* pb, const sfmx_ba_options* opt, sfmx_ba_summary* summary, double* trace,
                  int32_t trace_cap) {
    if (!summary) return fail(SFMX_EINVAL, "null summary");
    RC(validate(pb));
    sfmx_ba_options o;
    sfmx_ba_default_options(&o);
    if (opt) o = *opt;
    if (o.device < 0 || o.device >= 64) return fail(SFMX_EINVAL, "device index out of range");
    std::lock_guard<std::mutex> lk(g_solve_mu);
    sfmx_ba_ctx*& c = g_solve_ctx[o.device];
    int rc = SFMX_OK;
    if (!c) {
        rc = create(pb, &o, &c);
        if (rc) { c = nullptr; return rc; }
    } else {
        c->opt = o;
        rc = load_problem(c, pb);
    }
    int nt = 0;
    if (!rc) rc = run_lm(c, 0, summary, trace, trace_cap, &nt);
    if (!rc) rc = sfmx_ba_get(c, pb);   // write-back (BundleAdjustment.cpp:97-138)
    if (rc) { delete c; c = nullptr; }  // a failed call leaves no half-loaded context behind
    return rc ? rc : nt;
}

int sfmx_ba_jacobian(const sfmx_ba_problem* pb, int32_t device, double* r, double* Je, double* Jc, double* Ji) {
    sfmx_ba_options o;
    sfmx_ba_default_options(&o);
    o.device = device;
    sfmx_ba_ctx* c = nullptr;
    RC(create(pb, &o, &c));
    build_operm(*c->hscr, c->O, c->operm);
    int rc = SFMX_OK;
    {
        DeviceGuard dg(c->device);
        double cost;
        rc = eval_jacobian(c, c->x.as<double>(), &cost);
        if (!rc) {
            const int O = c->O, K = c->K, F = 20 + 2 * K, KL = c->intr_len;
            std::vector<double> h((size_t)F * O);
            if (O && (hipMemcpy(h.data(), c->J.p, sizeof(double) * h.size(), hipMemcpyDeviceToHost) != hipSuccess))
                rc = fail(SFMX_EDEVICE, "D2H");
            for (int q = 0; q < O && !rc; ++q) {
                const size_t o = (size_t)c->operm[q];   // caller's observation index
                for (int j = 0; j < 2; ++j) {
                    if (r) r[2 * o + j] = h[(size_t)q * F + j];
                    for (int i = 0; i < 3; ++i) if (Je) Je[6 * o + 3 * j + i] = h[(size_t)q * F + (2 + 3 * j + i)];
                    for (int i = 0; i < 6; ++i) if (Jc) Jc[12 * o + 6 * j + i] = h[(size_t)q * F + (8 + 6 * j + i)];
                    if (Ji) {   // the caller's intr layout; columns of other cameras 0
                        for (int i = 0; i < KL; ++i) Ji[2 * (size_t)KL * o + KL * j + i] = 0.0;
                        for (int i = 0; i < K; ++i)
                            if (c->isrc[i] >= 0) Ji[2 * (size_t)KL * o + KL * j + c->isrc[i]] = h[(size_t)q * F + (20 + K * j + i)];
                    }
                }
            }
        }
    }
    delete c;
    return rc;
}

#ifdef SFMX_DIAG
// diagnostic build only, no device needed: the host part of load_problem (locality order, point
// groups / chunks / batches / assembly tasks at `gpts` points per group, 0 = GPTS) and
// check_topology on it.  -> number of groups, or SFMX_EINTERNAL with the violation as last error.
// ms (optional, 3 entries): host time of the ordering + groups (host_setup), 0, and the check.
int sfmx_ba_debug_check_topology(const sfmx_ba_problem* pb, int32_t gpts, double* ms) {
    RC(validate(pb));
    IntrLayout L;
    RC(intr_layout(pb, L));
    using clk = std::chrono::steady_clock;
    auto d = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto t0 = clk::now();
    HostScratch hs;
    std::vector<int> pperm, operm, roc;
    host_setup(pb, L.K, gpts > 0 ? std::min(gpts, GPTS) : GPTS, false, hs, pperm, &operm);
    const auto t1 = clk::now();
    gather_obs(hs, pb->n_obs, roc, hs.tp.obs_lc, hs.tp.obs_row);
    const std::string why = check_topology(pb->n_points, pb->n_cams, pb->n_obs, L.K, hs.pt_start, roc.data(), hs.tp);
    int pose_pairs = 0;   // S_cc's nonzero 6 x 6 pose blocks (a <= b) the groups create: the factorization's pattern
    for (const ATask& t : hs.tp.tasks) pose_pairs += t.type == 0;
    if (ms) { ms[0] = d(t0, t1); ms[1] = pose_pairs; ms[2] = d(t1, clk::now()); }
    if (!why.empty()) return fail(SFMX_EINTERNAL, "BA topology check: " + why);
    return (int)hs.tp.grp.size();
}

// diagnostic build only: the camera co-visibility S_cc's pattern comes from (the pose pairs of the point
// groups, C x C bytes into adj) for `gpts` points per group (0 = GPTS), without a device.
int sfmx_ba_debug_adjacency(const sfmx_ba_problem* pb, int32_t gpts, uint8_t* adj) {
    RC(validate(pb));
    IntrLayout L;
    RC(intr_layout(pb, L));
    HostScratch hs;
    std::vector<int> pperm, operm;
    host_setup(pb, L.K, gpts > 0 ? std::min(gpts, GPTS) : GPTS, false, hs, pperm, &operm);
    const int C = pb->n_cams;
    std::memset(adj, 0, (size_t)C * C);
    for (const ATask& t : hs.tp.tasks)
        if (t.type == 0 && t.a != t.b) adj[(size_t)t.a * C + t.b] = adj[(size_t)t.b * C + t.a] = 1;
    return (int)hs.tp.grp.size();
}

// The host half of an update against a fresh load: problem a, then b on the same host caches (the
// incremental path), must give b's fresh layout exactly (orders, observation permutation, every
// topology array); -> buckets the update redid (out[0]) and all buckets (out[1]), or SFMX_EINTERNAL
// naming the first difference.  ms (optional, 11): the update's and the fresh load's host time, then
// the update's phases (HostScratch::tm).
int sfmx_ba_debug_incremental_check(const sfmx_ba_problem* a, const sfmx_ba_problem* b, int32_t gpts, int32_t* out,
                                    double* ms) {
    RC(validate(a));
    RC(validate(b));
    IntrLayout La, Lb;
    RC(intr_layout(a, La));
    RC(intr_layout(b, Lb));
    const int g = gpts > 0 ? std::min(gpts, GPTS) : GPTS;
    using clk = std::chrono::steady_clock;
    auto d = [](clk::time_point x, clk::time_point y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    HostScratch inc, fr;
    std::vector<int> pp, op, pp2, op2;
    host_setup(a, La.K, g, false, inc, pp, &op);
    for (Bucket& B : inc.bk) { B.io0 = B.io0_new; B.dirty = false; }
    inc.valid = true;
    const auto t0 = clk::now();
    host_setup(b, Lb.K, g, true, inc, pp, nullptr);   // (timed as the product runs it: no operm)
    const auto t1 = clk::now();
    host_setup(b, Lb.K, g, false, fr, pp2, nullptr);
    const auto t2 = clk::now();
    build_operm(inc, b->n_obs, op);
    build_operm(fr, b->n_obs, op2);
    if (ms) { ms[0] = d(t0, t1); ms[1] = d(t1, t2); for (int i = 0; i < 9; ++i) ms[2 + i] = inc.tm[i]; }
    if (out) { out[0] = inc.n_dirty; out[1] = (int)inc.bk.size(); }
    auto bytes = [](const auto& x, const auto& y) {
        return x.size() == y.size() && (x.empty() || std::memcmp(x.data(), y.data(), sizeof(x[0]) * x.size()) == 0);
    };
    const Topology &ti = inc.tp, &tf = fr.tp;
    std::vector<int> ri, rf;
    std::vector<short> li, lf, wi, wf;
    gather_obs(inc, b->n_obs, ri, li, wi);
    gather_obs(fr, b->n_obs, rf, lf, wf);
    const char* diff = !bytes(pp, pp2) ? "pperm" : !bytes(op, op2) ? "operm" : !bytes(inc.pt_start, fr.pt_start) ? "pt_start"
                     : !bytes(ri, rf) ? "obs_cam" : !bytes(li, lf) ? "obs_lc" : !bytes(wi, wf) ? "obs_row"
                     : !bytes(ti.grp, tf.grp) ? "groups" : !bytes(ti.chk, tf.chk) ? "chunks" : !bytes(ti.bat, tf.bat) ? "batches"
                     : !bytes(ti.gcam, tf.gcam) ? "gcam" : !bytes(ti.lcrow, tf.lcrow) ? "lcrow" : !bytes(ti.tasks, tf.tasks) ? "tasks"
                     : !bytes(ti.ents, tf.ents) ? "ents" : !bytes(ti.cref, tf.cref) ? "cref" : !bytes(ti.cref_start, tf.cref_start) ? "cref_start"
                     : (ti.sg_total != tf.sg_total || ti.h_total != tf.h_total || ti.rg_total != tf.rg_total || ti.dp_max != tf.dp_max) ? "totals"
                     : nullptr;
    if (diff) return fail(SFMX_EINTERNAL, std::string("incremental layout differs from the fresh one: ") + diff);
    return SFMX_OK;
}
#endif

#ifdef SFMX_DIAG
// diagnostic build only: the workgroups per CU the two launches whose occupancy is held by
// design actually get on this device: out[0] ba_gupdate<K> with its GUPDATE_LDS request (4: its static
// LDS + 33 KiB must keep 5 from fitting 160 KiB), out[1] ba_glin<K> at glin_lds(K) (2).
int sfmx_ba_debug_occupancy(int32_t K, int32_t* out) {
    if (!out || (K != 1 && K != 3 && K != 7)) return fail(SFMX_EINVAL, "K must be 1, 3 or 7");
    const void* gu = K == 1 ? (const void*)ba_gupdate<1, false> : K == 3 ? (const void*)ba_gupdate<3, false> : (const void*)ba_gupdate<7, false>;
    const void* gl = K == 1 ? (const void*)ba_glin<1, false> : K == 3 ? (const void*)ba_glin<3, false> : (const void*)ba_glin<7, false>;
    int a = 0, b = 0;
    const size_t lds = glin_lds(K);
    (void)hipFuncSetAttribute(gl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, gu, 256, GUPDATE_LDS));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, gl, 256, lds));
    out[0] = a;
    out[1] = b;
    return SFMX_OK;
}
#endif

#ifdef SFMX_DIAG
// diagnostic build only: the per-ticket timeline of the last chol_factor launch (ba_chol.hpp CHOL_TRACE),
// n_items x 16 int64 (stamps 0-13 in 100 MHz wall-clock ticks, [15] = XCC id << 32 | HW_ID)
int sfmx_ba_debug_chol_trace(long long* out, int32_t n_items) {
    if (n_items > sfmx::ba::CHOL_TRACE_MAX) n_items = sfmx::ba::CHOL_TRACE_MAX;
    if (n_items <= 0 || !out) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return SFMX_EDEVICE;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sfmx::ba::g_chol_trace), sizeof(long long) * 16 * n_items) != hipSuccess)
        return SFMX_EDEVICE;
    return n_items;
}
int sfmx_ba_debug_chol_items(sfmx_ba_ctx* c, int32_t* out, int32_t cap) {   // items (int4) of the current plan
    if (!c) return SFMX_EINVAL;
    const int n = c->n_ditems;
    if (out && cap >= 8 * n) {
        if (hipMemcpy(out, c->ditems.p, sizeof(int4) * n, hipMemcpyDeviceToHost) != hipSuccess) return SFMX_EDEVICE;
        if (hipMemcpy(out + 4 * n, c->dmask.p, sizeof(int4) * n, hipMemcpyDeviceToHost) != hipSuccess) return SFMX_EDEVICE;
    }
    return n;
}
#endif

#ifdef SFMX_BA_STAMPS
// diagnostic build only: read and clear the phase cycle totals (ba_group.hpp BA_STAMP)
int sfmx_ba_debug_stamps(unsigned long long* out, int32_t n) {
    if (n > 64) n = 64;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sfmx::ba::g_ba_stamps), sizeof(unsigned long long) * n) != hipSuccess) return SFMX_EDEVICE;
    std::vector<unsigned long long> z(64, 0);
    if (hipMemcpyToSymbol(HIP_SYMBOL(sfmx::ba::g_ba_stamps), z.data(), sizeof(unsigned long long) * 64) != hipSuccess) return SFMX_EDEVICE;
    return n;
}
#endif

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
