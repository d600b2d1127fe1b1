// SPDX-License-Identifier: MIT
// sfmx matcher — host driver behind the C ABI (include/sfmx.h).
//
// Mirrors the reference's strategy call
//   IFeatureMatchingStrategy::calculateShotMatches(scene, matcher, out)
//   (src/photogrammetrie/sfm/IFeatureMatchingStrategy.h:45-46, e.g.
//    UnorderedFeatureMatchingStrategy.cpp:27-90)
// followed by SfM::calculateShotMatches' filters (sfm/SfM.cpp:542-575):
//   set_images  = the descriptor matrices the Scene's shots own (CameraShot.h:39-42),
//                 uploaded once into an HBM pool and prepared (int8 + norms)
//   run         = the OpenMP pair loop (:40-88) as one batched launch sequence
//   fetch       = the vector<ShotMatches> hand-back, as packed DMatch lists
// No CPU fallback: every numeric step runs in the HIP kernels of
// match_kernels.hip; a missing/unsupported device returns SFMX_EDEVICE.
#include <hip/hip_runtime.h>
#include "diag.hpp"
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sfmx.h"
#include "match_common.hpp"

namespace sfmx {
hipError_t launch_prep_l2(const float*, int, int, int, int8_t*, int32_t*, int32_t*, int32_t*, int32_t*, hipStream_t);
hipError_t launch_probe_xor80(int8_t*, int64_t, hipStream_t);
hipError_t launch_publish_flags(const int32_t*, int, int32_t*, unsigned*, unsigned, hipStream_t);
hipError_t launch_prep_l2_batch(const PrepImg*, int, int, int8_t*, int32_t*, int32_t*, int32_t*, int32_t*, hipStream_t);
hipError_t launch_prep_f32(const float*, int, int, int, float*, hipStream_t);
hipError_t launch_prep_hamming(const uint8_t*, int, int, int, uint8_t*, hipStream_t);
hipError_t launch_sift_knn2(const WorkItem*, int, const PairDev*, const ImgDev*, const int8_t*, const int32_t*,
                            const int32_t*, const int32_t*, int32_t*, int32_t*, int, const int32_t*, WorkItem*,
                            int32_t*, int32_t*, float*, int2*, int32_t*, double, hipStream_t, hipEvent_t, int32_t*,
                            unsigned long long*);
hipError_t launch_sift_slow(const int2*, const int32_t*, const PairDev*, const ImgDev*, const int8_t*,
                            const int32_t*, int32_t*, float*, double, hipStream_t);
hipError_t launch_sift_f32(const WorkItem*, int, const PairDev*, const ImgDev*, const float*, int32_t*, float*,
                           double, hipStream_t);
hipError_t launch_orb_knn2(const WorkItem*, int, const PairDev*, const ImgDev*, const uint8_t*, int32_t*, float*,
                           double, hipStream_t);
hipError_t launch_prep_hamming_fp4(const uint8_t*, int, int, int, uint8_t*, int32_t*, hipStream_t);
hipError_t launch_orb_mfma(const WorkItem*, int, const PairDev*, const ImgDev*, const uint8_t*, const int32_t*,
                           int32_t*, int32_t*, int, const int32_t*, WorkItem*, int32_t*, int32_t*, float*, double,
                           hipStream_t, hipEvent_t, int32_t*, unsigned long long*);
int orb_variant();
int match_batches();
int pass2_variant();
hipError_t launch_two_pass_overlap(bool, const MatchBatch*, int, const WorkItem*, const PairDev*, const ImgDev*,
                                   const int8_t*, const int32_t*, const int32_t*, int32_t*, int32_t*, int, const int32_t*,
                                   int32_t*, float*, int2*, int32_t*, double, hipStream_t, hipEvent_t, int32_t*,
                                   unsigned long long*, const OverlapStreams&);
hipError_t launch_selftest_sqrt(int64_t, uint32_t*, hipStream_t);
int sift_variant();
int sift_block_queries(int variant);
hipError_t launch_assemble(const PairDev*, int, const ImgDev*, const int32_t*, const float*, int, int, int,
                           int64_t*, int32_t*, int64_t*, DMatchDev*, int32_t*, hipStream_t);
}  // namespace sfmx

using namespace sfmx;

namespace {

thread_local std::string g_last_error;
}  // namespace
void sfmx::set_last_error(const char* msg) { g_last_error = msg ? msg : ""; }
namespace {

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(e_ == hipErrorOutOfMemory ? SFMX_ENOMEM : SFMX_EDEVICE,               \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return SFMX_OK;
        if (p) (void)hipFree(p);
        p = nullptr; cap = 0;
        const size_t want = std::max<size_t>(bytes, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) { p = nullptr; return fail(SFMX_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)); }
        cap = want;
        return SFMX_OK;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// Pinned host staging for small H2D uploads (prep table, pair/work lists): truly
// asynchronous copies.  `busy` is recorded after the copies that read the buffer;
// a writer waits for it first, so a copy still in flight is never overwritten.
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipEvent_t busy = nullptr;
    bool pending = false;
    int ensure(size_t bytes) {
        if (pending) { (void)hipEventSynchronize(busy); pending = false; }
        if (bytes <= cap) return SFMX_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr; cap = 0;
        const size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) { p = nullptr; return fail(SFMX_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e)); }
        cap = want;
        return SFMX_OK;
    }
    int copied(hipStream_t st) {     // call after enqueueing the copies that read the buffer
        if (!busy && hipEventCreateWithFlags(&busy, hipEventDisableTiming) != hipSuccess) return fail(SFMX_EDEVICE, "hipEventCreate");
        if (hipEventRecord(busy, st) != hipSuccess) return fail(SFMX_EDEVICE, "hipEventRecord");
        pending = true;
        return SFMX_OK;
    }
    void release() {
        if (pending) (void)hipEventSynchronize(busy);
        if (busy) (void)hipEventDestroy(busy);
        if (p) (void)hipHostFree(p);
        p = nullptr; cap = 0; busy = nullptr; pending = false;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// Device guard: set the matcher's device for the duration of a call.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) { (void)hipGetDevice(&prev); (void)hipSetDevice(dev); }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

}  // namespace

struct sfmx_matcher {
    int device = 0;
    int norm = 0;
    bool orb_fp4 = false;   // ORB rows expanded to +-1 FP4 (MFMA path), else 32-byte rows (VALU path)
    int n_imgs = 0;
    std::vector<ImgDev> imgs;
    int64_t total_rows = 0;
    int max_rows = 0;
    bool any_nonintegral = false;
    DevBuf raw, desc8, normv, keyc, keyc2, f32, flags, imgs_d;
    // run state
    int n_pairs = 0;
    int64_t dense_total = 0;
    int64_t fp32_pairs = 0;
    DevBuf pairs_d, work_d, work32_d, dense_idx, dense_dist, slow_list, slow_count, counts, keep, offsets, out;
    DevBuf qlist, qcount;   // two-pass SIFT path: per pair, the queries the screening pass could not settle
    DevBuf qmask, top2;     // subset pass 2: per forwarded query its row-subset mask; per query the merged top-2 keys
    DevBuf porder, work2, work2_n;   // pair order (by train image) and the compacted pass-2 work list
    DevBuf unsettled;                // int32: pass-1 forwarded queries pass 2 never wrote (must stay 0)
    DevBuf prep_tab;                 // batched SIFT prep: one PrepImg per image
    PinnedBuf stage_prep, stage_run, stage_imgs, stage_flags; // pinned staging of the small uploads / flag readback
    int32_t* hflags = nullptr;   // host-coherent mapped: integrality flags [hflags_cap] + sequence word (publish_flags_kernel)
    int hflags_cap = 0;
    unsigned flag_seq = 0;
    // Run plan cache: the device pair/work lists of the last run stay valid while the
    // pair list, the images' row counts and integrality and the kernel variant are unchanged.
    std::vector<int32_t> plan_pairs;
    std::vector<int64_t> plan_imgs;
    int plan_variant = -1;
    bool plan_valid = false;
    int64_t plan_dense = 0;
    size_t plan_nwork = 0, plan_nwork32 = 0;
    int plan_max_nt = 0;
    bool has_run = false;
    // per run: start, main kernel end, run end, pass-1 end; a ring of EV_RING sets (r06) so the timing
    // of every run of a loop is readable afterwards (sfmx_matcher_timing_history) without a host sync
    // inside it; ev points at the current run's set
    static constexpr int EV_RING = 32;
    hipEvent_t evr[EV_RING][4] = {};
    hipEvent_t* ev = evr[0];
    long long runs = 0;
    bool ev_recorded = false;
    // overlapped two-pass matching (launch_two_pass_overlap): the plan's batches, two more streams
    std::vector<MatchBatch> batches;
    int plan_nb = 0;
    hipStream_t sx = nullptr, sp = nullptr;
    hipEvent_t ov_ev[3] = {nullptr, nullptr, nullptr};
    std::vector<hipEvent_t> bev;
    // r05: device-resident descriptors (set_images_device) are not waited on for their integrality:
    // the run assumes every image integral (SIFT descriptors always are) and the assumption is checked
    // when results are read (fetch / stats / device_results); a non-integral image then gets its fp32
    // rows and the last run is re-run on the exact paths.  The host no longer waits mid-step.
    bool flags_pending = false;
    unsigned flags_want = 0;
    hipStream_t flags_stream = nullptr;
    std::vector<const void*> last_src;     // the device descriptors of the last set_images_device
    hipStream_t run_stream = nullptr;      // the stream of the last run (the re-run is ordered behind it)
    hipEvent_t fix_ev[2] = {nullptr, nullptr};   // set-stream point / re-run end (resolve_flags)
    std::vector<int> last_cols;
    bool run_spec = false;                 // the last run assumed integrality not yet confirmed
    std::vector<int32_t> last_pairs;
    double last_ratio = 0.0;
    int last_distinct = 0, last_min_count = 0;
};

namespace {

int check_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(SFMX_EDEVICE, "no HIP device visible");
    if (dev < 0 || dev >= n) return fail(SFMX_EINVAL, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(SFMX_EDEVICE, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SFMX_EDEVICE, std::string("sfmx kernels are built for gfx950 only, device is ") + prop.gcnArchName);
    return SFMX_OK;
}

int set_images_impl(sfmx_matcher* m, const sfmx_desc* imgs, int n, int norm, hipStream_t st, bool device_src) {
    if (m) m->flags_pending = m->run_spec = false;   // (a pending check of earlier images is moot now)
    if (!m || (n > 0 && !imgs) || n < 0) return fail(SFMX_EINVAL, "null matcher/images");
    if (norm != SFMX_NORM_L2 && norm != SFMX_NORM_HAMMING) return fail(SFMX_EINVAL, "norm must be SFMX_NORM_L2 or SFMX_NORM_HAMMING");
    const int want_type = norm == SFMX_NORM_L2 ? SFMX_32F : SFMX_8U;
    const int max_cols = norm == SFMX_NORM_L2 ? SIFT_DIM : ORB_BYTES;
    for (int i = 0; i < n; ++i) {
        if (imgs[i].rows < 0 || imgs[i].cols < 0) return fail(SFMX_EINVAL, "negative descriptor shape");
        if (imgs[i].rows > 0 && imgs[i].type != want_type)
            return fail(SFMX_EINVAL, "descriptor type does not match norm (L2 needs CV_32F, HAMMING needs CV_8U)");
        if (imgs[i].rows > 0 && (imgs[i].cols < 1 || imgs[i].cols > max_cols))
            return fail(SFMX_EINVAL, "descriptor width unsupported (SIFT <= 128 floats, ORB <= 32 bytes)");
        if (imgs[i].rows >= (1 << 18))   // cv::BFMatcher asserts train rows < IMGIDX_ONE = 2^18 [ext]
            return fail(SFMX_EINVAL, "more than 2^18 - 1 descriptors in one image");
        if (imgs[i].rows > 0 && !imgs[i].data) return fail(SFMX_EINVAL, "null descriptor data");
    }
    DeviceGuard g(m->device);
    m->norm = norm;
    m->orb_fp4 = norm == SFMX_NORM_HAMMING && orb_variant() != 1;
    m->n_imgs = n;
    m->imgs.assign(n, ImgDev{});
    m->has_run = false;
    int64_t row = 0, raw_bytes = 0;
    std::vector<int64_t> raw_off(n);
    m->max_rows = 0;
    for (int i = 0; i < n; ++i) {
        ImgDev& d = m->imgs[i];
        d.rows = imgs[i].rows;
        d.rows_pad = (int32_t)align_up(d.rows, ROW_ALIGN);
        d.row0 = row;
        d.integral = 1;
        row += d.rows_pad;
        m->max_rows = std::max(m->max_rows, d.rows);
        const int64_t esz = norm == SFMX_NORM_L2 ? 4 : 1;
        raw_off[i] = raw_bytes;
        raw_bytes += align_up((int64_t)imgs[i].rows * imgs[i].cols * esz, 256);
    }
    m->total_rows = row;
    const int row_bytes = (norm == SFMX_NORM_L2 || m->orb_fp4) ? SIFT_DIM : ORB_BYTES;
    int rc;
    if ((rc = m->desc8.ensure((size_t)row * row_bytes))) return rc;
    if ((rc = m->flags.ensure(sizeof(int32_t) * std::max(n, 1)))) return rc;
    if ((rc = m->imgs_d.ensure(sizeof(ImgDev) * std::max(n, 1)))) return rc;
    if (norm == SFMX_NORM_L2 && (rc = m->normv.ensure((size_t)row * 4))) return rc;
    if ((norm == SFMX_NORM_L2 || m->orb_fp4) && (rc = m->keyc.ensure((size_t)row * 4))) return rc;
    if (norm == SFMX_NORM_L2 && (rc = m->keyc2.ensure((size_t)row * 4))) return rc;
    if (!device_src && (rc = m->raw.ensure((size_t)raw_bytes))) return rc;
    HIPCHK(hipMemsetAsync(m->flags.p, 0, sizeof(int32_t) * std::max(n, 1), st));
    std::vector<const void*> src(n);
    for (int i = 0; i < n; ++i) {
        const int64_t esz = norm == SFMX_NORM_L2 ? 4 : 1;
        const size_t bytes = (size_t)imgs[i].rows * imgs[i].cols * esz;
        if (device_src) src[i] = imgs[i].data;
        else {
            src[i] = m->raw.as<char>() + raw_off[i];
            if (bytes) HIPCHK(hipMemcpyAsync((void*)src[i], imgs[i].data, bytes, hipMemcpyHostToDevice, st));
        }
    }
    if (norm == SFMX_NORM_L2 && n > 0) {      // one launch for every image
        if ((rc = m->stage_prep.ensure(sizeof(PrepImg) * n))) return rc;
        if ((rc = m->prep_tab.ensure(sizeof(PrepImg) * n))) return rc;
        PrepImg* tab = m->stage_prep.as<PrepImg>();
        int max_pad = 0;
        for (int i = 0; i < n; ++i) {
            const ImgDev& d = m->imgs[i];
            tab[i] = PrepImg{(const float*)src[i], d.rows, imgs[i].cols, d.rows_pad, 0, d.row0};
            max_pad = std::max(max_pad, d.rows_pad);
        }
        HIPCHK(hipMemcpyAsync(m->prep_tab.p, tab, sizeof(PrepImg) * n, hipMemcpyHostToDevice, st));
        if ((rc = m->stage_prep.copied(st))) return rc;
        HIPCHK(launch_prep_l2_batch(m->prep_tab.as<PrepImg>(), n, max_pad, m->desc8.as<int8_t>(), m->normv.as<int32_t>(),
                                    m->keyc.as<int32_t>(), m->keyc2.as<int32_t>(), m->flags.as<int32_t>(), st));
    }
    for (int i = 0; i < n && norm != SFMX_NORM_L2; ++i) {
        const ImgDev& d = m->imgs[i];
        if (m->orb_fp4)
            HIPCHK(launch_prep_hamming_fp4((const uint8_t*)src[i], d.rows, imgs[i].cols, d.rows_pad,
                                           m->desc8.as<uint8_t>() + d.row0 * SIFT_DIM, m->keyc.as<int32_t>() + d.row0, st));
        else
            HIPCHK(launch_prep_hamming((const uint8_t*)src[i], d.rows, imgs[i].cols, d.rows_pad,
                                       m->desc8.as<uint8_t>() + d.row0 * ORB_BYTES, st));
    }
    m->any_nonintegral = false;
    if (norm == SFMX_NORM_L2 && n > 0) {
        if (n > m->hflags_cap) {
            if (m->hflags) (void)hipHostFree(m->hflags);
            m->hflags = nullptr;
            m->hflags_cap = 0;
            if (hipHostMalloc(reinterpret_cast<void**>(&m->hflags), sizeof(int32_t) * (n + 4),
                              hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
                return fail(SFMX_ENOMEM, "hipHostMalloc (integrality flags)");
            m->hflags_cap = n;
            m->hflags[n] = 0;
        }
        unsigned* hseq = reinterpret_cast<unsigned*>(m->hflags + m->hflags_cap);
        const unsigned want = ++m->flag_seq;
        HIPCHK(launch_publish_flags(m->flags.as<int32_t>(), n, m->hflags, hseq, want, st));
        if (device_src) {   // (see flags_pending) every image integral until the flags say otherwise
            m->flags_pending = true;
            m->flags_want = want;
            m->flags_stream = st;
            m->last_src = src;
            m->last_cols.resize(n);
            for (int i = 0; i < n; ++i) m->last_cols[i] = imgs[i].cols;
        }
        for (unsigned spins = 1; !device_src; ++spins) {   // host buffers: the flags before the run is planned
            if (__atomic_load_n(hseq, __ATOMIC_ACQUIRE) == want) break;
            if ((spins & 255) == 0) {
                const hipError_t e = hipStreamQuery(st);
                if (e != hipSuccess && e != hipErrorNotReady) return fail(SFMX_EDEVICE, std::string("set_images: ") + hipGetErrorString(e));
                if (e == hipSuccess && __atomic_load_n(hseq, __ATOMIC_ACQUIRE) != want)
                    return fail(SFMX_EINTERNAL, "set_images: stream drained without the flag handoff");
            }
            __builtin_ia32_pause();
        }
        const int32_t* fl = m->hflags;
        for (int i = 0; i < n && !device_src; ++i) {
            m->imgs[i].integral = fl[i] ? 0 : 1;
            m->any_nonintegral |= fl[i] != 0;
        }
        if (m->any_nonintegral) {
            // every image gets its fp32 rows: a pair takes the fp32 path when EITHER side is
            // non-integral, and then reads both sides from this buffer (an integral partner's rows
            // were left unwritten before r03: stale memory, caught by test_non_integral_fp32_fallback)
            if ((rc = m->f32.ensure((size_t)row * SIFT_DIM * 4))) return rc;
            for (int i = 0; i < n; ++i) {
                const ImgDev& d = m->imgs[i];
                HIPCHK(launch_prep_f32((const float*)src[i], d.rows, imgs[i].cols, d.rows_pad,
                                       m->f32.as<float>() + d.row0 * SIFT_DIM, st));
            }
        }
    }
#ifdef SFMX_DIAG
    if (norm == SFMX_NORM_L2 && SFMX_DIAG_ENV("SFMX_PROBE_XOR80"))   // timing probe only (wrong results)
        HIPCHK(launch_probe_xor80(m->desc8.as<int8_t>(), (int64_t)row * SIFT_DIM, st));
#endif
    if (n > 0) {
        if ((rc = m->stage_imgs.ensure(sizeof(ImgDev) * n))) return rc;
        std::memcpy(m->stage_imgs.p, m->imgs.data(), sizeof(ImgDev) * n);
        HIPCHK(hipMemcpyAsync(m->imgs_d.p, m->stage_imgs.p, sizeof(ImgDev) * n, hipMemcpyHostToDevice, st));
        if ((rc = m->stage_imgs.copied(st))) return rc;
    }
    if (!device_src) HIPCHK(hipStreamSynchronize(st));   // host buffers may be released by the caller
    return SFMX_OK;
}

int run_impl(sfmx_matcher* m, const int32_t* pairs, int n_pairs, double ratio, int distinct, int min_count,
             hipStream_t st) {
    if (!m) return fail(SFMX_EINVAL, "null matcher");
    if (m->norm == 0) return fail(SFMX_ESTATE, "run before set_images");
    if (n_pairs < 0 || (n_pairs > 0 && !pairs)) return fail(SFMX_EINVAL, "bad pair list");
    if (!(ratio == ratio)) return fail(SFMX_EINVAL, "ratio is NaN");
    DeviceGuard g(m->device);
    // Run plan: per-pair dense offsets, the pair order by train image and the work
    // items.  Reused (no host work, no uploads) while the pair list, the images'
    // row counts / integrality and the kernel variant are those of the last run.
    const int variant_key = m->norm == SFMX_NORM_L2 ? sift_variant() : 0;
    std::vector<int64_t> img_key(2 * (size_t)m->n_imgs);
    for (int i = 0; i < m->n_imgs; ++i) { img_key[2 * i] = m->imgs[i].rows; img_key[2 * i + 1] = m->imgs[i].integral; }
    const int nb_want = match_batches();
    const bool reuse = m->plan_valid && m->plan_variant == variant_key && m->plan_imgs == img_key && m->plan_nb == nb_want &&
                       m->plan_pairs.size() == 2 * (size_t)n_pairs &&
                       (n_pairs == 0 || std::memcmp(m->plan_pairs.data(), pairs, sizeof(int32_t) * 2 * n_pairs) == 0);
    int rc;
    if (!reuse) {
        m->plan_valid = false;
        std::vector<PairDev> pd(n_pairs);
        int64_t dense = 0;
        for (int p = 0; p < n_pairs; ++p) {
            const int L = pairs[2 * p], R = pairs[2 * p + 1];
            if (L < 0 || L >= m->n_imgs || R < 0 || R >= m->n_imgs) return fail(SFMX_EINVAL, "pair image index out of range");
            pd[p] = PairDev{L, R, dense};
            dense += m->imgs[L].rows;
        }
        // Work items: 512-query blocks, sorted by train image so XCD-contiguous
        // blocks stream the same train rows (L2 reuse); fp32 pairs separately.
        std::vector<WorkItem> work, work32;
        std::vector<int> order(n_pairs);
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return pd[a].right < pd[b].right; });
        m->fp32_pairs = 0;
        int max_nt = 0;
        for (int p : order) {
            const ImgDev& L = m->imgs[pd[p].left];
            const ImgDev& R = m->imgs[pd[p].right];
            max_nt = std::max(max_nt, R.rows);
            const bool f32path = m->norm == SFMX_NORM_L2 && !(L.integral && R.integral);
            m->fp32_pairs += f32path;
            const int bq = f32path ? 512 : (m->norm == SFMX_NORM_L2 ? sift_block_queries(sift_variant()) : 512);
            for (int q0 = 0; q0 < L.rows; q0 += bq) (f32path ? work32 : work).push_back(WorkItem{p, q0});
        }
        if ((rc = m->pairs_d.ensure(sizeof(PairDev) * std::max(n_pairs, 1)))) return rc;
        if ((rc = m->work_d.ensure(sizeof(WorkItem) * std::max<size_t>(work.size(), 1)))) return rc;
        if ((rc = m->work32_d.ensure(sizeof(WorkItem) * std::max<size_t>(work32.size(), 1)))) return rc;
        if ((rc = m->dense_idx.ensure(sizeof(int32_t) * std::max<int64_t>(dense, 1)))) return rc;
        if ((rc = m->dense_dist.ensure(sizeof(float) * std::max<int64_t>(dense, 1)))) return rc;
        if ((rc = m->slow_list.ensure(sizeof(int2) * std::max<int64_t>(dense, 1)))) return rc;
        if ((rc = m->slow_count.ensure(sizeof(int32_t)))) return rc;
        if ((rc = m->qlist.ensure(sizeof(int32_t) * std::max<int64_t>(dense, 1)))) return rc;
        if (m->norm == SFMX_NORM_L2 || m->orb_fp4) {
            if ((rc = m->qmask.ensure(sizeof(int32_t) * std::max<int64_t>(dense, 1)))) return rc;
            if ((rc = m->top2.ensure(2 * sizeof(uint64_t) * std::max<int64_t>(dense, 1)))) return rc;
        }
        if ((rc = m->qcount.ensure(sizeof(int32_t) * (n_pairs + 8)))) return rc;   // + the persistent screens' XCD tickets
        if ((rc = m->porder.ensure(sizeof(int32_t) * std::max(n_pairs, 1)))) return rc;
        if ((rc = m->work2.ensure(sizeof(WorkItem) * std::max<size_t>(4 * work.size(), 1)))) return rc;   // pass-2 items >= 128 queries
        if ((rc = m->work2_n.ensure(sizeof(int32_t)))) return rc;
        if ((rc = m->unsettled.ensure(sizeof(int32_t)))) return rc;
        if ((rc = m->counts.ensure(sizeof(int64_t) * std::max(n_pairs, 1)))) return rc;
        if ((rc = m->keep.ensure(sizeof(int32_t) * std::max(n_pairs, 1)))) return rc;
        if ((rc = m->offsets.ensure(sizeof(int64_t) * (n_pairs + 1)))) return rc;
        if ((rc = m->out.ensure(sizeof(DMatchDev) * std::max<int64_t>(dense, 1)))) return rc;
        // uploads from pinned staging: [pairs | order | work | work32], 256-B aligned parts
        const size_t b_pd = align_up(sizeof(PairDev) * n_pairs, 256), b_or = align_up(sizeof(int32_t) * n_pairs, 256),
                     b_w = align_up(sizeof(WorkItem) * work.size(), 256), b_w32 = sizeof(WorkItem) * work32.size();
        if ((rc = m->stage_run.ensure(b_pd + b_or + b_w + b_w32))) return rc;
        char* hs = m->stage_run.as<char>();
        std::memcpy(hs, pd.data(), sizeof(PairDev) * n_pairs);
        std::memcpy(hs + b_pd, order.data(), sizeof(int32_t) * n_pairs);
        std::memcpy(hs + b_pd + b_or, work.data(), sizeof(WorkItem) * work.size());
        std::memcpy(hs + b_pd + b_or + b_w, work32.data(), b_w32);
        if (n_pairs) HIPCHK(hipMemcpyAsync(m->pairs_d.p, hs, sizeof(PairDev) * n_pairs, hipMemcpyHostToDevice, st));
        if (n_pairs) HIPCHK(hipMemcpyAsync(m->porder.p, hs + b_pd, sizeof(int32_t) * n_pairs, hipMemcpyHostToDevice, st));
        if (!work.empty()) HIPCHK(hipMemcpyAsync(m->work_d.p, hs + b_pd + b_or, sizeof(WorkItem) * work.size(), hipMemcpyHostToDevice, st));
        if (!work32.empty()) HIPCHK(hipMemcpyAsync(m->work32_d.p, hs + b_pd + b_or + b_w, b_w32, hipMemcpyHostToDevice, st));
        if ((rc = m->stage_run.copied(st))) return rc;
        {   // batches of the overlapped two-pass path: whole pairs in `order`, about n_work / nb items each
            m->batches.clear();
            const int64_t per = ((int64_t)work.size() + nb_want - 1) / std::max(nb_want, 1);
            MatchBatch cur{0, 0, 0, 0};
            size_t w = 0;
            for (int i = 0; i < n_pairs; ++i) {
                const int p = order[i];
                const bool f32path = m->norm == SFMX_NORM_L2 && !(m->imgs[pd[p].left].integral && m->imgs[pd[p].right].integral);
                int items = 0;
                while (!f32path && w + items < work.size() && work[w + items].pair == p) ++items;
                cur.nw += items;
                cur.np += 1;
                w += items;
                if (cur.nw >= per && i + 1 < n_pairs && w < work.size()) {   // (trailing no-work pairs join the last batch)
                    m->batches.push_back(cur);
                    cur = MatchBatch{(int32_t)w, 0, i + 1, 0};
                }
            }
            if (cur.np > 0) m->batches.push_back(cur);
            if (w != work.size()) return fail(SFMX_EINTERNAL, "match batches do not cover the work list");
        }
        m->plan_nb = nb_want;
        m->plan_pairs.assign(pairs, pairs + 2 * (size_t)n_pairs);
        m->plan_imgs = img_key;
        m->plan_variant = variant_key;
        m->plan_dense = dense;
        m->plan_nwork = work.size();
        m->plan_nwork32 = work32.size();
        m->plan_max_nt = max_nt;
        m->plan_valid = true;
    }
    const int64_t dense = m->plan_dense;
    const size_t n_work = m->plan_nwork, n_work32 = m->plan_nwork32;
    if (!m->evr[0][0])
        for (auto& set : m->evr)
            for (auto& e : set) HIPCHK(hipEventCreate(&e));
    m->ev = m->evr[m->runs % sfmx_matcher::EV_RING];
    ++m->runs;
    HIPCHK(hipMemsetAsync(m->slow_count.p, 0, sizeof(int32_t), st));
    HIPCHK(hipMemsetAsync(m->unsettled.p, 0, sizeof(int32_t), st));
    HIPCHK(hipEventRecord(m->ev[0], st));
    HIPCHK(hipEventRecord(m->ev[3], st));   // re-recorded after pass 1 by the two-pass launchers
    // Pairs with an empty left image have no work item; pairs with an empty
    // right image are handled in-kernel (every query: no neighbour).
    const PairDev* P = m->pairs_d.as<PairDev>();
    const ImgDev* I = m->imgs_d.as<ImgDev>();
    // overlapped two-pass product path (SIFT: the default screen + subset pass 2; ORB: FP4 screen + subset)
    const bool overlap = m->batches.size() >= 2 && n_work > 0 &&
                         ((m->norm == SFMX_NORM_L2 && sift_variant() == 0 && pass2_variant() == 10) ||
                          (m->norm != SFMX_NORM_L2 && m->orb_fp4 && orb_variant() == 0));
    OverlapStreams os{};
    if (overlap) {
        if (!m->sx) {
            HIPCHK(hipStreamCreateWithFlags(&m->sx, hipStreamNonBlocking));
            HIPCHK(hipStreamCreateWithFlags(&m->sp, hipStreamNonBlocking));
            for (auto& e : m->ov_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        while (m->bev.size() < m->batches.size()) {
            hipEvent_t e = nullptr;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            m->bev.push_back(e);
        }
        os = OverlapStreams{m->sx, m->sp, m->ov_ev[0], m->ov_ev[1], m->ov_ev[2], m->bev.data()};
    }
    if (overlap) {
        const bool sift = m->norm == SFMX_NORM_L2;
        HIPCHK(launch_two_pass_overlap(sift, m->batches.data(), (int)m->batches.size(), m->work_d.as<WorkItem>(), P, I,
                                       m->desc8.as<int8_t>(), sift ? m->normv.as<int32_t>() : nullptr,
                                       sift ? m->keyc2.as<int32_t>() : m->keyc.as<int32_t>(), m->qlist.as<int32_t>(),
                                       m->qcount.as<int32_t>(), n_pairs, m->porder.as<int32_t>(),
                                       m->dense_idx.as<int32_t>(), m->dense_dist.as<float>(), m->slow_list.as<int2>(),
                                       m->slow_count.as<int32_t>(), ratio, st, m->ev[3], m->qmask.as<int32_t>(),
                                       m->top2.as<unsigned long long>(), os));
        HIPCHK(hipEventRecord(m->ev[1], st));
        if (sift) {
            HIPCHK(launch_sift_slow(m->slow_list.as<int2>(), m->slow_count.as<int32_t>(), P, I, m->desc8.as<int8_t>(),
                                    m->normv.as<int32_t>(), m->dense_idx.as<int32_t>(), m->dense_dist.as<float>(), ratio, st));
            if (n_work32)
                HIPCHK(launch_sift_f32(m->work32_d.as<WorkItem>(), (int)n_work32, P, I, m->f32.as<float>(),
                                       m->dense_idx.as<int32_t>(), m->dense_dist.as<float>(), ratio, st));
        }
    } else if (m->norm == SFMX_NORM_L2) {
        HIPCHK(launch_sift_knn2(m->work_d.as<WorkItem>(), (int)n_work, P, I, m->desc8.as<int8_t>(),
                                m->normv.as<int32_t>(), m->keyc.as<int32_t>(), m->keyc2.as<int32_t>(),
                                m->qlist.as<int32_t>(), m->qcount.as<int32_t>(), n_pairs, m->porder.as<int32_t>(),
                                m->work2.as<WorkItem>(), m->work2_n.as<int32_t>(), m->dense_idx.as<int32_t>(),
                                m->dense_dist.as<float>(), m->slow_list.as<int2>(), m->slow_count.as<int32_t>(), ratio, st,
                                m->ev[3], m->qmask.as<int32_t>(), m->top2.as<unsigned long long>()));
        HIPCHK(hipEventRecord(m->ev[1], st));
        HIPCHK(launch_sift_slow(m->slow_list.as<int2>(), m->slow_count.as<int32_t>(), P, I, m->desc8.as<int8_t>(),
                                m->normv.as<int32_t>(), m->dense_idx.as<int32_t>(), m->dense_dist.as<float>(), ratio, st));
        if (n_work32)
            HIPCHK(launch_sift_f32(m->work32_d.as<WorkItem>(), (int)n_work32, P, I, m->f32.as<float>(),
                                   m->dense_idx.as<int32_t>(), m->dense_dist.as<float>(), ratio, st));
    } else if (m->orb_fp4) {
        HIPCHK(launch_orb_mfma(m->work_d.as<WorkItem>(), (int)n_work, P, I, m->desc8.as<uint8_t>(),
                               m->keyc.as<int32_t>(), m->qlist.as<int32_t>(), m->qcount.as<int32_t>(), n_pairs,
                               m->porder.as<int32_t>(), m->work2.as<WorkItem>(), m->work2_n.as<int32_t>(),
                               m->dense_idx.as<int32_t>(), m->dense_dist.as<float>(), ratio, st, m->ev[3],
                               m->qmask.as<int32_t>(), m->top2.as<unsigned long long>()));
        HIPCHK(hipEventRecord(m->ev[1], st));
    } else {
        HIPCHK(launch_orb_knn2(m->work_d.as<WorkItem>(), (int)n_work, P, I, m->desc8.as<uint8_t>(),
                               m->dense_idx.as<int32_t>(), m->dense_dist.as<float>(), ratio, st));
        HIPCHK(hipEventRecord(m->ev[1], st));
    }
    const int max_nt = m->plan_max_nt;
    HIPCHK(launch_assemble(P, n_pairs, I, m->dense_idx.as<int32_t>(), m->dense_dist.as<float>(), distinct ? 1 : 0,
                           min_count, max_nt, m->counts.as<int64_t>(), m->keep.as<int32_t>(),
                           m->offsets.as<int64_t>(), m->out.as<DMatchDev>(), m->unsettled.as<int32_t>(), st));
    HIPCHK(hipEventRecord(m->ev[2], st));
    m->ev_recorded = true;
    m->n_pairs = n_pairs;
    m->dense_total = dense;
    m->has_run = true;
    m->run_stream = st;
    m->run_spec = m->flags_pending;
    if (m->run_spec) {   // what a re-run on the exact paths needs (resolve_flags)
        m->last_pairs.assign(pairs, pairs + 2 * (size_t)n_pairs);
        m->last_ratio = ratio;
        m->last_distinct = distinct;
        m->last_min_count = min_count;
    }
    return SFMX_OK;
}

// The integrality check of set_images_device, deferred to the first read of results (flags_pending):
// wait for the published flags (long since written); if an image is not integral, give every image
// its fp32 rows, mark the images, and re-run the last run, whose int8 results assumed integrality.
// Ordering: the fp32 prep and the re-run go on the last run's stream, after an event of
// the set stream (the images' prep), so they can neither overlap the original run nor the set; the
// reader's stream then waits on the re-run's end (fetch / stats), or the host does (device_results,
// whose pointers may be used on any stream).  The caller's device descriptors are re-read here:
// sfmx.h requires them to stay valid and unchanged until the run's results are read.
int resolve_flags(sfmx_matcher* m, hipStream_t reader, bool host_wait) {
    if (!m->flags_pending) return SFMX_OK;
    const hipStream_t st = m->flags_stream;
    const int n = m->n_imgs;
    unsigned* hseq = reinterpret_cast<unsigned*>(m->hflags + m->hflags_cap);
    for (unsigned spins = 1;; ++spins) {
        if (__atomic_load_n(hseq, __ATOMIC_ACQUIRE) == m->flags_want) break;
        if ((spins & 255) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e != hipSuccess && e != hipErrorNotReady) return fail(SFMX_EDEVICE, std::string("integrality flags: ") + hipGetErrorString(e));
            if (e == hipSuccess && __atomic_load_n(hseq, __ATOMIC_ACQUIRE) != m->flags_want)
                return fail(SFMX_EINTERNAL, "integrality flags: stream drained without the flag handoff");
        }
        __builtin_ia32_pause();
    }
    m->flags_pending = false;
    const int32_t* fl = m->hflags;
    bool any = false;
    for (int i = 0; i < n; ++i) any |= fl[i] != 0;
    if (!any) { m->run_spec = false; return SFMX_OK; }   // the assumption held
    m->any_nonintegral = true;
    for (int i = 0; i < n; ++i) m->imgs[i].integral = fl[i] ? 0 : 1;
    if (!m->fix_ev[0])
        for (auto& e : m->fix_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const hipStream_t rs = m->has_run ? m->run_stream : st;
    if (rs != st) {
        HIPCHK(hipEventRecord(m->fix_ev[0], st));
        HIPCHK(hipStreamWaitEvent(rs, m->fix_ev[0], 0));
    }
    int rc;
    if ((rc = m->f32.ensure((size_t)m->total_rows * SIFT_DIM * 4))) return rc;
    for (int i = 0; i < n; ++i) {
        const ImgDev& d = m->imgs[i];
        HIPCHK(launch_prep_f32((const float*)m->last_src[i], d.rows, m->last_cols[i], d.rows_pad,
                               m->f32.as<float>() + d.row0 * SIFT_DIM, rs));
    }
    if ((rc = m->stage_imgs.ensure(sizeof(ImgDev) * n))) return rc;
    std::memcpy(m->stage_imgs.p, m->imgs.data(), sizeof(ImgDev) * n);
    HIPCHK(hipMemcpyAsync(m->imgs_d.p, m->stage_imgs.p, sizeof(ImgDev) * n, hipMemcpyHostToDevice, rs));
    if ((rc = m->stage_imgs.copied(rs))) return rc;
    m->plan_valid = false;
    if (m->run_spec) {
        m->run_spec = false;
        const std::vector<int32_t> pairs = m->last_pairs;
        if ((rc = run_impl(m, pairs.data(), (int)(pairs.size() / 2), m->last_ratio, m->last_distinct,
                           m->last_min_count, rs))) return rc;
    }
    if (host_wait) HIPCHK(hipStreamSynchronize(rs));
    else if (reader != rs) {
        HIPCHK(hipEventRecord(m->fix_ev[1], rs));
        HIPCHK(hipStreamWaitEvent(reader, m->fix_ev[1], 0));
    }
    return SFMX_OK;
}

int fetch_impl(sfmx_matcher* m, sfmx_dmatch* out, int64_t cap, int64_t* required, int64_t* pair_offsets,
               int32_t* keep, hipStream_t st) {
    if (!m) return fail(SFMX_EINVAL, "null matcher");
    if (!m->has_run) return fail(SFMX_ESTATE, "fetch before run");
    DeviceGuard g(m->device);
    { const int rc_ = resolve_flags(m, st, false); if (rc_) return rc_; }
    std::vector<int64_t> off(m->n_pairs + 1);
    int32_t unsettled = 0;
    HIPCHK(hipMemcpyAsync(off.data(), m->offsets.p, sizeof(int64_t) * (m->n_pairs + 1), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&unsettled, m->unsettled.p, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (unsettled) return fail(SFMX_EINTERNAL, std::to_string(unsettled) + " forwarded queries were not settled by pass 2");
    const int64_t total = off[m->n_pairs];
    if (required) *required = total;
    if (pair_offsets) std::memcpy(pair_offsets, off.data(), sizeof(int64_t) * (m->n_pairs + 1));
    if (keep && m->n_pairs) HIPCHK(hipMemcpyAsync(keep, m->keep.p, sizeof(int32_t) * m->n_pairs, hipMemcpyDeviceToHost, st));
    if (out) {
        if (cap < total) { HIPCHK(hipStreamSynchronize(st)); return fail(SFMX_ECAPACITY, "output capacity too small"); }
        if (total) HIPCHK(hipMemcpyAsync(out, m->out.p, sizeof(sfmx_dmatch) * total, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    return SFMX_OK;
}

}  // namespace

static_assert(sizeof(sfmx_dmatch) == 16 && sizeof(DMatchDev) == 16, "DMatch layout");

extern "C" {

const char* sfmx_version(void) { return "sfmx 0.1 (gfx950)"; }
const char* sfmx_last_error(void) { return g_last_error.c_str(); }

int sfmx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return fail(SFMX_EDEVICE, "hipGetDeviceCount failed");
    int good = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) ++good;
    }
    return good;
}

int sfmx_selftest_sqrt(int32_t device, int64_t n, uint32_t* out_bits) {
    if (n < 0 || n > (int64_t)1 << 24 || (n > 0 && !out_bits)) return fail(SFMX_EINVAL, "n must be in [0, 2^24]");
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    DevBuf b;
    if ((rc = b.ensure(sizeof(uint32_t) * std::max<int64_t>(n, 1)))) return rc;
    hipError_t e = launch_selftest_sqrt(n, b.as<uint32_t>(), nullptr);
    if (e == hipSuccess) e = hipMemcpy(out_bits, b.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost);
    b.release();
    if (e != hipSuccess) return fail(SFMX_EDEVICE, hipGetErrorString(e));
    return SFMX_OK;
}

int sfmx_matcher_create(int32_t device, sfmx_matcher** out) {
    if (!out) return fail(SFMX_EINVAL, "null out");
    *out = nullptr;
    int rc = check_device(device);
    if (rc) return rc;
    auto* m = new (std::nothrow) sfmx_matcher();
    if (!m) return fail(SFMX_ENOMEM, "host allocation");
    m->device = device;
    *out = m;
    return SFMX_OK;
}

int sfmx_matcher_destroy(sfmx_matcher* m) {
    if (!m) return SFMX_OK;
    {
        DeviceGuard g(m->device);
        m->stage_prep.release();
        m->stage_run.release();
        m->stage_imgs.release();
        m->stage_flags.release();
        if (m->hflags) (void)hipHostFree(m->hflags);
        m->hflags = nullptr;
        DevBuf* bufs[] = {&m->raw, &m->desc8, &m->normv, &m->keyc, &m->keyc2, &m->qlist, &m->qcount, &m->porder, &m->work2, &m->work2_n, &m->f32, &m->flags, &m->imgs_d, &m->pairs_d, &m->prep_tab,
                          &m->work_d, &m->work32_d, &m->dense_idx, &m->dense_dist, &m->slow_list, &m->slow_count,
                          &m->unsettled, &m->counts, &m->keep, &m->offsets, &m->out};
        for (DevBuf* b : bufs) b->release();
        for (auto& set : m->evr)
            for (auto& e : set) if (e) (void)hipEventDestroy(e);
        for (auto& e : m->ov_ev) if (e) (void)hipEventDestroy(e);
        for (auto& e : m->fix_ev) if (e) (void)hipEventDestroy(e);
        for (auto& e : m->bev) if (e) (void)hipEventDestroy(e);
        if (m->sx) (void)hipStreamDestroy(m->sx);
        if (m->sp) (void)hipStreamDestroy(m->sp);
    }
    delete m;
    return SFMX_OK;
}

int sfmx_matcher_set_images(sfmx_matcher* m, const sfmx_desc* imgs, int32_t n, int32_t norm, void* stream) {
    return set_images_impl(m, imgs, n, norm, (hipStream_t)stream, false);
}

int sfmx_matcher_set_images_device(sfmx_matcher* m, const sfmx_desc* imgs, int32_t n, int32_t norm, void* stream) {
    return set_images_impl(m, imgs, n, norm, (hipStream_t)stream, true);
}

int sfmx_matcher_run(sfmx_matcher* m, const int32_t* pairs, int32_t n_pairs, double ratio, int32_t distinct,
                     int32_t min_count, void* stream) {
    return run_impl(m, pairs, n_pairs, ratio, distinct, min_count, (hipStream_t)stream);
}

int sfmx_matcher_fetch(sfmx_matcher* m, sfmx_dmatch* out, int64_t cap, int64_t* required, int64_t* pair_offsets,
                       int32_t* keep, void* stream) {
    return fetch_impl(m, out, cap, required, pair_offsets, keep, (hipStream_t)stream);
}

int sfmx_matcher_device_results(sfmx_matcher* m, const sfmx_dmatch** matches, const int64_t** pair_offsets,
                                const int32_t** keep) {
    if (!m) return fail(SFMX_EINVAL, "null matcher");
    if (!m->has_run) return fail(SFMX_ESTATE, "no results before run");
    {
        DeviceGuard g(m->device);
        { const int rc_ = resolve_flags(m, nullptr, true); if (rc_) return rc_; }
    }
    if (matches) *matches = m->out.as<const sfmx_dmatch>();
    if (pair_offsets) *pair_offsets = m->offsets.as<const int64_t>();
    if (keep) *keep = m->keep.as<const int32_t>();
    return SFMX_OK;
}

int sfmx_matcher_stats(sfmx_matcher* m, int64_t* slow_queries, int64_t* fp32_pairs, void* stream) {
    if (!m) return fail(SFMX_EINVAL, "null matcher");
    if (!m->has_run) return fail(SFMX_ESTATE, "no stats before run");
    DeviceGuard g(m->device);
    { const int rc_ = resolve_flags(m, (hipStream_t)stream, false); if (rc_) return rc_; }
    int32_t sc = 0, unsettled = 0;
    HIPCHK(hipMemcpyAsync(&sc, m->slow_count.p, sizeof(int32_t), hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIPCHK(hipMemcpyAsync(&unsettled, m->unsettled.p, sizeof(int32_t), hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    if (unsettled) return fail(SFMX_EINTERNAL, std::to_string(unsettled) + " forwarded queries were not settled by pass 2");
    if (slow_queries) *slow_queries = sc;
    if (fp32_pairs) *fp32_pairs = m->fp32_pairs;
    return SFMX_OK;
}

int sfmx_matcher_timing(sfmx_matcher* m, float* main_kernel_ms, float* total_ms) {
    if (!m) return fail(SFMX_EINVAL, "null matcher");
    if (!m->ev_recorded) return fail(SFMX_ESTATE, "no timing before run");
    DeviceGuard g(m->device);
    HIPCHK(hipEventSynchronize(m->ev[2]));
    float a = 0.f, b = 0.f;
    HIPCHK(hipEventElapsedTime(&a, m->ev[0], m->ev[1]));
    HIPCHK(hipEventElapsedTime(&b, m->ev[0], m->ev[2]));
    if (main_kernel_ms) *main_kernel_ms = a;
    if (total_ms) *total_ms = b;
    return SFMX_OK;
}

int sfmx_matcher_timing_history(sfmx_matcher* m, float* main_kernel_ms, float* screen_ms, int32_t n) {
    if (!m) return fail(SFMX_EINVAL, "null matcher");
    if (!m->ev_recorded) return fail(SFMX_ESTATE, "no timing before run");
    if (n < 0) return fail(SFMX_EINVAL, "negative count");
    DeviceGuard g(m->device);
    HIPCHK(hipEventSynchronize(m->ev[2]));
    const long long k = std::min<long long>({(long long)n, m->runs, (long long)sfmx_matcher::EV_RING});
    for (long long i = 0; i < k; ++i) {   // oldest first: runs (runs - k) .. (runs - 1)
        hipEvent_t* e = m->evr[(m->runs - k + i) % sfmx_matcher::EV_RING];
        float a = 0.f, b = 0.f;
        HIPCHK(hipEventElapsedTime(&a, e[0], e[1]));
        HIPCHK(hipEventElapsedTime(&b, e[0], e[3]));
        if (main_kernel_ms) main_kernel_ms[i] = a;
        if (screen_ms) screen_ms[i] = b;
    }
    return (int)k;
}

int sfmx_matcher_pass_timing(sfmx_matcher* m, float* screen_ms, float* pass2_ms) {
    if (!m) return fail(SFMX_EINVAL, "null matcher");
    if (!m->ev_recorded) return fail(SFMX_ESTATE, "no timing before run");
    DeviceGuard g(m->device);
    HIPCHK(hipEventSynchronize(m->ev[2]));
    float a = 0.f, b = 0.f;
    HIPCHK(hipEventElapsedTime(&a, m->ev[0], m->ev[3]));
    HIPCHK(hipEventElapsedTime(&b, m->ev[3], m->ev[1]));
    if (screen_ms) *screen_ms = a;
    if (pass2_ms) *pass2_ms = b;
    return SFMX_OK;
}

int sfmx_match_pairs(const sfmx_desc* imgs, int32_t n_imgs, const int32_t* pairs, int32_t n_pairs, int32_t norm,
                     double ratio, int32_t distinct, int32_t min_count, int32_t n_gpus, sfmx_dmatch* out,
                     int64_t cap, int64_t* required, int64_t* pair_offsets, int32_t* keep) {
    if (n_pairs < 0 || (n_pairs > 0 && !pairs)) return fail(SFMX_EINVAL, "bad pair list");
    int ndev = sfmx_device_count();
    if (ndev <= 0) return fail(SFMX_EDEVICE, "no gfx950 device");
    const int G = std::max(1, std::min<int>(n_gpus <= 0 ? ndev : n_gpus, ndev));
    // Split the pair list into G contiguous slices balanced by sum Nq*Nt.
    std::vector<double> cost(n_pairs);
    double tot = 0;
    for (int p = 0; p < n_pairs; ++p) {
        const int L = pairs[2 * p], R = pairs[2 * p + 1];
        if (L < 0 || L >= n_imgs || R < 0 || R >= n_imgs) return fail(SFMX_EINVAL, "pair image index out of range");
        cost[p] = (double)imgs[L].rows * imgs[R].rows + 1.0;
        tot += cost[p];
    }
    std::vector<int> cut(G + 1, n_pairs);
    cut[0] = 0;
    {
        double acc = 0; int g = 1;
        for (int p = 0; p < n_pairs && g < G; ++p) {
            acc += cost[p];
            if (acc >= tot * g / G) cut[g++] = p + 1;
        }
    }
    struct Slice { std::vector<sfmx_dmatch> m; std::vector<int64_t> off; std::vector<int32_t> keep; int rc = 0; std::string err; };
    std::vector<Slice> sl(G);
    auto work = [&](int g) {
        Slice& s = sl[g];
        const int np = cut[g + 1] - cut[g];
        sfmx_matcher* m = nullptr;
        if ((s.rc = sfmx_matcher_create(g, &m))) { s.err = g_last_error; return; }
        hipStream_t st = nullptr;
        {
            DeviceGuard dg(g);
            if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { s.rc = SFMX_EDEVICE; s.err = "stream"; sfmx_matcher_destroy(m); return; }
        }
        s.off.assign(np + 1, 0); s.keep.assign(np, 0);
        // upload only the images this GPU's slice references (remapped to a dense local table)
        std::vector<int32_t> local_of(n_imgs, -1), lpairs(2 * (size_t)np);
        std::vector<sfmx_desc> limgs;
        for (int q = 0; q < 2 * np; ++q) {
            const int im = pairs[2 * cut[g] + q];
            if (local_of[im] < 0) { local_of[im] = (int32_t)limgs.size(); limgs.push_back(imgs[im]); }
            lpairs[q] = local_of[im];
        }
        int64_t req = 0;
        if (!(s.rc = sfmx_matcher_set_images(m, limgs.data(), (int32_t)limgs.size(), norm, st)) &&
            !(s.rc = sfmx_matcher_run(m, lpairs.data(), np, ratio, distinct, min_count, st)) &&
            !(s.rc = sfmx_matcher_fetch(m, nullptr, 0, &req, s.off.data(), s.keep.data(), st))) {
            s.m.resize(req);
            s.rc = sfmx_matcher_fetch(m, s.m.data(), req, &req, nullptr, nullptr, st);
        }
        if (s.rc) s.err = g_last_error;
        { DeviceGuard dg(g); (void)hipStreamDestroy(st); }
        sfmx_matcher_destroy(m);
    };
    if (G == 1) work(0);
    else {
        std::vector<std::thread> th;
        for (int g = 0; g < G; ++g) th.emplace_back(work, g);
        for (auto& t : th) t.join();
    }
    int64_t total = 0;
    for (int g = 0; g < G; ++g) {
        if (sl[g].rc) return fail(sl[g].rc, sl[g].err);
        total += (int64_t)sl[g].m.size();
    }
    if (required) *required = total;
    if (out && cap < total) return fail(SFMX_ECAPACITY, "output capacity too small");
    int64_t base = 0;
    for (int g = 0; g < G; ++g) {
        const int np = cut[g + 1] - cut[g];
        for (int p = 0; p < np; ++p) {
            if (pair_offsets) pair_offsets[cut[g] + p] = base + sl[g].off[p];
            if (keep) keep[cut[g] + p] = sl[g].keep[p];
        }
        if (out && !sl[g].m.empty()) std::memcpy(out + base, sl[g].m.data(), sizeof(sfmx_dmatch) * sl[g].m.size());
        base += (int64_t)sl[g].m.size();
    }
    if (pair_offsets) pair_offsets[n_pairs] = base;
    return SFMX_OK;
}

}  // extern "C"
