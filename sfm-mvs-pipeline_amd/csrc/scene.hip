// SPDX-License-Identifier: MIT
// sfmx scene bookkeeping for gfx950.
//
//   sfmx_find_3d2d_matches            Scene::find3d2dMatches   (common/Scene.cpp:369-424)
//   sfmx_ba_observations_from_origins BundleAdjustment.cpp:50-91 problem assembly (host, O(n))
//
// The reference's 3D-2D search is a nested linear scan: for every point
// origin it walks the shot-match list (find_if) and then the pair's DMatch
// list comparing keypoint positions, O(P * origins * (pairs + matches)).  Here
// it is a hash join on the GPU:
//   1. (host, O(pairs)) for every other shot o, the first pair joining
//      {shot, o} in list order — the only pair find_if can return;
//   2. one open-addressing table per such pair, keyed by the exact float bits
//      of the keypoint position on o's side, value = the smallest match index
//      with that position (atomicMin: the first DMatch in list order, which is
//      what find_if returns);
//   3. one thread per origin record probes its pair's table with the origin's
//      cv::Point2d — equal to a float keypoint position iff both coordinates
//      are exactly representable as float and equal (NaN never matches; -0 and
//      +0 compare equal, so both are keyed as +0).
// Integer / byte work: HBM- and latency-bound, no MFMA.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/sfmx_scene.h"
#include "match_common.hpp"

namespace sfmx {
namespace scene {

constexpr unsigned long long EMPTY = ~0ull;

struct UsedPair {          // a pair that is the first one joining {shot, other}
    int32_t pair;
    int32_t other_is_left;  // 1: the other shot is the pair's left image (queryIdx side)
    int64_t table0;         // first slot of its table
    int32_t cap;            // table capacity (power of two)
    int32_t _pad;
};

__device__ __forceinline__ unsigned long long pos_key(float x, float y) {
    x = x == 0.f ? 0.f : x;   // -0 == +0 under cv::Point2d ==
    y = y == 0.f ? 0.f : y;
    return ((unsigned long long)__float_as_uint(x) << 32) | __float_as_uint(y);
}
__device__ __forceinline__ uint32_t mix(unsigned long long k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
    return (uint32_t)k;
}

// one thread per match of a used pair: table[pos] = min match index
__global__ __launch_bounds__(256)
void build_tables_kernel(const UsedPair* __restrict__ used, const int32_t* __restrict__ used_first_match,
                         int n_used, int64_t n_items, const int64_t* __restrict__ off,
                         const DMatchDev* __restrict__ matches, const float2* const* __restrict__ kp,
                         const int32_t* __restrict__ nkp, const int32_t* __restrict__ pairs,
                         unsigned long long* __restrict__ tkey, int32_t* __restrict__ tval) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_items) return;
    // locate the used pair (used_first_match is the exclusive scan of match counts)
    int lo = 0, hi = n_used - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (used_first_match[mid] <= g) lo = mid; else hi = mid - 1;
    }
    const UsedPair u = used[lo];
    const int i = (int)(g - used_first_match[lo]);
    const DMatchDev d = matches[off[u.pair] + i];
    const int oshot = u.other_is_left ? pairs[2 * u.pair] : pairs[2 * u.pair + 1];
    const int kidx = u.other_is_left ? d.queryIdx : d.trainIdx;
    if (kidx < 0 || kidx >= nkp[oshot]) return;
    const float2 q = kp[oshot][kidx];
    if (q.x != q.x || q.y != q.y) return;   // NaN never compares equal
    const unsigned long long key = pos_key(q.x, q.y);
    uint32_t h = mix(key) & (uint32_t)(u.cap - 1);
    for (int probe = 0; probe < u.cap; ++probe) {
        unsigned long long* slot = tkey + u.table0 + h;
        const unsigned long long prev = atomicCAS(slot, EMPTY, key);
        if (prev == EMPTY || prev == key) {
            atomicMin(tval + u.table0 + h, i);
            return;
        }
        h = (h + 1) & (uint32_t)(u.cap - 1);
    }
}

// one thread per origin record
__global__ __launch_bounds__(256)
void lookup_kernel(int64_t n_origins, const int32_t* __restrict__ origin_shot, const double* __restrict__ origin_xy,
                   int shot, int n_shots, const int32_t* __restrict__ used_of_shot, const UsedPair* __restrict__ used,
                   const unsigned long long* __restrict__ tkey, const int32_t* __restrict__ tval,
                   const int64_t* __restrict__ off, const DMatchDev* __restrict__ matches,
                   const float2* const* __restrict__ kp, const int32_t* __restrict__ nkp,
                   int32_t* __restrict__ out_kp, int32_t* __restrict__ out_pair, float* __restrict__ out_xy) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_origins) return;
    int res_kp = -1, res_pair = -1;
    float2 res_xy = make_float2(__builtin_nanf(""), __builtin_nanf(""));
    const int o = origin_shot[r];
    const int ui = (o >= 0 && o < n_shots && o != shot) ? used_of_shot[o] : -1;
    if (ui >= 0) {
        const double qx = origin_xy[2 * r], qy = origin_xy[2 * r + 1];
        const float fx = (float)qx, fy = (float)qy;
        if ((double)fx == qx && (double)fy == qy) {   // else no float keypoint position can equal it
            const UsedPair u = used[ui];
            const unsigned long long key = pos_key(fx, fy);
            uint32_t h = mix(key) & (uint32_t)(u.cap - 1);
            for (int probe = 0; probe < u.cap; ++probe) {
                const unsigned long long k = tkey[u.table0 + h];
                if (k == EMPTY) break;
                if (k == key) {
                    const int i = tval[u.table0 + h];
                    const DMatchDev d = matches[off[u.pair] + i];
                    const int sidx = u.other_is_left ? d.trainIdx : d.queryIdx;   // `shot`'s side
                    if (sidx >= 0 && sidx < nkp[shot]) {
                        res_kp = sidx;
                        res_pair = u.pair;
                        res_xy = kp[shot][sidx];
                    }
                    break;
                }
                h = (h + 1) & (uint32_t)(u.cap - 1);
            }
        }
    }
    out_kp[r] = res_kp;
    out_pair[r] = res_pair;
    if (out_xy) { out_xy[2 * r] = res_xy.x; out_xy[2 * r + 1] = res_xy.y; }
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

}  // namespace scene
}  // namespace sfmx

using namespace sfmx;
using namespace sfmx::scene;

#define SCHK(expr) do { if ((expr) != hipSuccess) { rc = SFMX_EDEVICE; set_last_error("HIP error in " #expr); goto done; } } while (0)

extern "C" {

float sfmx_find_3d2d_last_kernel_ms(void) { return g_last_ms; }

int sfmx_find_3d2d_matches(const sfmx_point2f* const* keypoints, const int32_t* n_keypoints, int32_t n_shots,
                           const int32_t* pairs, int32_t n_pairs, const sfmx_dmatch* matches,
                           const int64_t* pair_offsets, const int64_t* origin_offsets, int32_t n_points,
                           const int32_t* origin_shot, const double* origin_xy, int32_t shot,
                           int32_t inputs_on_device, int32_t device, void* stream, int32_t* out_keypoint,
                           int32_t* out_pair, float* out_xy) {
    if (n_shots < 0 || n_pairs < 0 || n_points < 0) { set_last_error("negative count"); return SFMX_EINVAL; }
    if (!keypoints || !n_keypoints || (n_pairs && (!pairs || !pair_offsets)) || !origin_offsets ||
        !out_keypoint || !out_pair) {
        set_last_error("null argument");
        return SFMX_EINVAL;
    }
    if (shot < 0 || shot >= n_shots) { set_last_error("shot index out of range"); return SFMX_EINVAL; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { set_last_error("no HIP device visible"); return SFMX_EDEVICE; }
    if (device < 0 || device >= ndev) { set_last_error("device index out of range"); return SFMX_EINVAL; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_last_error("sfmx kernels are built for gfx950 only");
        return SFMX_EDEVICE;
    }
    for (int p = 0; p < n_pairs; ++p)
        if (pairs[2 * p] < 0 || pairs[2 * p] >= n_shots || pairs[2 * p + 1] < 0 || pairs[2 * p + 1] >= n_shots) {
            set_last_error("pair shot index out of range");
            return SFMX_EINVAL;
        }
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    const hipStream_t st = (hipStream_t)stream;
    int rc = SFMX_OK;
    {
        Bufs b;
        std::vector<int64_t> hoff(n_pairs + 1, 0), hoo;
        int64_t n_origins = 0;
        // 1. first pair per other shot (Scene.cpp:389-394: find_if over the pair list)
        std::vector<int32_t> first(n_shots, -1);
        std::vector<UsedPair> used;
        std::vector<int32_t> used_of_shot(n_shots, -1), used_first;
        int64_t items = 0, slots = 0;
        if (inputs_on_device) {
            if (n_pairs) SCHK(hipMemcpyAsync(hoff.data(), pair_offsets, sizeof(int64_t) * (n_pairs + 1), hipMemcpyDeviceToHost, st));
            SCHK(hipMemcpyAsync(&n_origins, origin_offsets + n_points, sizeof(int64_t), hipMemcpyDeviceToHost, st));
            SCHK(hipStreamSynchronize(st));
        } else {
            if (n_pairs) std::memcpy(hoff.data(), pair_offsets, sizeof(int64_t) * (n_pairs + 1));
            n_origins = origin_offsets[n_points];
            if (n_origins && (!origin_shot || !origin_xy)) { set_last_error("null origin arrays"); rc = SFMX_EINVAL; goto done; }
        }
        for (int p = 0; p < n_pairs; ++p) {
            const int L = pairs[2 * p], R = pairs[2 * p + 1];
            if (L == R) continue;
            const int o = L == shot ? R : (R == shot ? L : -1);
            if (o >= 0 && first[o] < 0) first[o] = p;
        }
        for (int o = 0; o < n_shots; ++o) {
            const int p = first[o];
            if (p < 0) continue;
            const int64_t m = hoff[p + 1] - hoff[p];
            if (m <= 0) continue;
            int cap = 16;
            while (cap < 2 * m) cap <<= 1;
            used_of_shot[o] = (int32_t)used.size();
            used.push_back(UsedPair{p, pairs[2 * p] == o ? 1 : 0, slots, cap, 0});
            used_first.push_back((int32_t)items);
            items += m;
            slots += cap;
        }
        if (items >= INT32_MAX) { set_last_error("too many matches"); rc = SFMX_EINVAL; goto done; }
        if (!inputs_on_device) {   // host validation of keypoint indices of the used pairs
            for (const UsedPair& u : used)
                for (int64_t i = hoff[u.pair]; i < hoff[u.pair + 1]; ++i) {
                    const int L = pairs[2 * u.pair], R = pairs[2 * u.pair + 1];
                    if (matches[i].queryIdx < 0 || matches[i].queryIdx >= n_keypoints[L] || matches[i].trainIdx < 0 ||
                        matches[i].trainIdx >= n_keypoints[R]) {
                        set_last_error("match index outside its image's keypoints");
                        rc = SFMX_EINVAL;
                        goto done;
                    }
                }
        }
        {
            // device copies of the inputs
            std::vector<const float2*> kptr(std::max(n_shots, 1));
            const DMatchDev* dm = reinterpret_cast<const DMatchDev*>(matches);
            const int64_t* doff = pair_offsets;
            const int32_t* dshot = origin_shot;
            const double* dxy = origin_xy;
            int32_t *dokp = out_keypoint, *dopair = out_pair;
            float* doxy = out_xy;
            if (inputs_on_device) {
                for (int i = 0; i < n_shots; ++i) kptr[i] = reinterpret_cast<const float2*>(keypoints[i]);
            } else {
                int64_t nk = 0;
                for (int i = 0; i < n_shots; ++i) nk += n_keypoints[i];
                auto* kd = static_cast<float2*>(b.alloc(sizeof(float2) * nk));
                auto* md = static_cast<DMatchDev*>(b.alloc(sizeof(DMatchDev) * std::max<int64_t>(hoff[n_pairs], 1)));
                auto* od = static_cast<int64_t*>(b.alloc(sizeof(int64_t) * (n_pairs + 1)));
                auto* sd = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * std::max<int64_t>(n_origins, 1)));
                auto* xd = static_cast<double*>(b.alloc(sizeof(double) * 2 * std::max<int64_t>(n_origins, 1)));
                dokp = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * std::max<int64_t>(n_origins, 1)));
                dopair = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * std::max<int64_t>(n_origins, 1)));
                doxy = out_xy ? static_cast<float*>(b.alloc(sizeof(float) * 2 * std::max<int64_t>(n_origins, 1))) : nullptr;
                if (!kd || !md || !od || !sd || !xd || !dokp || !dopair || (out_xy && !doxy)) { rc = SFMX_ENOMEM; goto done; }
                int64_t o = 0;
                for (int i = 0; i < n_shots; ++i) {
                    if (n_keypoints[i]) SCHK(hipMemcpyAsync(kd + o, keypoints[i], sizeof(float2) * n_keypoints[i], hipMemcpyHostToDevice, st));
                    kptr[i] = kd + o;
                    o += n_keypoints[i];
                }
                if (hoff[n_pairs]) SCHK(hipMemcpyAsync(md, matches, sizeof(DMatchDev) * hoff[n_pairs], hipMemcpyHostToDevice, st));
                SCHK(hipMemcpyAsync(od, pair_offsets, sizeof(int64_t) * (n_pairs + 1), hipMemcpyHostToDevice, st));
                if (n_origins) {
                    SCHK(hipMemcpyAsync(sd, origin_shot, sizeof(int32_t) * n_origins, hipMemcpyHostToDevice, st));
                    SCHK(hipMemcpyAsync(xd, origin_xy, sizeof(double) * 2 * n_origins, hipMemcpyHostToDevice, st));
                }
                dm = md; doff = od; dshot = sd; dxy = xd;
            }
            auto* kpd = static_cast<const float2**>(b.alloc(sizeof(float2*) * kptr.size()));
            auto* nkd = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * std::max(n_shots, 1)));
            auto* prd = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * 2 * std::max(n_pairs, 1)));
            auto* usd = static_cast<UsedPair*>(b.alloc(sizeof(UsedPair) * std::max<size_t>(used.size(), 1)));
            auto* ufd = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * std::max<size_t>(used_first.size(), 1)));
            auto* uos = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * std::max(n_shots, 1)));
            auto* tk = static_cast<unsigned long long*>(b.alloc(sizeof(unsigned long long) * std::max<int64_t>(slots, 1)));
            auto* tv = static_cast<int32_t*>(b.alloc(sizeof(int32_t) * std::max<int64_t>(slots, 1)));
            if (!kpd || !nkd || !prd || !usd || !ufd || !uos || !tk || !tv) { rc = SFMX_ENOMEM; goto done; }
            SCHK(hipMemcpyAsync(kpd, kptr.data(), sizeof(float2*) * kptr.size(), hipMemcpyHostToDevice, st));
            SCHK(hipMemcpyAsync(nkd, n_keypoints, sizeof(int32_t) * n_shots, hipMemcpyHostToDevice, st));
            if (n_pairs) SCHK(hipMemcpyAsync(prd, pairs, sizeof(int32_t) * 2 * n_pairs, hipMemcpyHostToDevice, st));
            if (!used.empty()) {
                SCHK(hipMemcpyAsync(usd, used.data(), sizeof(UsedPair) * used.size(), hipMemcpyHostToDevice, st));
                SCHK(hipMemcpyAsync(ufd, used_first.data(), sizeof(int32_t) * used_first.size(), hipMemcpyHostToDevice, st));
            }
            SCHK(hipMemcpyAsync(uos, used_of_shot.data(), sizeof(int32_t) * n_shots, hipMemcpyHostToDevice, st));
            hipEvent_t e0 = nullptr, e1 = nullptr;
            SCHK(hipEventCreate(&e0));
            SCHK(hipEventCreate(&e1));
            SCHK(hipEventRecord(e0, st));
            if (slots) {
                SCHK(hipMemsetAsync(tk, 0xff, sizeof(unsigned long long) * slots, st));
                SCHK(hipMemsetAsync(tv, 0x7f, sizeof(int32_t) * slots, st));
            }
            if (items)
                build_tables_kernel<<<(unsigned)((items + 255) / 256), 256, 0, st>>>(usd, ufd, (int)used.size(), items, doff, dm,
                                                                                    kpd, nkd, prd, tk, tv);
            if (n_origins)
                lookup_kernel<<<(unsigned)((n_origins + 255) / 256), 256, 0, st>>>(n_origins, dshot, dxy, shot, n_shots, uos, usd,
                                                                                 tk, tv, doff, dm, kpd, nkd, dokp, dopair, doxy);
            SCHK(hipGetLastError());
            SCHK(hipEventRecord(e1, st));
            if (!inputs_on_device && n_origins) {
                SCHK(hipMemcpyAsync(out_keypoint, dokp, sizeof(int32_t) * n_origins, hipMemcpyDeviceToHost, st));
                SCHK(hipMemcpyAsync(out_pair, dopair, sizeof(int32_t) * n_origins, hipMemcpyDeviceToHost, st));
                if (out_xy) SCHK(hipMemcpyAsync(out_xy, doxy, sizeof(float) * 2 * n_origins, hipMemcpyDeviceToHost, st));
            }
            SCHK(hipStreamSynchronize(st));
            float ms = -1.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            g_last_ms = ms;
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
    done:;
    }
    if (rc == SFMX_ENOMEM) set_last_error("device allocation failed");
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
}

int sfmx_ba_observations_from_origins(const int64_t* origin_offsets, int32_t n_points, const int32_t* origin_shot,
                                      const double* origin_xy, int32_t n_shots, int32_t* obs_point, int32_t* obs_cam,
                                      double* obs_xy, int32_t* pose_of_shot, int32_t* shot_of_pose, int32_t* n_poses) {
    if (n_points < 0 || n_shots < 0 || !origin_offsets || !pose_of_shot || !shot_of_pose || !n_poses) {
        set_last_error("bad argument");
        return SFMX_EINVAL;
    }
    const int64_t n = origin_offsets[n_points];
    if (n && (!origin_shot || !origin_xy || !obs_point || !obs_cam || !obs_xy)) { set_last_error("null array"); return SFMX_EINVAL; }
    for (int s = 0; s < n_shots; ++s) pose_of_shot[s] = -1;
    int32_t np = 0;
    for (int p = 0; p < n_points; ++p) {
        if (origin_offsets[p + 1] < origin_offsets[p]) { set_last_error("origin offsets not ascending"); return SFMX_EINVAL; }
        for (int64_t r = origin_offsets[p]; r < origin_offsets[p + 1]; ++r) {
            const int s = origin_shot[r];
            if (s < 0 || s >= n_shots) { set_last_error("origin shot out of range"); return SFMX_EINVAL; }
            if (pose_of_shot[s] < 0) { pose_of_shot[s] = np; shot_of_pose[np] = s; ++np; }   // BundleAdjustment.cpp:64-79
            obs_point[r] = p;
            obs_cam[r] = pose_of_shot[s];
            obs_xy[2 * r] = (double)(float)origin_xy[2 * r];           // cv::Point2d -> cv::Point2f (ICamera.h:161)
            obs_xy[2 * r + 1] = (double)(float)origin_xy[2 * r + 1];
        }
    }
    *n_poses = np;
    return SFMX_OK;
}

}  // extern "C"
