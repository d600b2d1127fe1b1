// SPDX-License-Identifier: MIT
// sfmx ORB extraction on gfx950: the
// reference's cv::ORB::create(featureLimit) (cli/PhotogrammetrieCli.cpp:347-348)
// as SfM::extractFeatures runs it, detect() then compute() (sfm/SfM.cpp:586-587),
// i.e. OpenCV 4.5.1's ORB_Impl::detectAndCompute twice.  Bit-identical to the
// restatement in oracle/orb_oracle.cpp (which lists the OpenCV pieces restated).
//
// Device pipeline per chunk of same-size images (one HIP stream; every level of the pyramid lives in
// one packed u8 slab in HBM, level l at lv[l].off, rows lv[l].pitch = width rounded up to 64 bytes):
//   orb_copy_kernel       level 0 from the caller's image (4 pixels per thread)
//   orb_resize_kernel     level l = INTER_LINEAR_EXACT resize of level l-1 (8.8 fixed
//                         point; per-axis offset/coefficient tables from the host; 4 pixels per thread)
//   orb_fast_nms_kernel   FAST 9/16 scores + the 3x3 strict maximum + the border test on 64 x 32
//                         tiles (16-byte tile loads, scores in LDS): keep words and their counts;
//                         with descriptors, compute()'s 7x7 integer Gaussian of the same tile from
//                         its LDS image tile (r05)
//   orb_scan_kernel       the rows' corner counts scanned
//   orb_rows_kernel       ordered (raster) compaction, one wave per row, from the keep words
//   orb_retain_kernel     retainBest(2 n_l) per level on the FAST scores: the permutation of
//                         the reference's libstdc++ nth_element + partition, in parallel
//   orb_harris_kernel     Harris response (7x7 block, k = 0.04) per kept corner
//   orb_retain_kernel     retainBest(n_l) per level on the Harris responses
//   orb_keep_kernel       compute()'s runByImageBorder(31) test at full resolution, the kept
//                         keypoints' places in order (one workgroup per level)
//   orb_angle_kernel      intensity-centroid angle of the kept keypoints, one wavefront per
//                         keypoint, written in place
//   (orb_blur_kernel      the blur as a pass of its own: diagnostic A/B only)
//   orb_brief_kernel      rBRIEF, 32 lanes per keypoint, one descriptor byte per lane
// One host wait per chunk (the keypoint counts at the end).  Roofline: HBM-bound byte work (see
// DESIGN.md §3).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sfmx.h"
#include "../../include/sfmx_features.h"
#include "diag.hpp"
#include "xcd.hpp"
#include "match_common.hpp"

namespace sfmx {
namespace orb {

constexpr int PATCH = 31, HALF_PATCH = 15, HARRIS_BLOCK = 7, MAX_LEVELS = 16;
constexpr float HARRIS_K = 0.04f;

struct Lvl {              // one pyramid level in the packed slabs
    int64_t off;          // byte offset of (0, 0) in pyr / score / blur slabs
    int w, h;
    int pitch;            // bytes per row: w rounded up to 64 (r04: 16-byte tile loads, 4-byte stores)
    int row0;             // first global row index of this level (NMS rows)
    float scale, inv_scale;
    int ax_off, ay_off;   // offsets of this level's axis tables in the coefficient buffer (level >= 1)
    int xdmin, xdmax, ydmin, ydmax;
};

struct Kp { float x, y, size, angle, response; int32_t octave, class_id; };
static_assert(sizeof(Kp) == sizeof(sfmx_keypoint), "cv::KeyPoint layout");

struct AxisEnt { int32_t ofs; uint16_t m0, m1; };

// Batched launches (r04): a chunk of G same-size images runs as ONE set of launches, image g's
// per-image arrays at byte offset g * istride from image 0's (one scratch block per image, the
// layout of the one-image arena), its counters at stats + g * CS.  r03 issued ~22 launches, 3
// pageable uploads and one host wait per image from 8 host threads: the leg was host-bound.
struct ImgIO {             // per image of a chunk
    const uint8_t* img;    // the 8-bit input (device), pitch bytes per row
    int64_t pitch;
    Kp* kp_out;            // device keypoints (inputs_on_device) or nullptr
    uint8_t* desc_out;     // descriptor rows (the caller's device buffer or the image's staging)
    int32_t capacity, pad;
};
// stats ints per image: cnt1[16] | cnt2[16] | kcnt[16] (kept by compute()'s border test) | count, levels, corners, err
constexpr int ST_CNT2 = MAX_LEVELS, ST_KCNT = 2 * MAX_LEVELS, ST_TAIL = 3 * MAX_LEVELS, CS = ST_TAIL + 4;
template <class T>
__device__ __forceinline__ T* at(T* p, int64_t bo) { return reinterpret_cast<T*>(reinterpret_cast<char*>(p) + bo); }
template <class T>
__device__ __forceinline__ const T* at(const T* p, int64_t bo) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(p) + bo);
}

__constant__ int c_pattern[256 * 4] = {
#include "orb_pattern.inc"
};

__device__ __forceinline__ int round_f(float v) { return __float2int_rn(v); }   // cvRound(float)

// [t0, t1) of n items for this workgroup: contiguous ranges, the workgroups that share an XCD (blocks
// b, b + 8, ... under round-robin dispatch) given adjacent ranges (speed only, never correctness)
__device__ __forceinline__ void xcd_range(int n, int& t0, int& t1) {
    const int nwg = gridDim.x, b = blockIdx.x, q = nwg >> 3, r = nwg & 7, x = b & 7;
    const int rb = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
    const int per = (n + nwg - 1) / nwg;
    t0 = min(n, rb * per);
    t1 = min(n, t0 + per);
}

// ------------------------------------------------------------------ pyramid
// resize(prev, level, INTER_LINEAR_EXACT): horizontal 8.8 taps, then vertical taps,
// (sum + 2^15) >> 16; rows/columns outside [dmin, dmax) replicate the edge source
// row/column ((v + 2^7) >> 8 for the replicated rows).
__device__ __forceinline__ uint32_t hval(const uint8_t* __restrict__ r, const AxisEnt* __restrict__ ax, int x,
                                         int dmin, int dmax, int last_ofs) {
    if (x < dmin) return (uint32_t)r[0] << 8;
    if (x >= dmax) return (uint32_t)r[last_ofs] << 8;
    const AxisEnt e = ax[x];
    return min((uint32_t)e.m0 * r[e.ofs] + (uint32_t)e.m1 * r[e.ofs + 1], 0xFFFFu);
}

// r04: one workgroup per 128 x 32 output tile, 8 neighbouring outputs x 2 rows per thread, 8-byte stores (the
// level pitch is a multiple of 64).  A tile whose outputs all take the interpolating branch on both
// axes (and whose source span fits, i.e. scale factors up to ~2) stages its source rectangle in LDS by
// 16-byte loads and reads the taps' bytes from there; the tiles at the edges (replicated rows /
// columns, the padding past the width) keep the per-pixel form.  The same integer expressions either
// way.  r03 made 4 byte loads and a table load per output pixel, the level chain measured load-bound.
constexpr int RZ_PX = 8, RZ_RT = 2, RZ_X = 16 * RZ_PX, RZ_Y = 16 * RZ_RT;   // 8 columns x 2 rows per thread
constexpr int RZ_R = 2 * RZ_Y + 8, RZ_C = 2 * RZ_X + 16;                     // the largest staged source span
// the source offset linear_axis gives destination v (the same double expression, so the same value;
// the staged rectangle keeps a one-pixel margin either way)
__device__ __forceinline__ int src_ofs(double scale, int v) { return (int)floor(scale * ((double)v + 0.5) - 0.5); }
// D / S (this level and the one it is resized from) come as kernel arguments and the staged source
// rectangle from the axis scales, so the tile's loads do not wait on the level table or the axis tables
__global__ __launch_bounds__(256)
void orb_resize_kernel(uint8_t* __restrict__ pyr, const Lvl D, const Lvl S, double sx, double sy,
                       const AxisEnt* __restrict__ tables, int64_t istride, int xcd) {
    __shared__ __align__(16) uint8_t T[RZ_R][RZ_C];
    int tx, ty, tz;
    xcd_grid(xcd, tx, ty, tz);
    pyr = at(pyr, (int64_t)tz * istride);
    const int x0 = tx * RZ_X, y0 = ty * RZ_Y;
    const int x = x0 + RZ_PX * (threadIdx.x & 15), yb = y0 + (threadIdx.x >> 4);   // rows yb + 16 r
    const AxisEnt* ax = tables + D.ax_off;
    const AxisEnt* ay = tables + D.ay_off;
    const uint8_t* src = pyr + S.off;
    bool staged = x0 >= D.xdmin && x0 + RZ_X <= D.xdmax && y0 >= D.ydmin && y0 + RZ_Y <= D.ydmax;
    int bx = 0, sy0 = 0;
    AxisEnt hx[RZ_PX], ey[RZ_RT];   // this thread's table entries, loaded beside the tile
    if (staged) {
#pragma unroll
        for (int i = 0; i < RZ_PX; ++i) hx[i] = ax[x + i];
#pragma unroll
        for (int r = 0; r < RZ_RT; ++r) ey[r] = ay[yb + 16 * r];
        bx = max(0, src_ofs(sx, x0) - 1) & ~15;
        sy0 = max(0, src_ofs(sy, y0) - 1);
        const int ncols = min(S.w - 1, src_ofs(sx, x0 + RZ_X - 1) + 2) + 1 - bx;
        const int nrows = min(S.h - 1, src_ofs(sy, y0 + RZ_Y - 1) + 2) + 1 - sy0;
        staged = ncols <= RZ_C && nrows <= RZ_R;   // (block-uniform)
        if (staged) {
            const int nq = (ncols + 15) >> 4;   // (the last word ends inside the padded row)
            for (int e = threadIdx.x; e < nrows * nq; e += 256) {
                const int rr = e / nq, q = e - rr * nq;
                *reinterpret_cast<uint4*>(&T[rr][16 * q]) =
                    *reinterpret_cast<const uint4*>(src + (int64_t)(sy0 + rr) * S.pitch + bx + 16 * q);
            }
        }
        __syncthreads();
    }
    if (x >= D.w) return;
#pragma unroll
    for (int r = 0; r < RZ_RT; ++r) {
        const int y = yb + 16 * r;
        if (y >= D.h) break;
        uint32_t out[RZ_PX / 4] = {};
        if (staged) {
            const AxisEnt e = ey[r];
            const uint8_t* t0 = T[e.ofs - sy0];
            const uint8_t* t1 = T[e.ofs + 1 - sy0];
#pragma unroll
            for (int i = 0; i < RZ_PX; ++i) {
                const AxisEnt h = hx[i];
                const int o = h.ofs - bx;
                const uint32_t h0 = min((uint32_t)h.m0 * t0[o] + (uint32_t)h.m1 * t0[o + 1], 0xFFFFu);
                const uint32_t h1 = min((uint32_t)h.m0 * t1[o] + (uint32_t)h.m1 * t1[o + 1], 0xFFFFu);
                out[i >> 2] |= min((h0 * e.m0 + h1 * e.m1 + 32768u) >> 16, 255u) << (8 * (i & 3));
            }
        } else {
            const int last_ofs = ax[D.w - 1].ofs;
            if (y < D.ydmin || y >= D.ydmax) {
                const uint8_t* rw = src + (int64_t)(y < D.ydmin ? 0 : S.h - 1) * S.pitch;
#pragma unroll
                for (int i = 0; i < RZ_PX; ++i)
                    out[i >> 2] |= min((hval(rw, ax, x + i, D.xdmin, D.xdmax, last_ofs) + 128u) >> 8, 255u) << (8 * (i & 3));
            } else {
                const AxisEnt e = ay[y];
                const uint8_t* r0 = src + (int64_t)e.ofs * S.pitch;
                const uint8_t* r1 = r0 + S.pitch;
#pragma unroll
                for (int i = 0; i < RZ_PX; ++i) {
                    const uint32_t h0 = hval(r0, ax, x + i, D.xdmin, D.xdmax, last_ofs);
                    const uint32_t h1 = hval(r1, ax, x + i, D.xdmin, D.xdmax, last_ofs);
                    out[i >> 2] |= min((h0 * e.m0 + h1 * e.m1 + 32768u) >> 16, 255u) << (8 * (i & 3));
                }
            }
        }
        *reinterpret_cast<uint2*>(pyr + D.off + (int64_t)y * D.pitch + x) = make_uint2(out[0], out[1]);   // (x + 8 <= pitch)
    }
}

// level 0 from the caller's image: 16 pixels per thread (64 x 4 threads: 1024 columns of 4 rows), one
// 16-byte store into the padded row; 16-byte loads when the caller's rows are 16-byte aligned
__global__ __launch_bounds__(256)
void orb_copy_kernel(const ImgIO* __restrict__ io, int W, int H, int P0, uint8_t* __restrict__ dst, int64_t istride) {
    const int x = (blockIdx.x * 64 + (threadIdx.x & 63)) * 16, y = blockIdx.y * 4 + (threadIdx.x >> 6), g = blockIdx.z;
    if (x >= W || y >= H) return;
    const uint8_t* p = io[g].img + (int64_t)y * io[g].pitch + x;
    dst = at(dst, (int64_t)g * istride);
    uint4 v;
    if (((reinterpret_cast<uintptr_t>(io[g].img) | (uintptr_t)io[g].pitch) & 15) == 0 && x + 16 <= W) {
        v = *reinterpret_cast<const uint4*>(p);
    } else {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (x + i < W) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    *reinterpret_cast<uint4*>(dst + (int64_t)y * P0 + x) = v;   // (x + 16 <= P0: P0 is a multiple of 64)
}

// Flat tile grids (r04): blockIdx.x counts the tiles of level 0, then level 1, ... (tw x th pixels each);
// -> the level and the tile's pixel origin, or -1 past the last level.  A grid sized by the largest level
// for every level left ~2/3 of the workgroups with nothing to do.
template <int TW, int TH>
__device__ __forceinline__ int flat_tile(const Lvl* __restrict__ lv, int nl, int t, int& x0, int& y0) {
    for (int l = 0; l < nl; ++l) {
        const int w = lv[l].w, h = lv[l].h, ntx = (w + TW - 1) / TW, n = ntx * ((h + TH - 1) / TH);
        if (t < n) {
            y0 = (t / ntx) * TH;
            x0 = (t - (t / ntx) * ntx) * TW;
            return l;
        }
        t -= n;
    }
    return -1;
}
template <int TW, int TH>
int flat_tiles(const std::vector<Lvl>& lv) {
    int n = 0;
    for (const Lvl& L : lv) n += ((L.w + TW - 1) / TW) * ((L.h + TH - 1) / TH);
    return n;
}

// ------------------------------------------------------------------ compute()'s blur
// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on the 8U level through OpenCV's
// integer separable path: taps x 2^8, (sum + 2^15) >> 16, saturated.
constexpr int BT_X = 64, BT_Y = 32, BR = 3, BT_H = BT_Y + 2 * BR;
__constant__ int c_taps[7];

__device__ __forceinline__ int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

// The blurred 64 x 32 tile (x0, y0) of level L (src / dst: the level's (0, 0) in the pyramid / blur slabs).
// r04: 64 x 32 output tiles (halo rows 38 / 32 instead of 22 / 16); interior tiles load without the
// reflection; the row pass makes 4 neighbouring sums per thread from a 10-byte window, the column pass 8
// rows of one column from a 14-sum window (the same taps in the same order: the same integers).
// r05: ti (optional) is the FAST pass's LDS image tile (rows y0 - 4 .., columns x0 - 16 .., row stride
// TIC): an interior tile's rows come from there instead of a second read of the level.  r: BT_H x
// (BT_X + 1) ints of LDS.  Two halves, a workgroup barrier between them (the caller's: a barrier waits
// for the wave's outstanding global stores too, so the caller keeps its own stores after it).
template <int TIC>
__device__ __forceinline__ void blur_rows(const uint8_t* __restrict__ src, const Lvl& L, int x0, int y0,
                                          const uint8_t* ti, int (*r)[BT_X + 1]) {
    // Row pass (r04): each thread makes 4 neighbouring row sums from the 12 bytes x-4 .. x+7 of its
    // row, read as 3 aligned 4-byte words (interior tiles) or gathered with the reflection (border
    // tiles); per output the 7-byte window is two realigned words (v_alignbyte) dotted with the taps
    // (v_dot4_u32_u8, the 8th tap 0).  Integer sums: the same values as the tap-by-tap form.  The
    // byte tile in LDS it replaces cost bank conflicts and ~2x the VALU work (PMC r04h).
    const bool interior = x0 >= 64 && x0 + BT_X + 4 <= L.pitch && x0 + BT_X + BR <= L.w && y0 >= BR && y0 + BT_Y + BR <= L.h;
    const uint32_t T0 = (uint32_t)c_taps[0] | (uint32_t)c_taps[1] << 8 | (uint32_t)c_taps[2] << 16 | (uint32_t)c_taps[3] << 24;
    const uint32_t T1 = (uint32_t)c_taps[4] | (uint32_t)c_taps[5] << 8 | (uint32_t)c_taps[6] << 16;
    constexpr int ITEMS = BT_H * (BT_X / 4);
#pragma unroll
    for (int it = 0; it < (ITEMS + 255) / 256; ++it) {
        const int i = threadIdx.x + 256 * it;
        if (i < ITEMS) {
            const int ty = i / (BT_X / 4), tx = 4 * (i % (BT_X / 4));
            uint32_t wa, wb, wc;   // bytes x-4 .. x-1 | x .. x+3 | x+4 .. x+7 of the row, x = x0 + tx
            if (interior && ti) {   // (a branch of its own: the loads stay LDS loads, not flat ones)
                const uint32_t* q = reinterpret_cast<const uint32_t*>(ti + (ty + 4 - BR) * TIC + tx + 12);
                wa = q[0];
                wb = q[1];
                wc = q[2];
            } else if (interior) {
                const uint32_t* q = reinterpret_cast<const uint32_t*>(src + (int64_t)(y0 + ty - BR) * L.pitch + x0 + tx - 4);
                wa = q[0];
                wb = q[1];
                wc = q[2];
            } else {
                const uint8_t* row = src + (int64_t)reflect101(y0 + ty - BR, L.h) * L.pitch;
                uint32_t wv[3] = {0u, 0u, 0u};
#pragma unroll
                for (int k = 1; k <= 10; ++k)   // (bytes 0 and 11 are never used)
                    wv[k >> 2] |= (uint32_t)row[reflect101(x0 + tx - 4 + k, L.w)] << (8 * (k & 3));
                wa = wv[0];
                wb = wv[1];
                wc = wv[2];
            }
            // output q: bytes 1+q .. 7+q
            r[ty][tx + 0] = (int)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(wc, wb, 1), T1,
                                                        __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(wb, wa, 1), T0, 0u, false), false);
            r[ty][tx + 1] = (int)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(wc, wb, 2), T1,
                                                        __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(wb, wa, 2), T0, 0u, false), false);
            r[ty][tx + 2] = (int)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(wc, wb, 3), T1,
                                                        __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(wb, wa, 3), T0, 0u, false), false);
            r[ty][tx + 3] = (int)__builtin_amdgcn_udot4(wc, T1, __builtin_amdgcn_udot4(wb, T0, 0u, false), false);
        }
    }
}
__device__ __forceinline__ void blur_cols(const Lvl& L, int x0, int y0, const int (*r)[BT_X + 1], uint8_t* __restrict__ dst) {
    static_assert(BT_Y % 8 == 0 && (BT_X * BT_Y / 8) == 256, "one column strip of 8 rows per thread");
    const int tx = threadIdx.x % BT_X, ty0 = 8 * (threadIdx.x / BT_X);
    const int x = x0 + tx;
    if (x < L.w) {
        int w[14];
#pragma unroll
        for (int k = 0; k < 14; ++k) w[k] = r[ty0 + k][tx];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int y = y0 + ty0 + q;
            if (y >= L.h) break;
            int s = 0;
#pragma unroll
            for (int j = 0; j < 7; j++) s += c_taps[j] * w[q + j];
            dst[(int64_t)y * L.pitch + x] = (uint8_t)min(max((s + (1 << 15)) >> 16, 0), 255);
        }
    }
}

// the separate blur pass (diagnostic A/B of the fused one: SFMX_ORB_BLUR_SEPARATE) -- only the levels the
// kept keypoints use
__global__ __launch_bounds__(256)
void orb_blur_kernel(const uint8_t* __restrict__ pyr, const Lvl* __restrict__ lv, const int* __restrict__ st,
                     uint8_t* __restrict__ blur, int nl, int64_t istride, int xcd) {
    int bx, g, bz;   // grid (flat 64 x 32 tiles of all levels, images)
    xcd_grid(xcd, bx, g, bz);
    int x0, y0;
    const int l = flat_tile<BT_X, BT_Y>(lv, nl, bx, x0, y0);
    if (l < 0 || l >= st[(int64_t)g * CS + 1]) return;
    __shared__ int r[BT_H][BT_X + 1];
    const Lvl L = lv[l];
    blur_rows<0>(at(pyr, (int64_t)g * istride) + L.off, L, x0, y0, nullptr, r);
    __syncthreads();
    blur_cols(L, x0, y0, r, at(blur, (int64_t)g * istride) + L.off);
}

// ------------------------------------------------------------------ FAST 9/16 + NMS
// r04: FAST and the 3x3 strict-maximum test in one tile pass.  A workgroup owns 64 x 32 pixels of
// one level: the image tile (rows y0-4 .. y0+35, columns x0-16 .. x0+79) comes in as 16-byte
// loads, the FAST scores of the 66 x 34 ring around the tile go to LDS, and every wave tests its
// rows against LDS: one keep word per (row, 64-pixel word) from the ballot, its popcount, and the
// tile's scores (read back only at kept pixels).  r03 wrote the score map from one kernel and
// re-read every 3 x 3 neighbourhood from HBM in a second.
constexpr int FT_X = 64, FT_Y = 32;
constexpr int FI_R = FT_Y + 8, FI_C = 96;        // image tile
constexpr int FS_R = FT_Y + 2, FS_C = FT_X + 2;  // score tile

// cornerScore<16> of the pixel c points at, when it is a FAST 9/16 corner, else 0 (S: LDS row stride).
// With d_k = v - p_k on the ring, M = the largest minimum of d over the 16 arcs of 9 pixels and N = the
// smallest maximum: FAST_t<16> calls the pixel a corner iff some arc is all darker (min d > t) or all
// brighter (max d < -t), i.e. iff max(M, -N) > t; cornerScore<16> (its a0 / b0 loops over the arcs
// split as min(d[k+1..k+8]) with d[k] or d[k+9]) returns max(t, M, -N) - 1.  So the score is
// max(M, -N) - 1 for a corner, and both follow from sliding minima / maxima of width 3 and 9 (v_min3 /
// v_max3) without the dark / bright bit masks: r04, ~half the VALU work of the bit-mask test followed
// by cornerScore's loops (the tile pass measured VALU-bound: 372 M VALU instructions per 16 images).
template <int S>
__device__ __forceinline__ int fast_score_lds(const uint8_t* c, int threshold) {
    const int v = c[0];
    const int p[16] = {c[3 * S],  c[3 * S + 1],  c[2 * S + 2],  c[S + 3],  c[3],  c[-S + 3], c[-2 * S + 2], c[-3 * S + 1],
                       c[-3 * S], c[-3 * S - 1], c[-2 * S - 2], c[-S - 3], c[-3], c[S - 3],  c[2 * S - 2],  c[3 * S - 1]};
    int d[16], m3[16], x3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = v - p[k];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        m3[k] = min(min(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
        x3[k] = max(max(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
    }
    int M = INT_MIN, N = INT_MAX;
#pragma unroll
    for (int k = 0; k < 16; k++) {   // arc k .. k+8 = three runs of 3
        M = max(M, min(min(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]));
        N = min(N, max(max(x3[k], x3[(k + 3) & 15]), x3[(k + 6) & 15]));
    }
    const int e = max(M, -N);
    return e > threshold ? e - 1 : 0;
}

// grid (flat 64 x 32 tiles of all levels in runs of `strip`, images).  kmask / wcnt: (global row) x mw,
// the words [0, ceil(w / 64)) of every row of the level written (0 outside the border or without a
// corner); score: the FAST score of every kept pixel (other pixels are not written).  Scores are 0 in
// FAST's own 3-pixel frame; a corner needs b <= x < w - b, b <= y < h - b (b = max(border, 3)), a
// nonzero score and a score above all 8 neighbours'.
// r05: blur (optional: compute()'s blurred slab) -- the tile's 7x7 Gaussian from the same LDS image tile
// (blur_rows / blur_cols), so the blur no longer reads the level a second time or launches a pass of its
// own (r05s, 16-image chunks: FAST + NMS 259 us and blur 121 us -> 342 us together); only the kept
// pixels' scores are stored.  The grid is dealt to the XCDs in contiguous ranges (xcd = -1: whole
// images per XCD), so the lines a tile's halo shares with its neighbours come from the XCD's own L2:
// the pass's counter fetch 14.3 -> 3.2 MB per image for ~2 % of its time (r05m, r05r).  (Also measured:
// the kept scores packed per tile instead of the score map, 41 us per 16 images slower for 6 MB per
// image less written, r05s; 2 or 4 tiles per workgroup in turn, 94 VGPRs and 30 % slower, r05t.)
static_assert(BT_X == FT_X && BT_Y == FT_Y && BR < 4, "the blur tile is the FAST tile, its halo inside the image tile");
__global__ __launch_bounds__(256)
void orb_fast_nms_kernel(const uint8_t* __restrict__ pyr, const Lvl* __restrict__ lv, int threshold, int border,
                         uint8_t* __restrict__ score, uint64_t* __restrict__ kmask, uint8_t* __restrict__ wcnt, int mw,
                         int nl, int64_t istride, int xcd, uint8_t* __restrict__ blur) {
    // LDS: the image tile; the score tile + candidate list, later (aliased) the blur's row sums
    constexpr int TS_B = FS_R * (FS_C + 2), U_B = TS_B + FS_R * FS_C * 2, R_B = BT_H * (BT_X + 1) * 4;
    __shared__ __align__(16) uint8_t ti[FI_R][FI_C];
    __shared__ __align__(16) uint8_t u[U_B > R_B ? U_B : R_B];
    __shared__ int ncand;
    auto ts = reinterpret_cast<uint8_t (*)[FS_C + 2]>(u);
    auto cand = reinterpret_cast<uint16_t*>(u + TS_B);
    auto rs = reinterpret_cast<int (*)[BT_X + 1]>(u);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int bx, by, bz;
    xcd_grid(xcd, bx, by, bz);
    const int64_t bo = (int64_t)by * istride;   // y = image
    int x0, y0;
    const int lvl = flat_tile<FT_X, FT_Y>(lv, nl, bx, x0, y0);
    if (lvl < 0) return;
    const uint8_t* pyr_g = at(pyr, bo);
    uint8_t* score_g = at(score, bo);
    uint8_t* blur_g = blur ? at(blur, bo) : nullptr;
    kmask = at(kmask, bo);
    wcnt = at(wcnt, bo);
    {
        const Lvl L = lv[lvl];
        const int ny = min(FT_Y, L.h - y0), b = max(border, 3);
        const int64_t w0 = (int64_t)(L.row0 + y0) * mw + x0 / FT_X;
        uint64_t* km = kmask + w0;
        uint8_t* wc = wcnt + w0;
        const uint8_t* src = pyr_g + L.off;
        uint8_t* bl = blur_g ? blur_g + L.off : nullptr;
        if (!(x0 + FT_X > b && x0 < L.w - b && y0 + ny > b && y0 < L.h - b)) {   // no pixel of the tile may be a corner
            if (bl) {
                blur_rows<FI_C>(src, L, x0, y0, nullptr, rs);
                __syncthreads();
                blur_cols(L, x0, y0, rs, bl);
            }
            if ((int)threadIdx.x < ny) {
                km[(int64_t)threadIdx.x * mw] = 0;
                wc[(int64_t)threadIdx.x * mw] = 0;
            }
            return;
        }
        if (threadIdx.x == 0) ncand = 0;
        if (threadIdx.x < FI_R * (FI_C / 16)) {
            const int r = threadIdx.x / (FI_C / 16), q = threadIdx.x % (FI_C / 16);
            const int gy = min(max(y0 - 4 + r, 0), L.h - 1), gx = x0 - 16 + 16 * q;
            uint4 v = make_uint4(0, 0, 0, 0);   // (columns outside the row: only ever read for frame pixels)
            if (gx >= 0 && gx < L.pitch) v = *reinterpret_cast<const uint4*>(src + (int64_t)gy * L.pitch + gx);
            *reinterpret_cast<uint4*>(&ti[r][16 * q]) = v;
        }
        __syncthreads();
        // r04: a quick necessary test first -- an arc of 9 holds two ring pixels 4 apart among 0, 4, 8, 12
        // (any 8 consecutive positions hold two such, 4 apart), so a corner has some k in {0, 4, 8, 12} with
        // d_k, d_k+4 both > t or both < -t; the positions passing it are compacted in LDS and only they get
        // the full score (the tile pass was VALU-bound on the full score of every position, PMC r04h / r04i)
        // rows across the waves, columns across the lanes (no index division), then the last two columns
        auto pretest = [&](int sy, int sx, bool ok) {
            bool pass = false;
            if (ok) {
                const uint8_t* c = &ti[sy + 3][sx + 15];
                const int v = c[0], d0 = v - c[3 * FI_C], d4 = v - c[3], d8 = v - c[-3 * FI_C], d12 = v - c[-3];
                const int M = max(max(min(d0, d4), min(d4, d8)), max(min(d8, d12), min(d12, d0)));
                const int N = min(min(max(d0, d4), max(d4, d8)), min(max(d8, d12), max(d12, d0)));
                pass = M > threshold || N < -threshold;
            }
            ts[sy][sx] = 0;
            const uint64_t m = __ballot(pass);
            int wb = 0;
            if (lane == 0 && m) wb = atomicAdd(&ncand, __popcll(m));
            wb = __shfl(wb, 0);
            if (pass) cand[wb + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)(sy * FS_C + sx);
        };
        {
            const int xl = x0 - 1 + lane;
            const bool colok = xl >= 3 && xl < L.w - 3;
            for (int sy = wid; sy < FS_R; sy += 4) {
                const int y = y0 - 1 + sy;
                pretest(sy, lane, colok && y >= 3 && y < L.h - 3);
            }
            static_assert(FS_C - 64 == 2 && 2 * FS_R <= 128, "two trailing columns on waves 0 and 1");
            if (wid < 2) {
                const int e = threadIdx.x, sy = e >> 1, sx = 64 + (e & 1);
                const int xe = x0 - 1 + sx, y = y0 - 1 + sy;
                if (sy < FS_R) pretest(sy, sx, xe >= 3 && xe < L.w - 3 && y >= 3 && y < L.h - 3);
            }
        }
        __syncthreads();
        const int nc = ncand;
        for (int c = threadIdx.x; c < nc; c += 256) {
            const int i = cand[c], sy = i / FS_C, sx = i - sy * FS_C;
            ts[sy][sx] = (uint8_t)fast_score_lds<FI_C>(&ti[sy + 3][sx + 15], threshold);
        }
        __syncthreads();
        uint8_t* sc = score_g + L.off;
        const int x = x0 + lane;
        for (int ty = wid; ty < ny; ty += 4) {
            const int y = y0 + ty;
            const int s = ts[ty + 1][lane + 1];
            bool keep = false;
            if (s && y >= b && y < L.h - b && x >= b && x < L.w - b)
                keep = s > ts[ty][lane] && s > ts[ty][lane + 1] && s > ts[ty][lane + 2] && s > ts[ty + 1][lane] &&
                       s > ts[ty + 1][lane + 2] && s > ts[ty + 2][lane] && s > ts[ty + 2][lane + 1] && s > ts[ty + 2][lane + 2];
            const uint64_t m = __ballot(keep);
            if (lane == 0) {
                km[(int64_t)ty * mw] = m;
                wc[(int64_t)ty * mw] = (uint8_t)__popcll(m);
            }
            if (keep) sc[(int64_t)y * L.pitch + x] = (uint8_t)s;
        }
        if (bl) {
            __syncthreads();   // (the score tile and the candidate list are dead: rs aliases them)
            blur_rows<FI_C>(src, L, x0, y0, &ti[0][0], rs);
            __syncthreads();
            blur_cols(L, x0, y0, rs, bl);
        }
    }
}

__device__ __forceinline__ int find_level(const Lvl* lv, int nl, int row) {
    int l = 0;
    while (l + 1 < nl && row >= lv[l + 1].row0) l++;
    return l;
}

// exclusive scan of the n rows' corner counts (the sums of their mw word counts) into off[0..n]
// (one workgroup per image); also clears retainBest's error flag
__global__ __launch_bounds__(1024)
void orb_scan_kernel(const uint8_t* __restrict__ wcnt, int mw, int n, int* __restrict__ off, int64_t istride,
                     int* __restrict__ stats, const Lvl* __restrict__ lv, int nl) {
    __shared__ int part[1024];
    wcnt = at(wcnt, (int64_t)blockIdx.x * istride);
    off = at(off, (int64_t)blockIdx.x * istride);
    if (threadIdx.x == 0) stats[(int64_t)blockIdx.x * CS + ST_TAIL + 3] = 0;   // retainBest's error flag
    auto row_sum = [&](int i) {   // the row's level's ceil(w / 64) words; rows 4-byte aligned (mw % 4 == 0)
        const uint32_t* w = reinterpret_cast<const uint32_t*>(wcnt + (int64_t)i * mw);
        const int nw = (lv[find_level(lv, nl, i)].w + 63) >> 6;
        uint32_t s = 0;
        for (int k = 0; k < nw / 4; ++k) s = __builtin_amdgcn_sad_u8(w[k], 0u, s);
        if (nw & 3) s = __builtin_amdgcn_sad_u8(w[nw / 4] & ((1u << (8 * (nw & 3))) - 1u), 0u, s);
        return (int)s;
    };
    const int per = (n + 1023) / 1024;
    const int b = threadIdx.x * per, e = min(b + per, n);
    int cnt[8];
    int s = 0;
    for (int i = b, j = 0; i < e; i++, j++) {
        const int c = row_sum(i);
        if (j < 8) cnt[j] = c;
        s += c;
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (int i = b, j = 0; i < e; i++, j++) {
        off[i] = run;
        run += j < 8 ? cnt[j] : row_sum(i);
    }
    if (threadIdx.x == 1023) off[n] = part[1023];
}

// the corners of every row in raster order at the row's scanned offset (packed (y << 16) | x and the
// FAST score): one wave per row, the row's keep words in the lanes, walked word by word
__global__ __launch_bounds__(256)
void orb_rows_kernel(const uint8_t* __restrict__ score, const Lvl* __restrict__ lv, int nl, int rows,
                     const int* __restrict__ row_off, const uint64_t* __restrict__ kmask, int mw, int32_t* __restrict__ cpos,
                     uint8_t* __restrict__ cscore, int cap, int64_t istride) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    const int64_t bo = (int64_t)blockIdx.y * istride;
    row_off = at(row_off, bo);
    int base = row_off[row];
    if (row_off[row + 1] == base) return;
    score = at(score, bo);
    kmask = at(kmask, bo) + (int64_t)row * mw;
    cpos = at(cpos, bo);
    cscore = at(cscore, bo);
    const Lvl L = lv[find_level(lv, nl, row)];
    const int y = row - L.row0, nw = (L.w + 63) >> 6;
    const uint8_t* s = score + L.off + (int64_t)y * L.pitch;
    for (int c0 = 0; c0 < nw; c0 += 64) {
        const uint64_t mine = c0 + lane < nw ? kmask[c0 + lane] : 0;
        const int nn = min(64, nw - c0);
        for (int j = 0; j < nn; ++j) {
            const uint64_t m = __shfl(mine, j);
            if (!m) continue;
            if ((m >> lane) & 1) {
                const int k = base + __popcll(m & ((1ull << lane) - 1)), x = (c0 + j) * 64 + lane;
                if (k < cap) {   // (always: one strict maximum per 2 x 2 cell at most; the host checks the total)
                    cpos[k] = (y << 16) | x;
                    cscore[k] = s[x];
                }
            }
            base += __popcll(m);
        }
    }
}

// ------------------------------------------------------------------ device retainBest
// KeyPointsFilter::retainBest (std::nth_element + std::partition with libstdc++'s algorithms) on
// (response, payload) records, one 1024-thread workgroup per pyramid level, giving the permutation
// the reference's host call gives (tests/cpp/orb_select_sim.cpp checks the formulation against
// libstdc++ itself, tests/test_gpu_orb.py the kernels against the oracle):
//  * __introselect's loop, median-of-3 pivot, final insertion sort and __heap_select fallback run as
//    libstdc++ writes them (the serial pieces on thread 0);
//  * __unguarded_partition (comp = response greater) in parallel: its left scan stops at the
//    positions with response <= P (Ls, ascending), its right scan at response >= P (Rs, from the
//    right); the k-th stops are swapped while Ls[k] < Rs[k] (K pairs: Ls rises, Rs falls), every
//    stop is at an original position (swapped ones lie behind both scans), and the cut is
//    min(Ls[K + 1], Rs[K]);
//  * the bidirectional std::partition (pred = response >= the boundary response) the same way.
// Positions are found by per-thread contiguous chunks and one block scan; Ls / Rs live in scratch.
struct Resp { float response; int32_t idx; };
constexpr int RT = 1024;                      // threads of a selection workgroup
struct SelCounts { int n[MAX_LEVELS]; };      // the retainBest argument per level

__device__ __forceinline__ void wg_sync() { __threadfence_block(); __syncthreads(); }

// exclusive block scan of (a, b) over RT threads; the totals land in sh[32], sh[33] (sh: 36 ints)
__device__ __forceinline__ void scan2(int& a, int& b, int* sh) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int ia = a, ib = b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int xa = __shfl_up(ia, o), xb = __shfl_up(ib, o);
        if (lane >= o) { ia += xa; ib += xb; }
    }
    __syncthreads();   // sh may still be read by a previous step
    if (lane == 63) { sh[w] = ia; sh[16 + w] = ib; }
    __syncthreads();
    if (t == 0) {
        int sa = 0, sb = 0;
        for (int i = 0; i < RT / 64; ++i) {
            const int va = sh[i], vb = sh[16 + i];
            sh[i] = sa; sh[16 + i] = sb;
            sa += va; sb += vb;
        }
        sh[32] = sa; sh[33] = sb;
    }
    __syncthreads();
    a = sh[w] + ia - a;
    b = sh[16 + w] + ib - b;
}
__device__ __forceinline__ int block_sum_i(int v, int* sh) {
    const int t = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();
    if ((t & 63) == 0) sh[t >> 6] = v;
    __syncthreads();
    int s = 0;
    for (int i = 0; i < RT / 64; ++i) s += sh[i];
    return s;
}

// The pairing of two scans over [f, l): left stops where lstop(response), right stops where
// rstop(response).  Swaps the K pairs; returns K, with nL / nR and the stop lists in Ls / Rs.
template <class LS, class RS>
__device__ int wg_pair_swap(Resp* __restrict__ a, int f, int l, LS lstop, RS rstop, int* __restrict__ Ls,
                            int* __restrict__ Rs, int* sh, int& nL, int& nR) {
    const int t = threadIdx.x, n = l - f, chunk = (n + RT - 1) / RT;
    const int s = min(f + t * chunk, l), e = min(s + chunk, l);
    int cL = 0, cR = 0;
    for (int p = s; p < e; ++p) {
        const float v = a[p].response;
        cL += lstop(v);
        cR += rstop(v);
    }
    scan2(cL, cR, sh);
    nL = sh[32];
    nR = sh[33];
    for (int p = s; p < e; ++p) {
        const float v = a[p].response;
        if (lstop(v)) Ls[cL++] = p;
        if (rstop(v)) Rs[cR++] = p;
    }
    wg_sync();
    const int kmax = min(nL, nR);
    int c = 0;
    for (int k = t; k < kmax; k += RT) c += Ls[k] < Rs[nR - 1 - k];
    const int K = block_sum_i(c, sh);
    for (int k = t; k < K; k += RT) {
        const int pl = Ls[k], pr = Rs[nR - 1 - k];
        const Resp x = a[pl], y = a[pr];
        a[pl] = y;
        a[pr] = x;
    }
    wg_sync();
    return K;
}

__device__ __forceinline__ bool resp_gt(const Resp& x, const Resp& y) { return x.response > y.response; }

// libstdc++ stl_heap.h, thread 0 only (the depth-limit fallback of __introselect)
__device__ void heap_adjust(Resp* v, int hole, int len, Resp value) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (resp_gt(v[second], v[second - 1])) second--;
        v[hole] = v[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        v[hole] = v[second - 1];
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && resp_gt(v[parent], value)) {
        v[hole] = v[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    v[hole] = value;
}
__device__ void heap_select(Resp* v, int middle, int last) {   // on [0, last), heap [0, middle)
    if (middle >= 2)
        for (int parent = (middle - 2) / 2;; --parent) {
            heap_adjust(v, parent, middle, v[parent]);
            if (parent == 0) break;
        }
    for (int i = middle; i < last; ++i)
        if (resp_gt(v[i], v[0])) {
            const Resp value = v[i];
            v[i] = v[0];
            heap_adjust(v, 0, middle, value);
        }
}
__device__ __forceinline__ void swap_r(Resp* v, int i, int j) { const Resp x = v[i]; v[i] = v[j]; v[j] = x; }

// retainBest(n) on a[0, m): the kept count; a[0, count) holds the kept records in the order the
// reference's KeyPoint vector has them
__device__ int wg_retain(Resp* __restrict__ a, int m, int n, int* __restrict__ Ls, int* __restrict__ Rs, int* sh,
                         int* __restrict__ err) {
    const int t = threadIdx.x;
    if (m <= n) return m;
    if (n == 0) return 0;
    const int nth = n - 1;
    int first = 0, last = m, depth = 2 * (31 - __clz(m));
    bool heaped = false;
    while (last - first > 3) {
        if (depth == 0) {
            if (t == 0) {
                heap_select(a + first, nth + 1 - first, last - first);
                swap_r(a, first, nth);
            }
            wg_sync();
            heaped = true;
            break;
        }
        --depth;
        if (t == 0) {   // __move_median_to_first(first, first + 1, mid, last - 1)
            const int x = first + 1, y = first + (last - first) / 2, z = last - 1;
            int pick;
            if (resp_gt(a[x], a[y])) pick = resp_gt(a[y], a[z]) ? y : resp_gt(a[x], a[z]) ? z : x;
            else pick = resp_gt(a[x], a[z]) ? x : resp_gt(a[y], a[z]) ? z : y;
            swap_r(a, first, pick);
        }
        wg_sync();
        const float P = a[first].response;
        int nL, nR;
        const int K = wg_pair_swap(a, first + 1, last, [P](float v) { return v <= P; }, [P](float v) { return v >= P; },
                                   Ls, Rs, sh, nL, nR);
        int cut = INT_MAX;
        if (K < nL) cut = Ls[K];
        if (K >= 1) cut = min(cut, Rs[nR - K]);
        if (cut <= first || cut >= last) {   // impossible for the pairing above; never loop on it
            if (t == 0) atomicOr(err, 1);
            heaped = true;
            break;
        }
        if (cut <= nth) first = cut;
        else last = cut;
    }
    if (!heaped) {
        if (t == 0)   // __insertion_sort(first, last)
            for (int i = first + 1; i < last; ++i) {
                const Resp val = a[i];
                if (resp_gt(val, a[first])) {
                    for (int j = i; j > first; --j) a[j] = a[j - 1];
                    a[first] = val;
                } else {
                    int j = i;
                    while (resp_gt(val, a[j - 1])) { a[j] = a[j - 1]; --j; }
                    a[j] = val;
                }
            }
        wg_sync();
    }
    const float amb = a[nth].response;
    int nL, nR;
    wg_pair_swap(a, n, m, [amb](float v) { return v < amb; }, [amb](float v) { return v >= amb; }, Ls, Rs, sh, nL, nR);
    return n + nR;
}

__device__ __forceinline__ int lvl_first(const int* __restrict__ row_off, const Lvl& L) { return row_off[L.row0]; }

// mode 0: level l's FAST corners (raster order) -> retainBest(2 n_l) -> cnt[l] records in A (payload:
// the corner index); mode 1: the kept corners' Harris responses in B (payload: the position in the
// level's kept list) -> retainBest(n_l) -> cnt[l]
__global__ __launch_bounds__(RT)
void orb_retain_kernel(int mode, const Lvl* __restrict__ lv, const int* __restrict__ row_off,
                       const uint8_t* __restrict__ cscore, Resp* __restrict__ A, Resp* __restrict__ B,
                       int* __restrict__ Ls, int* __restrict__ Rs, const int* __restrict__ cnt_in,
                       int* __restrict__ cnt_out, SelCounts sel, int cap, int* __restrict__ err, int64_t istride) {
    __shared__ int sh[36];
    const int l = blockIdx.x, t = threadIdx.x, g = blockIdx.y;
    {   // image g: its arrays and its counters (cnt_in / cnt_out / err are offsets into the stats rows)
        const int64_t bo = (int64_t)g * istride;
        row_off = at(row_off, bo);
        cscore = at(cscore, bo);
        A = at(A, bo);
        B = at(B, bo);
        Ls = at(Ls, bo);
        Rs = at(Rs, bo);
        if (cnt_in) cnt_in += (int64_t)g * CS;
        cnt_out += (int64_t)g * CS;
        err += (int64_t)g * CS;
    }
    const Lvl L = lv[l];
    const int c0 = min(lvl_first(row_off, L), cap);   // (the corner count never exceeds cap: one per 2 x 2 cell)
    int m;
    Resp* a;
    if (mode == 0) {
        m = min(row_off[L.row0 + L.h], cap) - c0;
        a = A + c0;
        for (int j = t; j < m; j += RT) a[j] = Resp{(float)cscore[c0 + j], c0 + j};
        wg_sync();
    } else {
        m = cnt_in[l];
        a = B + c0;
    }
    const int k = wg_retain(a, m, sel.n[l], Ls + c0, Rs + c0, sh, err);
    if (t == 0) cnt_out[l] = k;
}

// Harris response (7x7 block, k = 0.04) of every kept corner: grid (x, level)
// EDGE (edgeThreshold < 4): windows may leave the level (the reflected reads); the default instantiation
// keeps r04's register budget
template <bool EDGE>
__global__ __launch_bounds__(256)
void orb_harris_kernel(const uint8_t* __restrict__ pyr, const Lvl* __restrict__ lv, const int* __restrict__ row_off,
                       const Resp* __restrict__ A, const int* __restrict__ cnt1, const int32_t* __restrict__ cpos,
                       Resp* __restrict__ B, int64_t istride) {
    const int l = blockIdx.y;
    {
        const int64_t bo = (int64_t)blockIdx.z * istride;
        pyr = at(pyr, bo);
        row_off = at(row_off, bo);
        A = at(A, bo);
        cnt1 += (int64_t)blockIdx.z * CS;
        cpos = at(cpos, bo);
        B = at(B, bo);
    }
    const Lvl L = lv[l];
    const int c0 = lvl_first(row_off, L), m = cnt1[l];
    const uint8_t* img = pyr + L.off;
    const int step = L.pitch;
    static_assert(HARRIS_BLOCK == 7, "9 x 9 pixel window");
    for (int j = blockIdx.x * 256 + threadIdx.x; j < m; j += gridDim.x * 256) {
        const int pos = cpos[A[c0 + j].idx], x0 = pos & 0xFFFF, y0 = pos >> 16;
        // r04: the 9 x 9 window (rows y0-4 .. y0+4, columns x0-4 .. x0+4) as 27 aligned 4-byte loads
        // (rows are 64-byte aligned; a corner lies >= 31 pixels inside its level), realigned with
        // v_alignbyte; r03 made 392 byte loads per corner.  The sums are integers: the same values.
        uint32_t win[9][3];
        if (!EDGE || (x0 >= 4 && x0 + 4 < L.w && y0 >= 4 && y0 + 4 < L.h)) {
            const int xa = (x0 - 4) & ~3, sh = (x0 - 4) & 3;
            const uint8_t* base = img + (int64_t)(y0 - 4) * step + xa;
#pragma unroll
            for (int rr = 0; rr < 9; ++rr) {
                const uint32_t* q = reinterpret_cast<const uint32_t*>(base + (int64_t)rr * step);
                const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
                win[rr][0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
                win[rr][1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
                win[rr][2] = __builtin_amdgcn_alignbyte(0u, w2, sh);
            }
        } else {   // (r05: edgeThreshold < 4) the window leaves the level: OpenCV's bordered pyramid, reflected
#pragma unroll
            for (int rr = 0; rr < 9; ++rr) {
                const uint8_t* row = img + (int64_t)reflect101(y0 - 4 + rr, L.h) * step;
                uint32_t w[3] = {0u, 0u, 0u};
#pragma unroll
                for (int cc = 0; cc < 9; ++cc) w[cc >> 2] |= (uint32_t)row[reflect101(x0 - 4 + cc, L.w)] << (8 * (cc & 3));
                win[rr][0] = w[0];
                win[rr][1] = w[1];
                win[rr][2] = w[2];
            }
        }
        auto px = [&](int rr, int cc) -> int { return (int)((win[rr][cc >> 2] >> (8 * (cc & 3))) & 255u); };
        int a = 0, b = 0, c = 0;
#pragma unroll
        for (int ii = 1; ii <= HARRIS_BLOCK; ii++) {
#pragma unroll
            for (int jj = 1; jj <= HARRIS_BLOCK; jj++) {
                const int Ix = (px(ii, jj + 1) - px(ii, jj - 1)) * 2 + (px(ii - 1, jj + 1) - px(ii - 1, jj - 1)) +
                               (px(ii + 1, jj + 1) - px(ii + 1, jj - 1));
                const int Iy = (px(ii + 1, jj) - px(ii - 1, jj)) * 2 + (px(ii + 1, jj - 1) - px(ii - 1, jj - 1)) +
                               (px(ii + 1, jj + 1) - px(ii - 1, jj + 1));
                a += Ix * Ix;
                b += Iy * Iy;
                c += Ix * Iy;
            }
        }
        const float scale = 1.f / ((1 << 2) * HARRIS_BLOCK * 255.f);
        const float scale_sq_sq = scale * scale * scale * scale;
        B[c0 + j] = Resp{((float)a * b - (float)c * c - HARRIS_K * ((float)a + b) * ((float)a + b)) * scale_sq_sq, j};
    }
}

__device__ float fast_atan2(float y, float x) {   // cv::fastAtan2
    constexpr float R2D = (float)(180 / 3.14159265358979323846);
    constexpr float P1 = 0.9997878412794807f * R2D, P3 = -0.3258083974640975f * R2D, P5 = 0.1555786518463281f * R2D,
                    P7 = -0.04432655554792128f * R2D;
    const float ax = fabsf(x), ay = fabsf(y);
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

// the final keypoints in level order -> cv::KeyPoint with ICAngles' angle (one wavefront per
// keypoint: the 31 patch rows u = -15..15 across lanes; integer moments, so the lane order is
// irrelevant), and compute()'s runByImageBorder(31) test at full resolution (Rect::contains(Point(pt)))
// EDGE (edgeThreshold < 15): patches may leave the level (the reflected reads)
template <bool EDGE>
__global__ __launch_bounds__(256)
void orb_angle_kernel(const uint8_t* __restrict__ pyr, const Lvl* __restrict__ lv, int nl,
                      const int* __restrict__ row_off, int rows, int* __restrict__ stats, const int* __restrict__ umax,
                      const Resp* __restrict__ kin, const int* __restrict__ sidx, Kp* __restrict__ out, int64_t istride) {
    const int lane = threadIdx.x & 63;
    {
        const int64_t bo = (int64_t)blockIdx.y * istride;
        pyr = at(pyr, bo);
        row_off = at(row_off, bo);
        stats += (int64_t)blockIdx.y * CS;
        kin = at(kin, bo);
        if (sidx) sidx = at(sidx, bo);
        out = at(out, bo);
    }
    __shared__ int sumax[HALF_PATCH + 1], lbase[MAX_LEVELS + 1], lfirst[MAX_LEVELS];
    if (threadIdx.x <= HALF_PATCH) sumax[threadIdx.x] = umax[threadIdx.x];
    if (threadIdx.x == 0) {   // the kept keypoints' level offsets; block 0 publishes count, levels, corners
        int b = 0, used = 0;
        for (int l = 0; l < nl; ++l) {
            lbase[l] = b;
            lfirst[l] = lvl_first(row_off, lv[l]);
            b += stats[ST_KCNT + l];
            if (stats[ST_KCNT + l] > 0) used = l + 1;
        }
        lbase[nl] = b;
        if (blockIdx.x == 0) {
            stats[ST_TAIL + 0] = b;
            stats[ST_TAIL + 1] = used;
            stats[ST_TAIL + 2] = row_off[rows];
        }
    }
    __syncthreads();
    // two keypoints per wave (r04), 32 lanes each: this lane's words of the 31 patch rows (9 aligned words a
    // row, 279 in all, 9 per lane), the same for every keypoint
    const int hl = lane & 31;
    constexpr int NWD = (2 * HALF_PATCH + 1) * 9, NK = (NWD + 31) / 32;
    bool wok[NK];
    int wd[NK], wrow[NK], wum[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const int idx = hl + 32 * k, r = idx / 9;
        wok[k] = idx < NWD;
        wd[k] = idx - 9 * r;
        wrow[k] = r - HALF_PATCH;
        wum[k] = wok[k] ? sumax[wrow[k] < 0 ? -wrow[k] : wrow[k]] : 0;
    }
    const int total = lbase[nl];   // the kept keypoints (orb_keep_kernel), walked in sidx's row order
    int t0, t1, tstep = 8;
    if (sidx) {
        xcd_range(total, t0, t1);
        t0 += (threadIdx.x >> 6) * 2 + (lane >> 5);
    } else {   // (diagnostic A/B: the kept order, strided over the grid, as r04)
        t0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
        t1 = total;
        tstep = gridDim.x * 8;
    }
    for (int ts = t0; ts < t1; ts += tstep) {
        const int f = sidx ? sidx[ts] : ts;
        int l = 0;
        while (f >= lbase[l + 1]) ++l;
        const Lvl L = lv[l];
        const Resp e = kin[lfirst[l] + f - lbase[l]];   // (response, packed position)
        const int pos = e.idx, cx = pos & 0xFFFF, cy = pos >> 16;
        const uint8_t* img = pyr + L.off;
        const int step = L.pitch;
        // the 31 patch rows as aligned 4-byte words (columns (cx-15) & ~3 ..); a pixel counts where
        // |u| <= umax[|v|] (integer moments: any order, the same sums).  r03 made 31 byte loads per
        // lane, one row at a time.
        const int xa = (cx - HALF_PATCH) & ~3;
        int m10 = 0, m01 = 0;
        if (EDGE && !(cx >= HALF_PATCH && cx + HALF_PATCH < L.w && cy >= HALF_PATCH && cy + HALF_PATCH < L.h)) {
            // (r05: edgeThreshold < 15) the patch leaves the level: OpenCV's bordered pyramid, reflected;
            // lane hl takes patch row v = hl - 15 pixel by pixel
            if (hl < 2 * HALF_PATCH + 1) {
                const int v = hl - HALF_PATCH, d = sumax[v < 0 ? -v : v];
                const uint8_t* row = img + (int64_t)reflect101(cy + v, L.h) * step;
                for (int u = -d; u <= d; ++u) {
                    const int I = row[reflect101(cx + u, L.w)];
                    m10 += u * I;
                    m01 += v * I;
                }
            }
        } else {
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            if (!wok[k]) continue;
            // the word's pixels inside the circle (|u| <= umax[|v|]) are one byte run [lo, hi]; with
            // the others masked off, sum I and sum i I come from two v_dot4_u32_u8:
            // sum u I = (X - cx) sum I + sum i I, X the word's first column
            const int X = xa + 4 * wd[k], lo = max(0, cx - wum[k] - X), hi = min(3, cx + wum[k] - X);
            const uint32_t mask = lo <= hi ? (0xFFFFFFFFu >> (8 * (3 - hi + lo))) << (8 * lo) : 0u;
            const uint32_t w = *reinterpret_cast<const uint32_t*>(img + (int64_t)(cy + wrow[k]) * step + X) & mask;
            const int s1 = (int)__builtin_amdgcn_udot4(w, 0x01010101u, 0u, false);
            const int si = (int)__builtin_amdgcn_udot4(w, 0x03020100u, 0u, false);
            m10 += (X - cx) * s1 + si;
            m01 += wrow[k] * s1;
        }
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) {   // the half-wave's sums (xor partners stay in the half)
            m10 += __shfl_xor(m10, o);
            m01 += __shfl_xor(m01, o);
        }
        if (hl == 0) {
            Kp q;
            q.x = (float)cx * L.scale;
            q.y = (float)cy * L.scale;
            q.size = PATCH * L.scale;
            q.angle = fast_atan2((float)m01, (float)m10);
            q.response = e.response;
            q.octave = l;
            q.class_id = -1;
            out[f] = q;
        }
    }
}

// compute()'s runByImageBorder(31) on the full-resolution positions (Rect::contains(Point(pt)), pt =
// the level position x scale) of every level's retained keypoints, and their places in the kept list,
// before the angles (r04: the angle kernel writes the kept keypoints in place; r03 wrote them all and
// compacted them in one workgroup per image).  One workgroup per (level, image), rounds of RT records
// scanned in order: kin[c0 + i] = (response, packed position) of the level's i-th kept keypoint,
// kcnt[l] = their count.
__global__ __launch_bounds__(RT)
void orb_keep_kernel(const Lvl* __restrict__ lv, const int* __restrict__ row_off, const Resp* __restrict__ A,
                     const Resp* __restrict__ B, int* __restrict__ stats, const int32_t* __restrict__ cpos, int width,
                     int height, int border, Resp* __restrict__ kin, int64_t istride) {
    __shared__ int sh[36];
    const int l = blockIdx.x, t = threadIdx.x;
    {
        const int64_t bo = (int64_t)blockIdx.y * istride;
        row_off = at(row_off, bo);
        A = at(A, bo);
        B = at(B, bo);
        stats += (int64_t)blockIdx.y * CS;
        cpos = at(cpos, bo);
        kin = at(kin, bo);
    }
    const Lvl L = lv[l];
    const int c0 = lvl_first(row_off, L), m = stats[ST_CNT2 + l];
    const bool fits = height > 2 * border && width > 2 * border;
    int base = 0;
    for (int r0 = 0; r0 < m; r0 += RT) {   // (block-uniform)
        const int j = r0 + t;
        int k = 0, pos = 0;
        float resp = 0.f;
        if (j < m) {
            const Resp e = B[c0 + j];
            pos = cpos[A[c0 + e.idx].idx];
            resp = e.response;
            const int x = round_f((float)(pos & 0xFFFF) * L.scale), y = round_f((float)(pos >> 16) * L.scale);
            k = fits && border <= x && x < width - border && border <= y && y < height - border;
        }
        int pre = k, dummy = 0;
        scan2(pre, dummy, sh);   // exclusive prefix over the round; its total in sh[32]
        if (k) kin[c0 + base + pre] = Resp{resp, pos};   // the level's kept keypoints, dense, in order
        base += sh[32];
    }
    if (t == 0) stats[ST_KCNT + l] = base;
}

// r05: the kept keypoints' processing order for the angle and rBRIEF passes.  Both
// read a patch around every keypoint; in the kept (retainBest) order the patches of consecutive
// keypoints are scattered over the level, so every patch row came from the MALL / HBM again (the
// angle pass fetched ~2 KB per keypoint).  sidx lists the kept keypoints (their output indices f)
// bucketed by level row (SB buckets of whole rows per level, one workgroup per (level, image)); the
// two passes walk it in contiguous ranges per workgroup, the ranges of one XCD adjacent (xcd_range), so
// neighbouring patches share L2 lines.  Only the order of the work changes: every output is written
// to its keypoint's own slot, bit-identical.
constexpr int SB = 2048;
__global__ __launch_bounds__(RT)
void orb_sort_kernel(const Lvl* __restrict__ lv, const int* __restrict__ row_off, const int* __restrict__ stats,
                     const Resp* __restrict__ kin, int* __restrict__ sidx, int64_t istride) {
    __shared__ int cnt[SB];
    __shared__ int sh[36];
    const int l = blockIdx.x, t = threadIdx.x;
    {
        const int64_t bo = (int64_t)blockIdx.y * istride;
        row_off = at(row_off, bo);
        stats += (int64_t)blockIdx.y * CS;
        kin = at(kin, bo);
        sidx = at(sidx, bo);
    }
    const Lvl L = lv[l];
    const int m = stats[ST_KCNT + l], c0 = lvl_first(row_off, L);
    int base = 0;
    for (int q = 0; q < l; ++q) base += stats[ST_KCNT + q];
    const int rb = (L.h + SB - 1) / SB;   // rows per bucket
    for (int b = t; b < SB; b += RT) cnt[b] = 0;
    __syncthreads();
    for (int i = t; i < m; i += RT) atomicAdd(&cnt[(kin[c0 + i].idx >> 16) / rb], 1);
    __syncthreads();
    int a = cnt[2 * t], b2 = cnt[2 * t + 1];   // (SB = 2 RT) exclusive scan of the bucket counts
    const int s0 = a + b2;
    int pre = s0, dummy = 0;
    scan2(pre, dummy, sh);
    __syncthreads();
    cnt[2 * t] = base + pre;
    cnt[2 * t + 1] = base + pre + a;
    __syncthreads();
    for (int i = t; i < m; i += RT) sidx[atomicAdd(&cnt[(kin[c0 + i].idx >> 16) / rb], 1)] = base + i;
}
static_assert(SB == 2 * RT, "two buckets per thread in the scan");

__global__ __launch_bounds__(256)
void orb_copy_kp_kernel(const Kp* __restrict__ src, const int* __restrict__ st, const ImgIO* __restrict__ io,
                        int64_t istride) {
    const int g = blockIdx.y;
    src = at(src, (int64_t)g * istride);
    Kp* dst = io[g].kp_out;
    const int m = min(st[(int64_t)g * CS], io[g].capacity);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < m; i += gridDim.x * 256) dst[i] = src[i];
}

// fdlibm-style double sin/cos for the descriptor angle (|x| < 8), the same operation
// sequence as oracle/orb_oracle.cpp:orb_sincos (this file is built with -ffp-contract=off)
__device__ void orb_sincos(double x, double* s, double* c) {
    const double q = rint(x * 6.36619772367581382433e-01);
    const double r = (x - q * 1.57079632673412561417e+00) - q * 6.07710050650619224932e-11;
    const double z = r * r;
    const double sr = r + (z * r) * (-1.66666666666666324348e-01 +
                      z * (8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 +
                      z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 +
                      z * 1.58969099521155010221e-10)))));
    const double cz = z * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 +
                      z * (2.48015872894767294178e-05 + z * (-2.75573143513906633035e-07 +
                      z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * cz);
    switch (((int)q) & 3) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
    }
}

// computeOrbDescriptors (WTA_K 2): 32 lanes per keypoint, lane i builds byte i from
// pattern pairs 8 i .. 8 i + 7; min(count, capacity) keypoints.
// r04: the lane's 16 pattern points are loaded once (they were 32 loads per keypoint, half the
// kernel's memory instructions, PMC r04h), and the keypoint's 37 x 37 sample window (|round(rotated
// pattern point)| <= 18: the pattern lies in [-13, 12]^2) is staged in LDS by 16-byte loads, one
// window per keypoint slot; keypoints whose window needs the edge clamp read the level directly.
constexpr int BW = 18;                 // window half-size
constexpr int BWR = 2 * BW + 1, BWC = 80;   // (80-byte rows: 20 banks apart, not 16 -- fewer conflicts)
// EDGE (edgeThreshold < 19): samples may leave the level (the bordered pyramid's unblurred reflected pixels);
// otherwise a window touching the edge stays inside it and reads the blurred level directly
template <bool EDGE>
__global__ __launch_bounds__(256)
void orb_brief_kernel(const uint8_t* __restrict__ blur, const uint8_t* __restrict__ pyr, const Lvl* __restrict__ lv,
                      const Kp* __restrict__ kps, const int* __restrict__ sidx, const int* __restrict__ st,
                      const ImgIO* __restrict__ io, int64_t istride, int xcd) {
    __shared__ __align__(16) uint8_t win[8][BWR * BWC];
    int bx, g, bz;   // (the output order: one XCD's workgroups take whole images, xcd_grid)
    xcd_grid(sidx ? 0 : xcd, bx, g, bz);
    blur = at(blur, (int64_t)g * istride);
    pyr = at(pyr, (int64_t)g * istride);
    kps = at(kps, (int64_t)g * istride);
    if (sidx) sidx = at(sidx, (int64_t)g * istride);
    uint8_t* desc = io[g].desc_out;
    if (!desc) return;   // this image's caller passed no descriptor buffer
    const int n = min(st[(int64_t)g * CS], io[g].capacity), i = threadIdx.x & 31, slot = threadIdx.x >> 5;
    uint8_t* wn = win[slot];
    float pxf[16], pyf[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        pxf[e] = (float)c_pattern[2 * (16 * i + e)];
        pyf[e] = (float)c_pattern[2 * (16 * i + e) + 1];
    }
    // the kept keypoints in sidx's row order (orb_sort_kernel), contiguous per workgroup; the first
    // min(count, capacity) of the output order are described
    int t0, t1, tstep = 8;
    if (sidx) {
        xcd_range(st[(int64_t)g * CS], t0, t1);
        t0 += slot;
    } else {   // the output order, strided over the image's workgroups
        t0 = bx * 8 + slot;
        t1 = n;
        tstep = gridDim.x * 8;
    }
    for (int ts = t0; ts < t1; ts += tstep) {
        const int j = sidx ? sidx[ts] : ts;
        if (j >= n) continue;
        const Kp k = kps[j];
        const Lvl L = lv[k.octave];
        float angle = k.angle;
        angle *= (float)(3.14159265358979323846 / 180.f);
        double sd, cd;
        orb_sincos((double)angle, &sd, &cd);
        const float a = (float)cd, b = (float)sd;
        const int cy = round_f(k.y * L.inv_scale), cx = round_f(k.x * L.inv_scale);
        const uint8_t* img = blur + L.off;
        const uint8_t* raw = pyr + L.off;
        const int xs = (cx - BW) & ~15;
        const bool staged = cy >= BW && cy + BW < L.h && cx >= BW && cx + BW < L.w;
        __builtin_amdgcn_wave_barrier();   // (the slot's previous window fully read)
        if (staged) {
            const int nq = (cx + BW - xs) / 16 + 1;   // 16-byte words a row (the last one ends inside the pitch)
            for (int e = i; e < BWR * 4; e += 32) {
                const int rr = e >> 2, q = e & 3;
                if (q < nq)
                    *reinterpret_cast<uint4*>(&wn[rr * BWC + 16 * q]) =
                        *reinterpret_cast<const uint4*>(img + (int64_t)(cy - BW + rr) * L.pitch + xs + 16 * q);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        auto value = [&](int e) -> int {
            // (r04: packed fp32 rotations measured slower, 155 -> 186 us per 16 images; kept scalar)
            const float x = pxf[e] * a - pyf[e] * b, y = pxf[e] * b + pyf[e] * a;
            if (staged) return wn[(round_f(y) + BW) * BWC + cx + round_f(x) - xs];
            if (!EDGE) {   // (edgeThreshold >= 19: every sample inside the level; r04's form, its codegen)
                const int yy = min(max(cy + round_f(y), 0), L.h - 1), xx = min(max(cx + round_f(x), 0), L.w - 1);
                return img[(int64_t)yy * L.pitch + xx];
            }
            // (r05: edgeThreshold < 19) a sample outside the level: compute() blurs each level in place
            // inside OpenCV's bordered pyramid, whose border keeps the unblurred reflected pixels
            const int yy = cy + round_f(y), xx = cx + round_f(x);
            if (yy >= 0 && yy < L.h && xx >= 0 && xx < L.w) return img[(int64_t)yy * L.pitch + xx];
            return raw[(int64_t)reflect101(yy, L.h) * L.pitch + reflect101(xx, L.w)];
        };
        int val = 0;
#pragma unroll
        for (int bit = 0; bit < 8; bit++) val |= (value(2 * bit) < value(2 * bit + 1)) << bit;
        desc[(int64_t)j * 32 + i] = (uint8_t)val;
    }
}

// ------------------------------------------------------------------ host
static int host_round_f(float v) { return (int)std::nearbyint(v); }
static int host_round_d(double v) { return (int)std::nearbyint(v); }
static float get_scale(int level, double sf) { return (float)std::pow(sf, (double)level); }

static void linear_axis(int dsize, int ssize, std::vector<AxisEnt>& out, int& dmin, int& dmax) {
    dmin = 0;
    dmax = dsize;
    const double inv = (double)dsize / ssize;
    const double scale = 1.0 / inv;
    for (int v = 0; v < dsize; v++) {
        AxisEnt e{0, 0, 0};
        const double fval = scale * ((double)v + 0.5) - 0.5;
        const int ival = (int)std::floor(fval);
        if (ival >= 0 && ssize > 1) {
            if (ival < ssize - 1) {
                e.ofs = ival;
                e.m1 = (uint16_t)host_round_d((fval - (double)ival) * 256.0);
                e.m0 = (uint16_t)(256 - e.m1);
            } else {
                e.ofs = ssize - 1;
                dmax = std::min(dmax, v);
            }
        } else {
            dmin = std::max(dmin, v + 1);
        }
        out.push_back(e);
    }
}

static void blur_taps(int taps[7]) {   // getGaussianKernel(7, 2, CV_32F) x 2^8 (see the oracle)
    const int n = 7;
    const double sigma = 2.0, scale2X = -0.125 / (sigma * sigma);
    double t[4], sum = 0;
    for (int i = 0, x = 1 - n; i < n / 2; i++, x += 2) {
        t[i] = std::exp((double)(x * x) * scale2X);
        sum += t[i];
    }
    sum *= 2.0;
    sum += 1.0;
    t[n / 2] = 1.0;
    for (int i = 0; i <= n / 2; i++) {
        const float k = (float)(t[i] / sum);
        taps[i] = taps[n - 1 - i] = host_round_d((double)k * 256.0);
    }
}

static std::vector<int> circle_umax() {
    std::vector<int> umax(HALF_PATCH + 2);
    const int vmax = (int)std::floor(HALF_PATCH * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(HALF_PATCH * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v) umax[v] = host_round_d(std::sqrt((double)HALF_PATCH * HALF_PATCH - v * v));
    for (int v = HALF_PATCH, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
    return umax;
}

thread_local float g_last_ms = -1.f;
std::once_flag g_const_once[64];

struct Arena {                 // per-thread device scratch, grown on demand
    int dev = -1;
    char* p = nullptr;
    size_t cap = 0, used = 0;
    bool overflow = false;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    void release() {
        if (dev < 0) return;
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev);
        if (p) (void)hipFree(p);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (prev >= 0) (void)hipSetDevice(prev);
        p = nullptr; cap = 0; e0 = e1 = nullptr; dev = -1;
    }
    bool reserve(int device, size_t bytes) {
        if (dev != device) {
            release();
            (void)hipSetDevice(device);
            dev = device;
        }
        used = 0;
        overflow = false;
        if (bytes > cap) {
            if (p) (void)hipFree(p);
            p = nullptr;
            cap = 0;
            if (hipMalloc(&p, bytes) != hipSuccess) {
                p = nullptr;
                (void)hipGetLastError();   // clear it: a later launch check must not report this
                return false;
            }
            cap = bytes;
        }
        if (!e0 && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) return false;
        return true;
    }
    template <class T> T* take(size_t n) {
        T* r = reinterpret_cast<T*>(p + used);
        used += (sizeof(T) * n + 255) & ~(size_t)255;
        if (used > cap) overflow = true;
        return r;
    }
};

bool is_gfx950(int device) {
    static std::atomic<int> state[64];
    if (device < 0 || device >= 64) return false;
    int v = state[device].load();
    if (v == 0) {
        hipDeviceProp_t prop;
        v = (hipGetDeviceProperties(&prop, device) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) ? 1 : 2;
        state[device].store(v);
    }
    return v == 1;
}

}  // namespace orb
}  // namespace sfmx

using namespace sfmx;
using namespace sfmx::orb;

#define OCHK(expr) do { if ((expr) != hipSuccess) { rc = SFMX_EDEVICE; set_last_error("HIP error in " #expr); goto done; } } while (0)

extern "C" {

void sfmx_orb_default_params(sfmx_orb_params* p) {
    if (!p) return;
    p->nfeatures = 500;
    p->scale_factor = 1.2f;
    p->n_levels = 8;
    p->edge_threshold = 31;
    p->first_level = 0;
    p->wta_k = 2;
    p->score_type = 0;
    p->patch_size = 31;
    p->fast_threshold = 20;
}

float sfmx_orb_last_kernel_ms(void) { return g_last_ms; }

}  // extern "C"

namespace {

struct Scratch {            // image-size buffers / corner-count buffers, grown on demand
    Arena img;
    char* pin = nullptr;    // pinned staging: the chunk's tables / levels / umax / ImgIO up, its stats down
    size_t pin_cap = 0;
    int pin_dev = -1;
    bool pin_reserve(int device, size_t bytes) {
        if (pin && pin_cap >= bytes && pin_dev == device) return true;
        if (pin) (void)hipHostFree(pin);
        pin = nullptr;
        pin_cap = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&pin), bytes, hipHostMallocDefault) != hipSuccess) return false;
        pin_cap = bytes;
        pin_dev = device;
        return true;
    }
};
thread_local Scratch g_scratch;

struct OrbImage { const uint8_t* data; int32_t width, height; int64_t pitch; };

// detect() + compute() of a chunk of G images of one size as one set of launches (image g's arrays
// at g * istride in the arena, its counters at stats + g * CS).  Per image: keypoints[g] /
// descriptors[g] / capacities[g] as the one-image call, n_keypoints[g], rcs[g] its status.
// Returns the first failure that is not a per-image capacity report.
int orb_chunk(const OrbImage* ims, int G, const sfmx_orb_params* P, int32_t inputs_on_device, int32_t device,
              hipStream_t st, sfmx_keypoint* const* keypoints, uint8_t* const* descriptors, const int32_t* capacities,
              int32_t* n_keypoints, int* rcs, Scratch& scratch, float* last_ms) {
    if (!ims || !P || !n_keypoints || G < 1) {
        set_last_error("null argument");
        return SFMX_EINVAL;
    }
    const int width = ims[0].width, height = ims[0].height;
    for (int g = 0; g < G; ++g) {
        const OrbImage& im = ims[g];
        if (!im.data || capacities[g] < 0 || (capacities[g] > 0 && !keypoints[g])) { set_last_error("null argument"); return SFMX_EINVAL; }
        if (im.width < 1 || im.height < 1 || im.pitch < im.width || im.width > 16384 || im.height > 16384) {
            set_last_error("image size must be 1..16384 with pitch >= width");
            return SFMX_EINVAL;
        }
        if (im.width != width || im.height != height) { set_last_error("internal: a chunk mixes image sizes"); return SFMX_EINTERNAL; }
    }
    if (P->nfeatures < 0 || !(P->scale_factor > 1.f) || P->n_levels < 1 || P->n_levels > MAX_LEVELS ||
        P->edge_threshold < 0 || P->edge_threshold > 256 || P->first_level != 0 || P->wta_k != 2 ||
        P->score_type != 0 || P->patch_size != 31 || P->fast_threshold < 0) {
        // (r05: every edgeThreshold from 0: the Harris window, the angle patch and rBRIEF's samples that leave
        // a level read OpenCV's bordered pyramid -- its BORDER_REFLECT_101 copy of the level, unblurred)
        set_last_error("unsupported ORB parameters (edgeThreshold 0..256, firstLevel 0, WTA_K 2, HARRIS_SCORE, patchSize 31)");
        return SFMX_EINVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { set_last_error("no HIP device visible"); return SFMX_EDEVICE; }
    if (device < 0 || device >= ndev) { set_last_error("device index out of range"); return SFMX_EINVAL; }
    if (!is_gfx950(device)) { set_last_error("sfmx kernels are built for gfx950 only"); return SFMX_EDEVICE; }
    // levels, their packed layout and resize tables (host)
    const double sf = (double)P->scale_factor;
    const int nl = P->n_levels, border = P->edge_threshold;
    const int thr = std::min(std::max(P->fast_threshold, 0), 255);
    std::vector<Lvl> lv(nl);
    std::vector<AxisEnt> tables;
    int64_t px = 0;
    int rows = 0, maxw = 0, maxh = 0;
    for (int l = 0; l < nl; l++) {
        Lvl& L = lv[l];
        L = Lvl{};
        L.scale = get_scale(l, sf);
        L.inv_scale = 1.f / L.scale;
        const float inv = 1.0f / L.scale;
        L.w = host_round_f(width * inv);
        L.h = host_round_f(height * inv);
        if (L.w < 1 || L.h < 1) { set_last_error("pyramid level of zero size (image too small for n_levels)"); return SFMX_EINVAL; }
        L.pitch = (L.w + 63) & ~63;
        L.off = px;
        L.row0 = rows;
        px += ((int64_t)L.pitch * L.h + 255) & ~(int64_t)255;
        rows += L.h;
        maxw = std::max(maxw, L.w);
        maxh = std::max(maxh, L.h);
        if (l > 0) {
            L.ax_off = (int)tables.size();
            linear_axis(L.w, lv[l - 1].w, tables, L.xdmin, L.xdmax);
            L.ay_off = (int)tables.size();
            linear_axis(L.h, lv[l - 1].h, tables, L.ydmin, L.ydmax);
        }
    }
    std::vector<int> per(nl);                  // computeKeyPoints' nfeaturesPerLevel
    {
        const float factor = (float)(1.0 / sf);
        float nd = P->nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
        int sum = 0;
        for (int l = 0; l < nl - 1; l++) {
            per[l] = host_round_f(nd);
            sum += per[l];
            nd *= factor;
        }
        per[nl - 1] = std::max(P->nfeatures - sum, 0);
    }
    const std::vector<int> umax = circle_umax();
    const int64_t CAND_CAP = px / 4 + 1024;    // strict 3x3 maxima: at most one per 2 x 2 cell
    int capmax = 0;
    for (int g = 0; g < G; ++g) capmax = std::max(capmax, (int)capacities[g]);
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    int rc = SFMX_OK;
    {
        // one image's block: pyr / score / blur slabs, corner records (cpos 4 + cscore 1 + A, B 8 + 8 + Ls, Rs
        // 4 + 4 + kept keypoints 28 + kept records 8), row offsets, keep words / counts, the input copy and the
        // descriptor staging (host buffers) -- every part 256-B aligned, so the offsets are the same in
        // every block
        auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
        const int mw = (maxw + 255) / 256 * 4;   // keep words per row (64 pixels each; a multiple of 4)
        const size_t blk = 3 * r(px) + r(CAND_CAP * 4) + r(CAND_CAP) + 2 * r(CAND_CAP * sizeof(Resp)) + 2 * r(CAND_CAP * 4) +
                           r(CAND_CAP * sizeof(Kp)) + r(CAND_CAP * sizeof(Resp)) + r((size_t)(rows + 1) * 4) +
                           r((size_t)rows * mw * 8) + r((size_t)rows * mw) +
                           (inputs_on_device ? 0 : r((size_t)width * height) + r((size_t)std::max(capmax, 1) * 32));
        const size_t shared_b = r(std::max<size_t>(tables.size(), 1) * sizeof(AxisEnt)) + r(sizeof(Lvl) * nl) +
                                r(sizeof(int) * umax.size()) + r(sizeof(ImgIO) * G) + r(sizeof(int) * CS * G);
        if (!scratch.img.reserve(device, blk * G + shared_b)) { rc = SFMX_ENOMEM; set_last_error("device allocation failed"); goto done; }
        if (!scratch.pin_reserve(device, shared_b)) { rc = SFMX_ENOMEM; set_last_error("pinned staging allocation failed"); goto done; }
        std::call_once(g_const_once[device], [] {
            int taps[7];
            blur_taps(taps);
            (void)hipMemcpyToSymbol(HIP_SYMBOL(c_taps), taps, sizeof(taps));
        });
        {
            Arena& A = scratch.img;
            uint8_t* pyr = A.take<uint8_t>(px);
            uint8_t* score = A.take<uint8_t>(px);
            uint8_t* blur = A.take<uint8_t>(px);
            int32_t* cpos = A.take<int32_t>(CAND_CAP);
            uint8_t* cscore = A.take<uint8_t>(CAND_CAP);
            Resp* rA = A.take<Resp>(CAND_CAP);
            Resp* rB = A.take<Resp>(CAND_CAP);
            int* sLs = A.take<int>(CAND_CAP);
            int* sRs = A.take<int>(CAND_CAP);
            Kp* dfin = A.take<Kp>(CAND_CAP);
            Resp* kin = A.take<Resp>(CAND_CAP);
            int* row_off = A.take<int>(rows + 1);
            uint64_t* kmask = A.take<uint64_t>((size_t)rows * mw);
            uint8_t* wcnt = A.take<uint8_t>((size_t)rows * mw);
            uint8_t* t = inputs_on_device ? nullptr : A.take<uint8_t>((size_t)width * height);
            uint8_t* ddesc = inputs_on_device ? nullptr : A.take<uint8_t>((size_t)std::max(capmax, 1) * 32);
            const int64_t istride = (int64_t)A.used;   // == blk (every part 256-B rounded)
            if ((size_t)istride != blk) { set_last_error("internal: ORB block layout"); rc = SFMX_EINTERNAL; goto done; }
            A.used = blk * G;
            AxisEnt* dtab = A.take<AxisEnt>(std::max<size_t>(tables.size(), 1));
            Lvl* dlv = A.take<Lvl>(nl);
            int* dumax = A.take<int>(umax.size());
            ImgIO* dio = A.take<ImgIO>(G);
            int* stats = A.take<int>((size_t)CS * G);
            if (A.overflow) { set_last_error("internal: ORB scratch arena too small"); rc = SFMX_ECAPACITY; goto done; }
            int* cnt1 = stats;
            int* cnt2 = stats + ST_CNT2;
            int* sst = stats + ST_TAIL;   // count, levels, corners, err
            // the chunk's small inputs through pinned staging (one copy each, no pageable staging)
            char* hp = scratch.pin;
            const size_t o_tab = 0, o_lv = o_tab + r(std::max<size_t>(tables.size(), 1) * sizeof(AxisEnt)),
                         o_um = o_lv + r(sizeof(Lvl) * nl), o_io = o_um + r(sizeof(int) * umax.size()),
                         o_st = o_io + r(sizeof(ImgIO) * G);
            if (!tables.empty()) std::memcpy(hp + o_tab, tables.data(), tables.size() * sizeof(AxisEnt));
            std::memcpy(hp + o_lv, lv.data(), sizeof(Lvl) * nl);
            std::memcpy(hp + o_um, umax.data(), sizeof(int) * umax.size());
            ImgIO* hio = reinterpret_cast<ImgIO*>(hp + o_io);
            for (int g = 0; g < G; ++g) {
                ImgIO& e = hio[g];
                e.img = inputs_on_device ? ims[g].data : t + (int64_t)g * istride;
                e.pitch = inputs_on_device ? ims[g].pitch : width;
                e.kp_out = inputs_on_device ? reinterpret_cast<Kp*>(keypoints[g]) : nullptr;
                e.desc_out = !descriptors ? nullptr : inputs_on_device ? descriptors[g] : ddesc + (int64_t)g * istride;
                e.capacity = capacities[g];
                e.pad = 0;
            }
            if (!inputs_on_device)
                for (int g = 0; g < G; ++g)
                    OCHK(hipMemcpy2DAsync(t + (int64_t)g * istride, width, ims[g].data, ims[g].pitch, width, height,
                                          hipMemcpyHostToDevice, st));
            OCHK(hipMemcpyAsync(dtab, hp, o_st, hipMemcpyHostToDevice, st));   // tables | levels | umax | ImgIO: contiguous
            OCHK(hipEventRecord(A.e0, st));
            const unsigned gz = (unsigned)G;
            // XCD order of the tile passes (xcd.hpp; A/B: SFMX_ORB_XCD_RUN, 0 = the plain grids of r04).  r05m
            // (one-stream traces, 16-image chunks): contiguous ranges per XCD cut the halo passes' counter
            // bytes 2-4x; the resize chain is unchanged (26.4 vs 26.8 us a level), the separate blur slower
            // (121 plain / 134 contiguous / 147 us runs of 8-128), FAST + NMS with the fused blur +2.5 %
            // (r05u) for 14.3 -> 3.3 MB fetched per image, rBRIEF faster (159 -> 152 us)
            int xcd = -1, xcd_blur = 0;
            if (const char* v = SFMX_DIAG_ENV("SFMX_ORB_XCD_RUN")) xcd = xcd_blur = std::atoi(v);
            // compute()'s blur inside the FAST + NMS tile pass (A/B: SFMX_ORB_BLUR_SEPARATE, r04's own pass)
            const bool fuse_blur = descriptors && capmax > 0 && !SFMX_DIAG_ENV("SFMX_ORB_BLUR_SEPARATE");
            const int xcd_brief = -1;   // rBRIEF: whole images per XCD (the working set is one image's blurred levels)
            // ---- detect(): pyramid, FAST, NMS
            orb_copy_kernel<<<dim3((width + 1023) / 1024, (height + 3) / 4, gz), 256, 0, st>>>(dio, width, height, lv[0].pitch,
                                                                                          pyr, istride);
            for (int l = 1; l < nl; l++)   // (the axis scales as linear_axis computes them)
                orb_resize_kernel<<<dim3((lv[l].w + RZ_X - 1) / RZ_X, (lv[l].h + RZ_Y - 1) / RZ_Y, gz), 256, 0, st>>>(
                    pyr, lv[l], lv[l - 1], 1.0 / ((double)lv[l].w / lv[l - 1].w), 1.0 / ((double)lv[l].h / lv[l - 1].h), dtab,
                    istride, xcd);
            orb_fast_nms_kernel<<<dim3(flat_tiles<FT_X, FT_Y>(lv), gz), 256, 0, st>>>(pyr, dlv, thr, border, score, kmask, wcnt,
                                                                                   mw, nl, istride, xcd, fuse_blur ? blur : nullptr);
            orb_scan_kernel<<<gz, 1024, 0, st>>>(wcnt, mw, rows, row_off, istride, stats, dlv, nl);
            orb_rows_kernel<<<dim3((rows + 3) / 4, gz), 256, 0, st>>>(score, dlv, nl, rows, row_off, kmask, mw, cpos, cscore,
                                                                      (int)CAND_CAP, istride);
            // retainBest(2 n_l) on the FAST scores, Harris responses, retainBest(n_l) on them (device)
            SelCounts s1{}, s2{};
            for (int l = 0; l < nl; l++) { s1.n[l] = 2 * per[l]; s2.n[l] = per[l]; }
            orb_retain_kernel<<<dim3(nl, gz), RT, 0, st>>>(0, dlv, row_off, cscore, rA, rB, sLs, sRs, nullptr, cnt1, s1,
                                                           (int)CAND_CAP, sst + 3, istride);
            // reads that may leave a level (small edgeThreshold: the bordered-pyramid instantiations)
            const bool e_h = border < 4, e_a = border < HALF_PATCH, e_b = border < BW + 1;
            if (e_h) orb_harris_kernel<true><<<dim3(64, nl, gz), 256, 0, st>>>(pyr, dlv, row_off, rA, cnt1, cpos, rB, istride);
            else orb_harris_kernel<false><<<dim3(64, nl, gz), 256, 0, st>>>(pyr, dlv, row_off, rA, cnt1, cpos, rB, istride);
            orb_retain_kernel<<<dim3(nl, gz), RT, 0, st>>>(1, dlv, row_off, cscore, rA, rB, sLs, sRs, cnt1, cnt2, s2,
                                                           (int)CAND_CAP, sst + 3, istride);
            orb_keep_kernel<<<dim3(nl, gz), RT, 0, st>>>(dlv, row_off, rA, rB, stats, cpos, width, height, border, kin,
                                                         istride);
            int* sidx = sLs;   // (the retain kernels' scratch is free from here: the processing order)
            if (SFMX_DIAG_ENV("SFMX_ORB_KEPT_ORDER")) sidx = nullptr;   // A/B: the r04 order
            if (sidx) orb_sort_kernel<<<dim3(nl, gz), RT, 0, st>>>(dlv, row_off, stats, kin, sidx, istride);
            if (e_a)
                orb_angle_kernel<true><<<dim3(G > 1 ? 256 : 1024, gz), 256, 0, st>>>(pyr, dlv, nl, row_off, rows, stats, dumax,
                                                                                    kin, sidx, dfin, istride);
            else
                orb_angle_kernel<false><<<dim3(G > 1 ? 256 : 1024, gz), 256, 0, st>>>(pyr, dlv, nl, row_off, rows, stats, dumax,
                                                                                     kin, sidx, dfin, istride);
            // ---- compute(): blur of the levels used, rBRIEF of min(count, capacity) keypoints
            if (descriptors && capmax > 0) {
                if (!fuse_blur) orb_blur_kernel<<<dim3(flat_tiles<BT_X, BT_Y>(lv), gz), 256, 0, st>>>(
                    pyr, dlv, sst, blur, nl, istride, xcd_blur);
                // rBRIEF keeps the output order, whole images per XCD (37 -> 7 MB per image, 159 -> 152 us per
                // 16 images, r05m); in the row order it read 7.6 MB but took 181 us (r05j A/B,
                // profiles/r05j_ab_orb_order.txt: it is not bandwidth-bound); the angle pass keeps the row order
                int* bsidx = SFMX_DIAG_ENV("SFMX_ORB_BRIEF_SORTED") ? sidx : nullptr;
                const dim3 bg(std::min(G > 1 ? 1024 : 4096, (capmax + 7) / 8), gz);
                if (e_b) orb_brief_kernel<true><<<bg, 256, 0, st>>>(blur, pyr, dlv, dfin, bsidx, sst, dio, istride, xcd_brief);
                else orb_brief_kernel<false><<<bg, 256, 0, st>>>(blur, pyr, dlv, dfin, bsidx, sst, dio, istride, xcd_brief);
            }
            if (inputs_on_device && capmax > 0)
                orb_copy_kp_kernel<<<dim3(std::min(1024, (capmax + 255) / 256), gz), 256, 0, st>>>(dfin, sst, dio, istride);
            OCHK(hipGetLastError());
            int* hst = reinterpret_cast<int*>(hp + o_st);
            OCHK(hipMemcpyAsync(hst, stats, sizeof(int) * CS * G, hipMemcpyDeviceToHost, st));
            OCHK(hipEventRecord(A.e1, st));
            OCHK(hipStreamSynchronize(st));
            for (int g = 0; g < G; ++g) {
                const int* s = hst + (size_t)g * CS + ST_TAIL;
                if (s[2] > CAND_CAP) { set_last_error("internal: corner buffer overflow"); rc = SFMX_EINTERNAL; goto done; }
                if (s[3]) { set_last_error("internal: device retainBest made no progress"); rc = SFMX_EINTERNAL; goto done; }
            }
            bool copies = false;
            for (int g = 0; g < G; ++g) {
                const int n = hst[(size_t)g * CS + ST_TAIL];
                n_keypoints[g] = n;
                const int m = std::min(n, (int)capacities[g]);
                if (!inputs_on_device && m > 0) {   // host buffers: the kept keypoints and descriptors back
                    OCHK(hipMemcpyAsync(keypoints[g], reinterpret_cast<const char*>(dfin) + (int64_t)g * istride,
                                        sizeof(Kp) * m, hipMemcpyDeviceToHost, st));
                    if (descriptors && descriptors[g])
                        OCHK(hipMemcpyAsync(descriptors[g], ddesc + (int64_t)g * istride, (size_t)m * 32,
                                            hipMemcpyDeviceToHost, st));
                    copies = true;
                }
                rcs[g] = n > capacities[g] ? SFMX_ECAPACITY : SFMX_OK;
            }
            if (copies) OCHK(hipStreamSynchronize(st));
            float ms = -1.f;
            (void)hipEventElapsedTime(&ms, A.e0, A.e1);
            *last_ms = ms;
        }
    done:;
        if (rc != SFMX_OK) (void)hipStreamSynchronize(st);   // nothing of this chunk in flight from the pinned staging
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
}

int orb_impl(const uint8_t* image, int32_t width, int32_t height, int64_t pitch, const sfmx_orb_params* P,
             int32_t inputs_on_device, int32_t device, void* stream, sfmx_keypoint* keypoints, uint8_t* descriptors,
             int32_t capacity, int32_t* n_keypoints, Scratch& scratch, float* last_ms) {
    if (!image || !P || !n_keypoints || capacity < 0 || (capacity > 0 && !keypoints)) {
        set_last_error("null argument");
        return SFMX_EINVAL;
    }
    const OrbImage im{image, width, height, pitch};
    sfmx_keypoint* kp[1] = {keypoints};
    uint8_t* dd[1] = {descriptors};
    int rcs[1] = {SFMX_OK};
    const int rc = orb_chunk(&im, 1, P, inputs_on_device, device, (hipStream_t)stream, kp, descriptors ? dd : nullptr,
                             &capacity, n_keypoints, rcs, scratch, last_ms);
    if (rc) return rc;
    if (rcs[0] == SFMX_ECAPACITY) set_last_error("keypoint capacity too small");
    return rcs[0];
}

struct BatchSlot {
    Scratch arena;
    hipStream_t stream = nullptr;
    int device = -1;
};
std::mutex g_batch_mu;
std::vector<std::unique_ptr<BatchSlot>> g_slots;

}  // namespace

extern "C" {

int sfmx_orb_detect_compute(const uint8_t* image, int32_t width, int32_t height, int64_t pitch,
                            const sfmx_orb_params* params, int32_t inputs_on_device, int32_t device, void* stream,
                            sfmx_keypoint* keypoints, uint8_t* descriptors, int32_t capacity, int32_t* n_keypoints) {
    return orb_impl(image, width, height, pitch, params, inputs_on_device, device, stream, keypoints, descriptors,
                    capacity, n_keypoints, g_scratch, &g_last_ms);
}

int sfmx_orb_detect_compute_batch(const sfmx_gray_image* images, int32_t n_images, const sfmx_orb_params* params,
                                  int32_t inputs_on_device, int32_t device, int32_t n_streams,
                                  sfmx_keypoint* const* keypoints, uint8_t* const* descriptors,
                                  const int32_t* capacities, int32_t* n_keypoints, int32_t* status) {
    if (n_images < 0 || (n_images > 0 && (!images || !keypoints || !capacities || !n_keypoints)) || !params) {
        set_last_error("null argument");
        return SFMX_EINVAL;
    }
    if (n_streams < 1 || n_streams > 16) { set_last_error("n_streams must be 1..16"); return SFMX_EINVAL; }
    if (n_images == 0) { g_last_ms = 0.f; return SFMX_OK; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { set_last_error("no HIP device visible"); return SFMX_EDEVICE; }
    if (device < 0 || device >= ndev) { set_last_error("device index out of range"); return SFMX_EINVAL; }
    std::lock_guard<std::mutex> lock(g_batch_mu);
    const int ns = std::min<int>(n_streams, n_images);
    while ((int)g_slots.size() < ns) g_slots.emplace_back(new BatchSlot());
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    for (int i = 0; i < ns; ++i) {
        BatchSlot& sl = *g_slots[i];
        if (sl.device != device) {
            if (sl.stream) (void)hipStreamDestroy(sl.stream);
            sl.stream = nullptr;
            if (hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess) {
                if (prev >= 0) (void)hipSetDevice(prev);
                set_last_error("hipStreamCreate failed");
                return SFMX_EDEVICE;
            }
            sl.device = device;
        }
    }
    // chunks: runs of consecutive same-size images, G <= 16 per chunk (one launch set each), spread
    // over the slots' streams; an image that fails the per-image checks is reported alone
    std::vector<int> rcs(n_images, SFMX_OK);
    std::vector<std::string> errs(n_images);
    std::vector<std::vector<int>> chunks;
    {
        // chunk size: at most 16, and the chunks a whole number of rounds over the streams (200 images on
        // 8 streams: 16 chunks of 13 rather than 13 chunks of 16, whose second round left 3 streams idle)
        const int rounds = std::max(1, (n_images + ns * 16 - 1) / (ns * 16));
        int gmax = std::max(1, std::min(16, (n_images + ns * rounds - 1) / (ns * rounds)));
        {   // a chunk reserves its per-image scratch (~19 B per pyramid pixel, ~60 B per image
            // pixel) for each of its G images on each stream: G is also cut to what 80 % of the free device
            // memory holds over the ns streams (a chunk that still fails is re-run image by image below)
            int64_t maxpx = 1;
            for (int i = 0; i < n_images; ++i)
                if (images[i].data) maxpx = std::max<int64_t>(maxpx, (int64_t)images[i].width * images[i].height);
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > 0) {
                const double per_image = 64.0 * (double)maxpx + (1 << 20);
                const double budget = 0.8 * (double)fr / ns;
                gmax = std::max(1, std::min<int>(gmax, (int)std::min(16.0, budget / per_image)));
            }
        }
        for (int i = 0; i < n_images; ++i) {
            const sfmx_gray_image& im = images[i];
            if (!im.data || capacities[i] < 0 || (capacities[i] > 0 && !keypoints[i])) {
                rcs[i] = SFMX_EINVAL;
                errs[i] = "null argument";
                continue;
            }
            if (im.width < 1 || im.height < 1 || im.pitch < im.width || im.width > 16384 || im.height > 16384) {
                rcs[i] = SFMX_EINVAL;
                errs[i] = "image size must be 1..16384 with pitch >= width";
                continue;
            }
            if (chunks.empty() || (int)chunks.back().size() >= gmax || images[chunks.back()[0]].width != im.width ||
                images[chunks.back()[0]].height != im.height)
                chunks.emplace_back();
            chunks.back().push_back(i);
        }
    }
    std::atomic<int> next{0};
    std::vector<float> kms(ns, 0.f);
    auto work = [&](int slot) {
        (void)hipSetDevice(device);
        BatchSlot& sl = *g_slots[slot];
        std::vector<OrbImage> ims;
        std::vector<sfmx_keypoint*> kp;
        std::vector<uint8_t*> dd;
        std::vector<int32_t> caps, nk;
        std::vector<int> crc;
        for (int c; (c = next.fetch_add(1)) < (int)chunks.size();) {
            const std::vector<int>& ch = chunks[c];
            const int G = (int)ch.size();
            ims.clear(); kp.clear(); dd.clear(); caps.clear();
            for (int i : ch) {
                ims.push_back(OrbImage{images[i].data, images[i].width, images[i].height, images[i].pitch});
                kp.push_back(keypoints[i]);
                dd.push_back(descriptors ? descriptors[i] : nullptr);
                caps.push_back(capacities[i]);
            }
            nk.assign(G, 0);
            crc.assign(G, SFMX_OK);
            float ms = 0.f;
            const int rc = orb_chunk(ims.data(), G, params, inputs_on_device, device, sl.stream, kp.data(),
                                     descriptors ? dd.data() : nullptr, caps.data(), nk.data(), crc.data(), sl.arena, &ms);
            if (rc != SFMX_OK && G > 1) {
                // a chunk-level failure (device memory, a launch, an internal check): the chunk's images
                // again one at a time, so each gets its own status (r03's per-image semantics)
                for (int k = 0; k < G; ++k) {
                    const int i = ch[k];
                    int32_t nk1 = 0, crc1 = SFMX_OK;
                    float ms1 = 0.f;
                    const int r1 = orb_chunk(&ims[k], 1, params, inputs_on_device, device, sl.stream, &kp[k],
                                             descriptors ? &dd[k] : nullptr, &caps[k], &nk1, &crc1, sl.arena, &ms1);
                    n_keypoints[i] = nk1;
                    rcs[i] = r1 ? r1 : crc1;
                    if (r1) errs[i] = sfmx_last_error();
                    else if (crc1 == SFMX_ECAPACITY) errs[i] = "keypoint capacity too small";
                    if (!r1) kms[slot] += ms1;
                }
                continue;
            }
            for (int k = 0; k < G; ++k) {
                const int i = ch[k];
                n_keypoints[i] = nk[k];
                rcs[i] = rc ? rc : crc[k];
                if (rc) errs[i] = sfmx_last_error();
                else if (crc[k] == SFMX_ECAPACITY) errs[i] = "keypoint capacity too small";
            }
            if (!rc) kms[slot] += ms;
        }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < ns; ++i) th.emplace_back(work, i);
    work(0);
    for (auto& t : th) t.join();
    if (prev >= 0) (void)hipSetDevice(prev);
    float total = 0.f;
    for (float k : kms) total += k;
    g_last_ms = total / n_images;
    int rc = SFMX_OK;
    for (int i = 0; i < n_images; ++i) {
        if (status) status[i] = rcs[i];
        if (rcs[i] != SFMX_OK && rc == SFMX_OK) {
            rc = rcs[i];
            set_last_error(("image " + std::to_string(i) + ": " + errs[i]).c_str());
        }
    }
    return rc;
}

}  // extern "C"
