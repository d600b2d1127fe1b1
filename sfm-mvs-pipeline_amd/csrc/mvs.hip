// SPDX-License-Identifier: MIT
// sfmx undistortion for the openMVS export, gfx950.
//
//   sfmx_undistort_images   cv::undistort(in, out, K, dist) of every recovered
//                           shot (OpenMvsUtils.cpp:142-150 -> ICamera::undistort,
//                           common/ICamera.cpp:72-80), OpenCV 4.5.1 semantics.
//
// cv::undistort works in horizontal stripes of max(1, 4096 / cols) rows.  For
// each stripe starting at row y it sets the new camera matrix's (1,2) entry to
// v0 - y, inverts it (cv::invert's 3x3 adjugate / det formula), builds the
// inverse map with initUndistortRectifyMap into CV_16SC2 + CV_16UC1 (positions
// in 1/32 px, round-half-even) and resamples with cv::remap INTER_LINEAR,
// BORDER_CONSTANT 0 (15-bit fixed-point bilinear weights).
//
// For the camera matrices the reference produces (zero skew, K[3] = K[6] =
// K[7] = 0, K[8] = 1) the inverse has ir[1] = ir[3] = ir[6] = ir[7] = 0 and
// ir[0], ir[2], ir[8] do not depend on the stripe, so the running sum
// `_x += ir[0]` of initUndistortRectifyMap's inner loop is the same sequence
// for every row: it is summed once per image on the host (in the same order)
// and read as a column table.  Everything per row (ir[5], 1/_w, y) and per
// pixel (the distortion polynomial, the fixed-point map, the bilinear sum) is
// recomputed here in the reference's operation order; the file is built with
// -ffp-contract=off so no a*b+c is fused.  Result: bit-identical to the
// restatement in oracle/mvs_oracle.cpp.
//
// Byte work: HBM-bound.  Algorithmic bytes per output pixel = 2 * channels
// (the source read once, the destination written once).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <array>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/sfmx_mvs.h"
#include "match_common.hpp"

namespace sfmx {
namespace mvs {

constexpr int PX_PER_THREAD = 4;

// global (not flat) address space: the image pointers come out of a descriptor in
// memory, so the compiler cannot infer it and would emit flat_load/flat_store
#define GPTR(T) __attribute__((address_space(1))) T*
#define CGPTR(T) const __attribute__((address_space(1))) T*
constexpr int THREADS = 256;
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int PX_PER_BLOCK = PX_PER_THREAD * THREADS;

struct UndImg {
    const uint8_t* src;
    uint8_t* dst;
    int64_t src_pitch, dst_pitch;
    const double2* xcol;     // per column: x = _x * (1/_w) and x*x (_x: initUndistortRectifyMap's running sum)
    int64_t blk0;            // first block of this image in the launch
    int32_t W, H, C, stripe0;
    int32_t bpr;             // blocks per row
    int32_t dst_words;       // 1: dst rows and base are 4-byte aligned (dword stores)
    int32_t src_words;       // 1: src rows and base are 4-byte aligned and W >= 2 (dword tap loads)
    int32_t radial;          // 1: p1 = p2 = k3 = 0 (SimpleRadialCamera): the zero terms drop out exactly
    int32_t mpitch;          // map row pitch in pixels (bpr * PX_PER_BLOCK) when `map` is set
    const int2* map;         // shared inverse map (iu, iv) of this image's unit, or null: computed per pixel
    double w;                // 1/_w = 1/ir[8]
    double t0, t2;           // ir[0], ir[2]
    double K0, K5, d, t4, t8;
    double fx, fy, u0, v0, k1, k2, p1, p2, k3;
};

// A run of launch blocks: g images whose blocks are interleaved image-fastest
// (block rb -> image first + rb % g, row block rb / g), so images that share one
// inverse map (same size, K and distortion -- the reference's toOpenMVS export:
// one camera for every shot) read each map tile g times while it sits in L2.
struct UndUnit {
    int64_t blk0;            // first block of the unit in the launch
    int32_t first, g;        // image range [first, first + g) of the launch's image array
};

// cvRound of a double on x86 (cvtsd2si): round half to even, and the
// "integer indefinite" INT_MIN for NaN / out of range.
__device__ __forceinline__ int cv_round(double v) {
    const double r = rint(v);
    if (!(r >= -2147483648.0 && r <= 2147483647.0)) return INT_MIN;
    return (int)r;
}

// The two horizontal taps (bx, bx + 1) of one source row, as two packed C-byte
// values.  WORDS: one aligned 2- or 3-dword load covering both pixels and a byte
// funnel shift (v_alignbyte); it may read up to 8 bytes past the last row, which
// the host checks against the allocation (else the image takes the byte path).
template <int C, bool WORDS>
__device__ __forceinline__ void fetch_taps(CGPTR(uint8_t) row, int bx, bool two, uint32_t& t0, uint32_t& t1) {
    const int o = bx * C;
    if constexpr (WORDS) {
        const int oa = o & ~3, sh = o & 3;
        CGPTR(uint32_t) p = reinterpret_cast<CGPTR(uint32_t)>(row + oa);
        if constexpr (C == 3) {
            const uint32_t a = p[0], b = p[1], c = p[2];
            const uint32_t lo = __builtin_amdgcn_alignbyte(b, a, sh), hi = __builtin_amdgcn_alignbyte(c, b, sh);
            t0 = lo & 0xFFFFFFu;
            t1 = (lo >> 24) | ((hi & 0xFFFFu) << 8);
        } else {
            const uint32_t a = p[0], b = p[1];
            if constexpr (C == 4) {
                t0 = a;
                t1 = b;
            } else {
                const uint32_t lo = __builtin_amdgcn_alignbyte(b, a, sh);
                t0 = lo & ((1u << (8 * C)) - 1);
                t1 = (lo >> (8 * C)) & ((1u << (8 * C)) - 1);
            }
        }
    } else {
        t0 = t1 = 0;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            t0 |= (uint32_t)row[o + c] << (8 * c);
            if (two) t1 |= (uint32_t)row[o + C + c] << (8 * c);
        }
    }
}

// initUndistortRectifyMap for PX_PER_THREAD consecutive pixels of row Y (columns
// past the last one repeat it): source position in 1/32 px, as cvRound gives it.
__device__ __forceinline__ void map4(const UndImg& im, int Y, int x0, int (&iu)[PX_PER_THREAD], int (&iv)[PX_PER_THREAD]) {
    // per row: the stripe's inverse (cv::invert adjugate; see header comment)
    const int ys = (Y / im.stripe0) * im.stripe0;
    const int i = Y - ys;
    const double m12 = im.K5 - (double)ys;                 // Ar(1,2) = v0 - y
    const double t5 = (0.0 - im.K0 * m12) * im.d;           // (a02*a10 - a00*a12) * d
    const double yr = ((double)i * im.t4 + t5);             // _y = i*ir[4] + ir[5]
    const double y = yr * im.w;                             // w = 1/_w, _w = i*ir[7] + ir[8] = ir[8]
    const double y2 = y * y;

    const int W = im.W;
    CGPTR(double) xc = (CGPTR(double))im.xcol;
    const bool radial = im.radial;
#pragma unroll
    for (int p = 0; p < PX_PER_THREAD; ++p) {
        const int j = min(x0 + p, W - 1);
        const double x = xc[2 * j], x2 = xc[2 * j + 1];
        const double r2 = x2 + y2;
        double u, v;
        if (radial) {
            // k3 = 0: (0*r2 + k2) == k2; p1 = p2 = 0: the tangential terms are +-0 and
            // x*kr + +-0 can only differ from x*kr in the sign of a zero, which
            // fx*xd + u0 and the rounding below cannot see
            const double kr = 1 + (im.k2 * r2 + im.k1) * r2;
            u = im.fx * (x * kr) + im.u0;
            v = im.fy * (y * kr) + im.v0;
        } else {
            const double _2xy = 2 * x * y;
            const double kr = 1 + ((im.k3 * r2 + im.k2) * r2 + im.k1) * r2;   // / (1 + 0) == exact
            const double xd = x * kr + im.p1 * _2xy + im.p2 * (r2 + 2 * x2);
            const double yd = y * kr + im.p1 * (r2 + 2 * y2) + im.p2 * _2xy;
            u = im.fx * xd + im.u0;
            v = im.fy * yd + im.v0;
        }
        iu[p] = cv_round(u * 32);
        iv[p] = cv_round(v * 32);
    }
}

// One thread: PX_PER_THREAD consecutive pixels of row Y.  Three phases so the
// tap loads of all pixels are in flight together: (1) the inverse map of every
// pixel in fp64, (2) the 2 x PX tap-pair loads, (3) the fixed-point blends.
template <int C, bool WORDS, bool MAPPED>
__device__ __forceinline__ void undistort_px(const UndImg& im, int Y, int x0) {
    const int W = im.W, H = im.H;
    CGPTR(uint8_t) S = (CGPTR(uint8_t))im.src;
    const unsigned sp = (unsigned)im.src_pitch;

    // (1) map: source position in 1/32 px -- from the unit's shared map, or computed here
    int iu[PX_PER_THREAD], iv[PX_PER_THREAD];
    if constexpr (MAPPED) {
        CGPTR(i32x4) m = (CGPTR(i32x4))(im.map + (int64_t)Y * im.mpitch + x0);
        static_assert(PX_PER_THREAD == 4, "two 16-byte map loads per thread");
        const i32x4 m0 = m[0], m1 = m[1];
        iu[0] = m0.x; iv[0] = m0.y; iu[1] = m0.z; iv[1] = m0.w;
        iu[2] = m1.x; iv[2] = m1.y; iu[3] = m1.z; iv[3] = m1.w;
    } else {
        map4(im, Y, x0, iu, iv);
    }
    // Interior threads (every pixel's four taps inside the image -- all but the
    // border bands of a photo) skip the clamps, the tap-validity weights and the
    // border tap selection; the general path below handles the rest.  In the
    // interior the two paths compute the same sums term for term, except that
    // the saturated w0 (a = bb = 0) is left at 32768: its taps' other weights are
    // 0, so s = p*32768 vs p*32767 and (s + 16384) >> 15 = p either way (p <= 255).
    bool interior = W >= 2 && H >= 2;
#pragma unroll
    for (int p = 0; p < PX_PER_THREAD; ++p) {
        const int sx = (int)(short)(iu[p] >> 5), sy = (int)(short)(iv[p] >> 5);
        interior = interior && (unsigned)sx <= (unsigned)(W - 2) && (unsigned)sy <= (unsigned)(H - 2);
    }
    uint32_t out[C];                                        // 4 px x C bytes, packed
#pragma unroll
    for (int k = 0; k < C; ++k) out[k] = 0;
    if (interior) {
        uint32_t ta0[PX_PER_THREAD], ta1[PX_PER_THREAD], tb0[PX_PER_THREAD], tb1[PX_PER_THREAD];
#pragma unroll
        for (int p = 0; p < PX_PER_THREAD; ++p) {
            const int sx = (int)(short)(iu[p] >> 5), sy = (int)(short)(iv[p] >> 5);
            CGPTR(uint8_t) r0 = S + __umul24((unsigned)sy, sp);
            fetch_taps<C, WORDS>(r0, sx, true, ta0[p], ta1[p]);
            fetch_taps<C, WORDS>(r0 + sp, sx, true, tb0[p], tb1[p]);
        }
#pragma unroll
        for (int p = 0; p < PX_PER_THREAD; ++p) {
            const int a = iu[p] & 31, bb = iv[p] & 31;
            const int w0 = (32 - bb) * (32 - a) * 32, w1 = (32 - bb) * a * 32;
            const int w2 = bb * (32 - a) * 32, w3 = bb * a * 32;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int s = (int)((ta0[p] >> (8 * c)) & 255) * w0 + (int)((ta1[p] >> (8 * c)) & 255) * w1 +
                              (int)((tb0[p] >> (8 * c)) & 255) * w2 + (int)((tb1[p] >> (8 * c)) & 255) * w3;
                const uint32_t o = (uint32_t)((s + 16384) >> 15);
                const int byte = p * C + c;
                out[byte >> 2] |= o << (8 * (byte & 3));
            }
        }
    } else {
        // (2) taps.  Both taps of a row come from the pixel pair (bx, bx + 1), bx
        // clamped into [0, W - 2]; at the borders the in-image tap is the pair's
        // first (sx = -1) or second (sx = W - 1) pixel, the other tap weighs 0.
        uint32_t ta0[PX_PER_THREAD], ta1[PX_PER_THREAD], tb0[PX_PER_THREAD], tb1[PX_PER_THREAD];
#pragma unroll
        for (int p = 0; p < PX_PER_THREAD; ++p) {
            const int sx = (int)(short)(iu[p] >> 5), sy = (int)(short)(iv[p] >> 5);
            const int bx = W >= 2 ? min(max(sx, 0), W - 2) : 0;
            const unsigned cy0 = (unsigned)min(max(sy, 0), H - 1), cy1 = (unsigned)min(max(sy + 1, 0), H - 1);
            // row offsets: cy < 2^15 and pitch < 2^24 (checked on the host) -> 24-bit multiplies
            fetch_taps<C, WORDS>(S + __umul24(cy0, sp), bx, W >= 2, ta0[p], ta1[p]);
            fetch_taps<C, WORDS>(S + __umul24(cy1, sp), bx, W >= 2, tb0[p], tb1[p]);
        }
        // (3) blend: cv::remap INTER_LINEAR, 15-bit weights, BORDER_CONSTANT 0
#pragma unroll
        for (int p = 0; p < PX_PER_THREAD; ++p) {
            const int sx = (int)(short)(iu[p] >> 5), sy = (int)(short)(iv[p] >> 5);
            const int a = iu[p] & 31, bb = iv[p] & 31;
            const bool x0in = (unsigned)sx < (unsigned)W, x1in = (unsigned)(sx + 1) < (unsigned)W;
            const bool y0in = (unsigned)sy < (unsigned)H, y1in = (unsigned)(sy + 1) < (unsigned)H;
            int w0 = (32 - bb) * (32 - a) * 32;
            if (w0 == 32768) w0 = 32767;                        // saturate_cast<short> of the table entry
            w0 = (y0in && x0in) ? w0 : 0;
            const int w1 = (y0in && x1in) ? (32 - bb) * a * 32 : 0;
            const int w2 = (y1in && x0in) ? bb * (32 - a) * 32 : 0;
            const int w3 = (y1in && x1in) ? bb * a * 32 : 0;
            uint32_t a0 = ta0[p], a1 = ta1[p], b0 = tb0[p], b1 = tb1[p];
            if (W == 1) { a1 = a0; b1 = b0; }
            const bool first_is_t1 = sx < 0, second_is_t0 = sx >= W - 1;
            const uint32_t p00 = second_is_t0 ? a1 : a0, p01 = first_is_t1 ? a0 : a1;
            const uint32_t p10 = second_is_t0 ? b1 : b0, p11 = first_is_t1 ? b0 : b1;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int s = (int)((p00 >> (8 * c)) & 255) * w0 + (int)((p01 >> (8 * c)) & 255) * w1 +
                              (int)((p10 >> (8 * c)) & 255) * w2 + (int)((p11 >> (8 * c)) & 255) * w3;
                const uint32_t o = (uint32_t)((s + 16384) >> 15);   // 0 <= s <= 255 * 32768: no saturation needed
                const int byte = p * C + c;                     // compile-time after unrolling
                out[byte >> 2] |= o << (8 * (byte & 3));
            }
        }
    }
    const int npx = min(PX_PER_THREAD, W - x0);
    GPTR(uint8_t) D = (GPTR(uint8_t))im.dst + (int64_t)Y * im.dst_pitch + (int64_t)x0 * C;
    if (im.dst_words && npx == PX_PER_THREAD) {             // 4 px * C bytes = C dwords, 4-aligned
        GPTR(uint32_t) Dw = reinterpret_cast<GPTR(uint32_t)>(D);
#pragma unroll
        for (int k = 0; k < C; ++k) Dw[k] = out[k];
    } else {
        for (int k = 0; k < npx * C; ++k) D[k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
    }
}

// Logical block of a launch: hardware dispatches block b to XCD b % 8; give every
// XCD a contiguous run of logical blocks so neighbouring blocks share its L2.
__device__ __forceinline__ int xcd_block(int n_blocks) {
    const int b = blockIdx.x;
    const int q = n_blocks / 8, r = n_blocks % 8;
    const int xcd = b % 8, idx = b / 8;
    return xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
}

__device__ __forceinline__ int find_unit(const UndUnit* __restrict__ units, int n_units, int lb) {
    int lo = 0, hi = n_units - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (units[mid].blk0 <= lb) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <int C>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(C == 1 ? 1 : 8)))  // C >= 2: <= 64 VGPRs, 8 waves/SIMD
void undistort_kernel(const UndUnit* __restrict__ units, int n_units, const UndImg* __restrict__ imgs, int n_blocks) {
    const int lb = xcd_block(n_blocks);
    const UndUnit& u = units[find_unit(units, n_units, lb)];
    const int rb = lb - (int)u.blk0;
    const int rest = rb / u.g;
    const UndImg& im = imgs[u.first + (rb - rest * u.g)];
    const int Y = rest / im.bpr;
    const int x0 = (rest - Y * im.bpr) * PX_PER_BLOCK + (int)threadIdx.x * PX_PER_THREAD;
    if (Y >= im.H || x0 >= im.W) return;
    if (im.map) {
        if (im.src_words) undistort_px<C, true, true>(im, Y, x0);
        else undistort_px<C, false, true>(im, Y, x0);
    } else {
        if (im.src_words) undistort_px<C, true, false>(im, Y, x0);
        else undistort_px<C, false, false>(im, Y, x0);
    }
}

// The shared inverse map of every unit with g >= 2, from its first image: (iu, iv)
// per pixel, rows padded to mpitch with the last column repeated (map4 clamps).
// units[k].first = that image; g = 1.
__global__ __launch_bounds__(THREADS)
void map_kernel(const UndUnit* __restrict__ units, int n_units, const UndImg* __restrict__ imgs, int n_blocks) {
    const int lb = xcd_block(n_blocks);
    const UndUnit& u = units[find_unit(units, n_units, lb)];
    const UndImg& im = imgs[u.first];
    const int rb = lb - (int)u.blk0;
    const int Y = rb / im.bpr;
    const int x0 = (rb - Y * im.bpr) * PX_PER_BLOCK + (int)threadIdx.x * PX_PER_THREAD;
    if (Y >= im.H) return;
    int iu[PX_PER_THREAD], iv[PX_PER_THREAD];
    map4(im, Y, x0, iu, iv);
    GPTR(i32x4) m = (GPTR(i32x4))(const_cast<int2*>(im.map) + (int64_t)Y * im.mpitch + x0);
    m[0] = i32x4{iu[0], iv[0], iu[1], iv[1]};
    m[1] = i32x4{iu[2], iv[2], iu[3], iv[3]};
}

// initUndistortRectifyMap's running sum _x += ir[0] (from _x = ir[2]) and the
// row-invariant x = _x * (1/_w), x*x, for one image: sequential as in the
// reference loop.  Host code: one dependent fp64 add per column is a few
// microseconds on a CPU core (and ~25 ns per column as a single GPU lane); IEEE
// binary64 add/mul round identically on both, and no a*b+c here can fuse.
static void xcol_table(const UndImg& u, double2* xc) {
    double xs = 0.0 + u.t2;
    for (int j = 0; j < u.W; ++j, xs += u.t0) {
        const double x = xs * u.w;
        xc[j] = make_double2(x, x * x);
    }
}

thread_local float g_last_ms = -1.f;

// per-thread device scratch (descriptors + column tables) and timing events,
// grown on demand and kept across calls
struct Scratch {
    int dev = -1;
    void* p = nullptr;
    size_t cap = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    void* get(int device, size_t bytes) {
        if (dev != device) {   // free the old device's buffer and events on that device first
            if (dev >= 0) {
                int prev = -1;
                (void)hipGetDevice(&prev);
                (void)hipSetDevice(dev);
                if (p) (void)hipFree(p);
                if (e0) (void)hipEventDestroy(e0);
                if (e1) (void)hipEventDestroy(e1);
                if (prev >= 0) (void)hipSetDevice(prev);
            }
            p = nullptr; cap = 0; e0 = e1 = nullptr; dev = device;
        }
        if (bytes > cap) {
            if (p) (void)hipFree(p);
            p = nullptr;
            cap = 0;
            if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
            cap = bytes;
        }
        if (!e0 && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) return nullptr;
        return p;
    }
};
thread_local Scratch g_scratch;

bool is_gfx950(int device) {
    static std::atomic<int> state[64];   // 0 unknown, 1 yes, 2 no
    if (device < 0 || device >= 64) return false;
    int v = state[device].load();
    if (v == 0) {
        hipDeviceProp_t prop;
        v = (hipGetDeviceProperties(&prop, device) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) ? 1 : 2;
        state[device].store(v);
    }
    return v == 1;
}

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

}  // namespace mvs
}  // namespace sfmx

using namespace sfmx;
using namespace sfmx::mvs;

#define UCHK(expr) do { if ((expr) != hipSuccess) { rc = SFMX_EDEVICE; set_last_error("HIP error in " #expr); goto done; } } while (0)

extern "C" {

float sfmx_undistort_last_kernel_ms(void) { return g_last_ms; }

int sfmx_undistort_images(const sfmx_undistort_image* images, int32_t n_images, int32_t inputs_on_device,
                          int32_t device, void* stream) {
    if (n_images < 0 || (n_images && !images)) { set_last_error("bad image list"); return SFMX_EINVAL; }
    for (int n = 0; n < n_images; ++n) {
        const sfmx_undistort_image& g = images[n];
        if (!g.src || !g.dst || g.src == g.dst) { set_last_error("null or aliased image buffer"); return SFMX_EINVAL; }
        if (g.width <= 0 || g.height <= 0 || g.width >= 32767 || g.height >= 32767) {
            set_last_error("image size outside (0, 32767)");
            return SFMX_EINVAL;
        }
        if (g.channels < 1 || g.channels > 4) { set_last_error("channels must be 1..4"); return SFMX_EINVAL; }
        if (g.src_pitch < (int64_t)g.width * g.channels || g.dst_pitch < (int64_t)g.width * g.channels) {
            set_last_error("pitch smaller than a row");
            return SFMX_EINVAL;
        }
        if (g.src_pitch >= (1 << 24)) { set_last_error("source pitch must be < 16 MiB"); return SFMX_EINVAL; }
        if (g.K[1] != 0 || g.K[3] != 0 || g.K[6] != 0 || g.K[7] != 0 || g.K[8] != 1) {
            set_last_error("camera matrix must be [fx 0 cx; 0 fy cy; 0 0 1] (ICamera::getK)");
            return SFMX_EINVAL;
        }
        if (!(g.K[0] * g.K[4] != 0) || !std::isfinite(g.K[0] * g.K[4])) {
            set_last_error("singular camera matrix");
            return SFMX_EINVAL;
        }
    }
    if (n_images == 0) return SFMX_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { set_last_error("no HIP device visible"); return SFMX_EDEVICE; }
    if (device < 0 || device >= ndev) { set_last_error("device index out of range"); return SFMX_EINVAL; }
    if (!is_gfx950(device)) { set_last_error("sfmx kernels are built for gfx950 only"); return SFMX_EDEVICE; }
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    const hipStream_t st = (hipStream_t)stream;
    int rc = SFMX_OK;
    {
        Bufs b;   // host-mode staging only
        std::vector<UndImg> h(n_images);
        std::vector<uint8_t*> staged_dst(n_images);
        for (int n = 0; n < n_images; ++n) {
            const sfmx_undistort_image& g = images[n];
            UndImg& u = h[n];
            u.W = g.width; u.H = g.height; u.C = g.channels;
            u.stripe0 = std::min(std::max(1, (1 << 12) / std::max(g.width, 1)), g.height);
            u.bpr = (g.width + PX_PER_BLOCK - 1) / PX_PER_BLOCK;
            // cv::invert (3x3, DECOMP_LU) of the stripe's new camera matrix: det3 and
            // the adjugate rows that do not depend on the stripe (header comment)
            const double K0 = g.K[0], K2 = g.K[2], K4 = g.K[4];
            const double det = K0 * K4;
            const double d = 1. / det;
            const double t0 = K4 * d, t2 = (0.0 - K2 * K4) * d;
            u.K0 = K0; u.K5 = g.K[5]; u.d = d;
            u.t4 = K0 * d; u.t8 = det * d;
            u.fx = K0; u.fy = K4; u.u0 = K2; u.v0 = g.K[5];
            u.k1 = g.dist[0]; u.k2 = g.dist[1]; u.p1 = g.dist[2]; u.p2 = g.dist[3]; u.k3 = g.dist[4];
            u.w = 1. / u.t8;                                       // 1/_w, the same for every row
            u.t0 = t0; u.t2 = t2;                                  // column table: xcol_table
            u.radial = (g.dist[2] == 0 && g.dist[3] == 0 && g.dist[4] == 0) ? 1 : 0;
            u.mpitch = u.bpr * PX_PER_BLOCK;
            u.map = nullptr;
            u.xcol = nullptr;
            u.blk0 = 0;                                            // unused by the kernels (units carry it)
            u.src_pitch = g.src_pitch; u.dst_pitch = g.dst_pitch;
            u.src = g.src; u.dst = g.dst;
        }
        if (!inputs_on_device) {   // stage every image on the device, packed rows
            for (int n = 0; n < n_images; ++n) {
                const sfmx_undistort_image& g = images[n];
                const int64_t row = (int64_t)g.width * g.channels;
                auto* s = static_cast<uint8_t*>(b.alloc(row * g.height + 16));   // + overread pad
                auto* o = static_cast<uint8_t*>(b.alloc(row * g.height));
                if (!s || !o) { rc = SFMX_ENOMEM; goto done; }
                UCHK(hipMemcpy2DAsync(s, row, g.src, g.src_pitch, row, g.height, hipMemcpyHostToDevice, st));
                h[n].src = s; h[n].dst = o;
                h[n].src_pitch = h[n].dst_pitch = row;
            }
        }
        for (UndImg& u : h)
            u.dst_words = ((uintptr_t)u.dst % 4 == 0 && u.dst_pitch % 4 == 0) ? 1 : 0;
        for (UndImg& u : h) {
            // dword tap loads read up to 8 bytes past the last row: allowed only when the
            // allocation holding the image extends that far (host-staged copies are padded)
            bool safe = false;
            hipDeviceptr_t base = nullptr;
            size_t range = 0;
            if (hipMemGetAddressRange(&base, &range, (hipDeviceptr_t)u.src) == hipSuccess && base) {
                const uintptr_t end = (uintptr_t)u.src + (uintptr_t)(u.H - 1) * u.src_pitch + (uintptr_t)u.W * u.C + 8;
                safe = end <= (uintptr_t)base + range;
            }
            (void)hipGetLastError();
            u.src_words = (safe && (uintptr_t)u.src % 4 == 0 && u.src_pitch % 4 == 0 && u.W >= 2) ? 1 : 0;
        }
        for (int n = 0; n < n_images; ++n) staged_dst[n] = h[n].dst;
        {
            // Launch order: by channel count (one launch each, the kernel is specialised
            // on it), then by the inputs of the inverse map (size, K, distortion), so
            // images sharing a map are adjacent and form one unit.
            // bitwise key: a total order, and equal keys = identical maps
            auto key = [](const UndImg& u) {
                std::array<uint64_t, 12> k{(uint64_t)u.C, (uint64_t)u.W, (uint64_t)u.H};
                const double v[9] = {u.fx, u.fy, u.u0, u.v0, u.k1, u.k2, u.p1, u.p2, u.k3};
                std::memcpy(k.data() + 3, v, sizeof v);
                return k;
            };
            auto same_map = [&](const UndImg& p, const UndImg& q) { return key(p) == key(q); };
            std::stable_sort(h.begin(), h.end(), [&](const UndImg& p, const UndImg& q) { return key(p) < key(q); });
            std::vector<UndUnit> units, maps;                     // units: per C contiguous; maps: g >= 2 units
            int ufirst_c[5] = {0, 0, 0, 0, 0}, ucnt_c[5] = {0, 0, 0, 0, 0};
            int64_t blk_c[5] = {0, 0, 0, 0, 0}, map_blocks = 0, map_bytes = 0;
            std::vector<int64_t> map_off;                         // per maps entry: byte offset in the map area
            for (int n = 0; n < n_images;) {
                int e = n + 1;
                while (e < n_images && same_map(h[n], h[e])) ++e;
                const int c = h[n].C;
                if (ucnt_c[c] == 0) ufirst_c[c] = (int)units.size();
                ucnt_c[c]++;
                const int64_t blocks = (int64_t)h[n].bpr * h[n].H;
                units.push_back(UndUnit{blk_c[c], n, e - n});
                blk_c[c] += blocks * (e - n);
                if (e - n >= 2) {
                    maps.push_back(UndUnit{map_blocks, n, 1});
                    map_off.push_back(map_bytes);
                    map_blocks += blocks;
                    map_bytes += ((int64_t)h[n].mpitch * h[n].H * (int64_t)sizeof(int2) + 255) & ~(int64_t)255;
                }
                n = e;
            }
            for (int c = 1; c <= 4; ++c)
                if (blk_c[c] >= (int64_t)INT32_MAX) { set_last_error("images too large for one launch"); rc = SFMX_EINVAL; goto done; }
            if (map_blocks >= (int64_t)INT32_MAX) { set_last_error("images too large for one launch"); rc = SFMX_EINVAL; goto done; }
            // device scratch: descriptors | units | map jobs | column tables | maps
            auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
            const size_t o_units = al(sizeof(UndImg) * n_images);
            const size_t o_maps = o_units + al(sizeof(UndUnit) * units.size());
            std::vector<int> need;                                // images whose map is computed from xcol
            for (const UndUnit& q : units) need.push_back(q.first);   // singleton, or the map's source
            const size_t o_col = o_maps + al(sizeof(UndUnit) * std::max<size_t>(maps.size(), 1));
            int64_t ncol_need = 0;
            for (int i : need) ncol_need += h[i].W;
            const size_t o_map = o_col + al(sizeof(double2) * ncol_need);
            auto* scratch = static_cast<uint8_t*>(g_scratch.get(device, o_map + (size_t)map_bytes));
            if (!scratch) { rc = SFMX_ENOMEM; goto done; }
            auto* dimg = reinterpret_cast<UndImg*>(scratch);
            auto* dunits = reinterpret_cast<UndUnit*>(scratch + o_units);
            auto* dmaps = reinterpret_cast<UndUnit*>(scratch + o_maps);
            auto* dcol = reinterpret_cast<double2*>(scratch + o_col);
            std::vector<uint8_t> blob(o_map);
            {
                int64_t co = 0;
                for (int i : need) {
                    h[i].xcol = dcol + co;                     // the unit's other images never read it
                    xcol_table(h[i], reinterpret_cast<double2*>(blob.data() + o_col) + co);
                    co += h[i].W;
                }
            }
            for (size_t k = 0; k < maps.size(); ++k) {
                const UndUnit& m = maps[k];
                const UndUnit* un = nullptr;
                for (const UndUnit& q : units) if (q.first == m.first) { un = &q; break; }
                auto* mp = reinterpret_cast<int2*>(scratch + o_map + map_off[k]);
                for (int i = un->first; i < un->first + un->g; ++i) h[i].map = mp;
            }
            std::memcpy(blob.data(), h.data(), sizeof(UndImg) * n_images);
            std::memcpy(blob.data() + o_units, units.data(), sizeof(UndUnit) * units.size());
            if (!maps.empty()) std::memcpy(blob.data() + o_maps, maps.data(), sizeof(UndUnit) * maps.size());
            UCHK(hipMemcpyAsync(scratch, blob.data(), o_map, hipMemcpyHostToDevice, st));
            hipEvent_t e0 = g_scratch.e0, e1 = g_scratch.e1;
            UCHK(hipEventRecord(e0, st));
            if (map_blocks)
                map_kernel<<<(unsigned)map_blocks, THREADS, 0, st>>>(dmaps, (int)maps.size(), dimg, (int)map_blocks);
            for (int c = 1; c <= 4; ++c) {
                if (ucnt_c[c] == 0) continue;
                const int nb = (int)blk_c[c];
                const UndUnit* du = dunits + ufirst_c[c];
                if (c == 1) undistort_kernel<1><<<(unsigned)nb, THREADS, 0, st>>>(du, ucnt_c[c], dimg, nb);
                if (c == 2) undistort_kernel<2><<<(unsigned)nb, THREADS, 0, st>>>(du, ucnt_c[c], dimg, nb);
                if (c == 3) undistort_kernel<3><<<(unsigned)nb, THREADS, 0, st>>>(du, ucnt_c[c], dimg, nb);
                if (c == 4) undistort_kernel<4><<<(unsigned)nb, THREADS, 0, st>>>(du, ucnt_c[c], dimg, nb);
                UCHK(hipGetLastError());
            }
            UCHK(hipEventRecord(e1, st));
            if (!inputs_on_device)
                for (int n = 0; n < n_images; ++n) {
                    const sfmx_undistort_image& g = images[n];
                    const int64_t row = (int64_t)g.width * g.channels;
                    UCHK(hipMemcpy2DAsync(g.dst, g.dst_pitch, staged_dst[n], row, row, g.height, hipMemcpyDeviceToHost, st));
                }
            UCHK(hipStreamSynchronize(st));
            float ms = -1.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            g_last_ms = ms;
        }
    done:;
    }
    if (rc == SFMX_ENOMEM) set_last_error("device allocation failed");
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
}

}  // extern "C"
