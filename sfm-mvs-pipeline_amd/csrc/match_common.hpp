// SPDX-License-Identifier: MIT
// sfmx matcher — device data layout shared by the host driver and the kernels.
//
// HBM layout (one matcher context, one device):
//   SIFT (NORM_L2):  desc8[row][128]  int8   a' = a - 128   (exact: SIFT values are integers 0..255)
//                    norm [row]       int32  ||a'||^2        (<= 2^21)
//                    keyc [row]       int32  -(||a'||^2 << 8) + 255 - (row & 255)   (see match_kernels.hip)
//                    f32  [row][128]  float  only when an image is not integer-valued (fp32 fallback)
//   ORB (NORM_HAMMING): desc8[row][32] uint8 (rows padded with zeros)
// Images are concatenated; each starts at a row offset that is a multiple of
// ROW_ALIGN and is padded to a multiple of ROW_ALIGN rows with zero rows
// (int8 0 == descriptor value 128: contributes 0 to every dot product).
#pragma once
#include <cstdint>
#include <string>

#include <hip/hip_runtime_api.h>

namespace sfmx {

constexpr int ROW_ALIGN = 512;       // = query rows per work item = 2 x key chunk (256)
constexpr int SIFT_DIM = 128;
constexpr int ORB_BYTES = 32;
// Queries whose best-2 squared distance reaches this value take the exact
// float-sqrt slow path: below it sqrtf is injective on integers (first
// collision is at s = 4,197,201), so ranking on the integer
// s equals ranking on sqrtf(s) bits.
constexpr int64_t SQRT_SAFE = 1 << 22;

struct ImgDev {
    int32_t rows;       // real descriptor rows (Nq or Nt)
    int32_t rows_pad;   // multiple of ROW_ALIGN
    int64_t row0;       // first row in the pool
    int32_t integral;   // SIFT: 1 if all values are integers in [0,255]
    int32_t _pad;
};

struct PairDev {
    int32_t left, right;   // image indices: left = query, right = train
    int64_t dense_base;    // offset of this pair's per-query results (sum of previous Nq)
};

struct WorkItem {          // one 512-query block of one pair
    int32_t pair;
    int32_t q0;
};

struct DMatchDev { int32_t queryIdx, trainIdx, imgIdx; float distance; };

struct PrepImg {           // one image of a batched prep launch
    const float* src;
    int32_t rows, cols, rows_pad, _pad;
    int64_t row0;
};

// Overlapped two-pass matching (match_kernels.hip launch_two_pass_overlap): a batch of the work list,
// and the matcher's extra streams / events.
struct MatchBatch { int32_t w0, nw, p0, np; };   // work items [w0, w0 + nw), pair-order slots [p0, p0 + np)
struct OverlapStreams {
    hipStream_t sx, sp;                          // second screen stream, pass-2 stream
    hipEvent_t start, sx_done, sp_done;          // after the qcount clear; the two joins
    hipEvent_t* screen;                          // one per batch
};
// product default (SFMX_MATCH_BATCHES in the diagnostic build): 1 = one screen launch, then pass 2.  The
// overlapped form (8 batches, screens on two streams, pass 2 on a third) measured slower on C2 in r04a
// (launch span 6.94 vs 6.20 ms: concurrent screens and subset kernels contend for the CUs; the subset
// dispatches stretch to 0.67 ms each, profiles/r04a_c2_span.txt); kept selectable and tested.
constexpr int MATCH_BATCHES = 1;

// Thread-local last-error text shared by every C-ABI entry point (sfmx_last_error).
void set_last_error(const char* msg);

}  // namespace sfmx
