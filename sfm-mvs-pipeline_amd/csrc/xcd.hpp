// SPDX-License-Identifier: MIT
// sfmx: XCD-aware block order for tile passes (gfx950: 8 XCDs, each with its own L2).
#pragma once
#include <hip/hip_runtime.h>

namespace sfmx {

// A tile pass reads a halo around every tile.  Under round-robin dispatch (block b on XCD b % 8) the
// tiles either side of a tile run on other XCDs, whose L2s each fetch the shared lines again (from the
// MALL or HBM; FETCH_SIZE counts both).  xcd_grid remaps the grid's linear (x, y, z) block order so that
// one XCD's workgroups take neighbouring blocks: run < 0, a contiguous 1/8 of the grid per XCD; run > 0,
// runs of `run` consecutive blocks dealt to the XCDs in turn (the remainder past the last full round of
// 8 runs keeps its place); run = 0, the plain grid.  Speed only: every block still runs exactly once.
// Whether it pays is measured per pass (ORB: orb_features.hip; SIFT: sift_features.hip).
__device__ __forceinline__ void xcd_grid(int run, int& bx, int& by, int& bz) {
    bx = blockIdx.x; by = blockIdx.y; bz = blockIdx.z;
    if (!run) return;
    const int gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
    const int b = bx + gx * (by + gy * bz), x = b & 7, k = b >> 3;
    int lin = b;
    if (run < 0) {
        const int q = n >> 3, r = n & 7;
        lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
    } else if (b < n / (8 * run) * (8 * run)) {
        lin = ((k / run) * 8 + x) * run + k % run;
    }
    bx = lin % gx;
    const int t = lin / gx;
    by = t % gy;
    bz = t / gy;
}

}  // namespace sfmx
