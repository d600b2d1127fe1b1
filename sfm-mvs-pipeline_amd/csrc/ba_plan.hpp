// SPDX-License-Identifier: MIT
// sfmx bundle adjustment — factorization plan of the reduced camera system (host only).
//
// Ceres' DENSE_SCHUR (CeresUtils.cpp:43-50) factors the reduced camera matrix (6C + k unknowns)
// with a dense LLT in natural order, the shared intrinsics block last.  The solution does not
// depend on the elimination order, only its rounding does; the length of the chain of panel
// steps does.  The k intrinsics rows couple to every camera, so they are kept out of the tiles:
// the solver eliminates them last through their k x k Schur complement (a bordered system, see
// ba_chol.hpp), and the plan covers the 6C camera rows S_cc only.  It
//   1. orders the cameras by nested dissection of the camera co-visibility graph (BFS level-set
//      separators, children before separators), with every dissection node starting on a fresh
//      64-row tile (padding rows are identity rows of S_cc, zero right-hand sides);
//   2. computes the tile pattern of S and its symbolic fill, the tile elimination tree, and each
//      tile's level (leaves 0, a parent one above its highest child);
//   3. schedules block LDL^T by level: launch 0 inverts the diagonal tiles of the level-0 panels;
//      launch l + 1 applies every update from the panels of level l (one workgroup per
//      destination tile, its source panels in ascending order: fixed, deterministic) and inverts
//      the diagonal tiles of level l + 1 as soon as their last update is in.
// The ordering candidates (natural order, nested dissection with leaves of 1/2/4 tiles) are
// compared with a latency model of the schedule and the cheapest is used.  A dense camera graph
// has no separators: nested dissection then returns the natural order, a chain of T panels.
#pragma once
#include <cstdint>
#include <vector>

namespace sfmx {
namespace ba {

#ifndef SFMX_BA_NB
#define SFMX_BA_NB 64
#endif
constexpr int PLAN_NB = SFMX_BA_NB;   // tile size (== NB of the kernels, ba_kernels.hpp)

struct PlanTask { int a, b, s0, s1; };   // destination tile (a, b), a >= b; source panels src[s0 .. s1)
// Row-level zero structure of the factorization (ba_plan.cpp row_masks): per src entry (task, source k) the
// 16-row strips of A_ak (ra) and A_bk (rb) and the 4-column chunks of their columns (ka, kb) that
// can be nonzero; per tile the 16-row panels that are identity padding (bit q = rows 16q .. 16q + 15).
struct RowMask { int ra, rb, ka, kb; };

struct FactorPlan {
    int C = 0, npad = 0, T = 0, order = 0;          // order: 0 natural, 1 nested dissection
    int leaf_tiles = 0;                             // nested dissection leaf size (tiles)
    std::vector<int> camrow;                        // per camera: first of its 6 rows
    std::vector<int> rowmap;                        // per row: natural unknown 6c + d, or -1 (padding)
    std::vector<int> padrows;                       // identity rows
    std::vector<char> nz;                           // T x T lower tile pattern incl. fill
    std::vector<int> parent, level;                 // tile elimination tree, per tile
    int height = 0;                                 // max level
    std::vector<int> leaves;                        // panels of level 0 (their inverses: launch 0)
    // launch l + 1 (l = 0 .. height - 1): tasks[task_start[l] .. task_start[l + 1]); the first
    // ninv[l] of them are diagonal tiles that are inverted after their updates
    std::vector<int> task_start, ninv;
    std::vector<PlanTask> tasks;
    std::vector<int> src;
    // back solve by level, descending: per panel i the upper tiles (i, k) of its ancestors k
    // (bs_start[i] .. bs_start[i + 1] in bs_k); panels grouped by level in lvl_panels
    std::vector<int> bs_start, bs_k, lvl_start, lvl_panels;
    int tiles_nz = 0;
    double predicted_us = 0.0;
    std::vector<RowMask> src_mask;                  // per src entry (r06, row_masks; made with the plan)
    std::vector<int> pad_panels;                    // per tile
};

// adj: C x C row-major 0/1, the global camera co-visibility (symmetric; the diagonal is ignored).
// order_mode: -1 automatic (latency model), 0 natural, 1 nested dissection (leaf_tiles chosen by
// the model), 2/3/4 nested dissection with leaves of 1/2/4 tiles.
void make_plan(int C, const std::vector<char>& adj, int order_mode, FactorPlan& out);

// (computed at the end of make_plan into P.src_mask / P.pad_panels)
void row_masks(const FactorPlan& P, const std::vector<char>& adj, std::vector<RowMask>& src_mask,
               std::vector<int>& pad_panels);

}  // namespace ba
}  // namespace sfmx
