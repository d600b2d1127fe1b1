// SPDX-License-Identifier: MIT
// sfmx bundle adjustment — factorization plan (see ba_plan.hpp).
#include "ba_plan.hpp"

#include "../../include/sfmx.h"
#include "../../include/sfmx_ba.h"
#include "match_common.hpp"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <utility>

namespace sfmx {
namespace ba {
namespace {

constexpr int NBP = PLAN_NB;

// ---- nested dissection of the camera graph ----------------------------------------------
// The recursion is recorded as a tree of calls (r04): its splits do not depend on the leaf size, only
// where it stops does, so the plans of the larger leaf sizes are read off the tree of the smallest
// (derive) instead of dissecting the graph once per candidate.
struct Nd {
    const std::vector<std::vector<int>>& g;
    int leaf;                       // cameras per leaf node
    std::vector<int> in, seen, lvl, taken;
    int epoch = 0, stamp = 0;
    struct Call {
        std::vector<int> verts;     // sorted
        int kind = 0;               // 0 one node (verts), 1 connected components (kids), 2 split (kids = left, right; then sep)
        std::vector<int> kids, sep;
    };
    std::vector<Call> calls;
    Nd(const std::vector<std::vector<int>>& g_, int leaf_)
        : g(g_), leaf(leaf_), in(g_.size(), 0), seen(g_.size(), 0), lvl(g_.size(), 0), taken(g_.size(), 0) {}

    // the nodes (children before their separator) of the dissection stopping at `lf` >= leaf cameras
    void derive(int c, int lf, std::vector<std::vector<int>>& nodes) const {
        const Call& k = calls[c];
        if ((int)k.verts.size() <= lf || k.kind == 0) { nodes.push_back(k.verts); return; }
        for (int kid : k.kids) derive(kid, lf, nodes);
        if (k.kind == 2 && !k.sep.empty()) nodes.push_back(k.sep);
    }

    // BFS from root inside the current set (in == ep): level sets
    void levels(int root, int ep, std::vector<std::vector<int>>& L) {
        L.clear();
        const int s = ++stamp;
        seen[root] = s;
        lvl[root] = 0;
        L.push_back({root});
        for (;;) {
            std::vector<int> nx;
            for (int v : L.back())
                for (int w : g[v])
                    if (in[w] == ep && seen[w] != s) { seen[w] = s; lvl[w] = (int)L.size(); nx.push_back(w); }
            if (nx.empty()) break;
            std::sort(nx.begin(), nx.end());
            L.push_back(std::move(nx));
        }
    }
    int degree(int v, int ep) const {
        int d = 0;
        for (int w : g[v]) d += in[w] == ep;
        return d;
    }
    // lowest-index vertex of minimum degree in `vs`
    int min_degree(const std::vector<int>& vs, int ep) const {
        int best = vs[0], bd = degree(vs[0], ep);
        for (int v : vs) { const int d = degree(v, ep); if (d < bd) { bd = d; best = v; } }
        return best;
    }

    int rec(std::vector<int> verts) {
        std::sort(verts.begin(), verts.end());
        const int me = (int)calls.size();
        calls.emplace_back();
        calls[me].verts = verts;
        if ((int)verts.size() <= leaf) return me;
        const int ep = ++epoch;
        for (int v : verts) in[v] = ep;
        {   // connected components (each dissected on its own, no separator between them)
            std::vector<std::vector<int>> comps, L;
            for (int v : verts) {
                if (taken[v] == ep) continue;
                levels(v, ep, L);
                std::vector<int> comp;
                for (const auto& l : L)
                    for (int w : l) { taken[w] = ep; comp.push_back(w); }
                comps.push_back(std::move(comp));
            }
            if (comps.size() > 1) {
                calls[me].kind = 1;
                for (auto& c : comps) {
                    const int kid = rec(std::move(c));
                    calls[me].kids.push_back(kid);
                }
                return me;
            }
        }
        // pseudo-peripheral root: repeated BFS from the farthest minimum-degree vertex
        std::vector<std::vector<int>> L;
        int root = min_degree(verts, ep);
        levels(root, ep, L);
        for (int it = 0; it < 4; ++it) {
            const int cand = min_degree(L.back(), ep);
            std::vector<std::vector<int>> L2;
            levels(cand, ep, L2);
            if (L2.size() <= L.size()) break;
            root = cand;
            L.swap(L2);
        }
        levels(root, ep, L);   // leaves lvl[] of this BFS
        const int h = (int)L.size(), n = (int)verts.size();
        if (h < 3) return me;
        // separator level: smallest level set among the balanced ones (each side >= n/4), ties to
        // the most balanced; none balanced: the most balanced
        int m = -1;
        long best_sz = 0, best_im = 0;
        int cum = 0;
        std::vector<int> before(h, 0);
        for (int i = 0; i < h; ++i) { before[i] = cum; cum += (int)L[i].size(); }
        for (int i = 1; i + 1 < h; ++i) {
            const int lo = before[i], hi = n - before[i] - (int)L[i].size();
            if (4 * lo < n || 4 * hi < n) continue;
            const long sz = (long)L[i].size(), im = std::labs((long)lo - hi);
            if (m < 0 || sz < best_sz || (sz == best_sz && im < best_im)) { m = i; best_sz = sz; best_im = im; }
        }
        if (m < 0)
            for (int i = 1; i + 1 < h; ++i) {
                const long im = std::labs((long)before[i] - (n - before[i] - (long)L[i].size()));
                if (m < 0 || im < best_im) { m = i; best_im = im; }
            }
        std::vector<int> left, right, sep;
        for (int i = 0; i < m; ++i) left.insert(left.end(), L[i].begin(), L[i].end());
        for (int i = m + 1; i < h; ++i) right.insert(right.end(), L[i].begin(), L[i].end());
        for (int v : L[m]) {   // a separator vertex with no neighbour beyond it belongs to the near side
            bool touches = false;
            for (int w : g[v]) if (in[w] == ep && lvl[w] == m + 1) { touches = true; break; }
            (touches ? sep : left).push_back(v);
        }
        calls[me].kind = 2;
        const int kl = rec(std::move(left));
        calls[me].kids.push_back(kl);
        const int kr = rec(std::move(right));
        calls[me].kids.push_back(kr);
        std::sort(sep.begin(), sep.end());
        calls[me].sep = std::move(sep);
        return me;
    }
};

// ---- layout, pattern, schedule ------------------------------------------------------------
void layout(int C, const std::vector<std::vector<int>>& nodes, FactorPlan& P) {
    P.camrow.assign(C, 0);
    int row = 0;
    const int nn = (int)nodes.size();
    P.rowmap.clear();
    P.padrows.clear();
    for (int i = 0; i < nn; ++i) {
        const int r0 = row;
        const int used = 6 * (int)nodes[i].size();
        for (size_t j = 0; j < nodes[i].size(); ++j) {
            P.camrow[nodes[i][j]] = r0 + 6 * (int)j;
            for (int d = 0; d < 6; ++d) P.rowmap.push_back(6 * nodes[i][j] + d);
        }
        const int span = std::max(1, (used + NBP - 1) / NBP) * NBP;
        for (int r = used; r < span; ++r) { P.padrows.push_back(r0 + r); P.rowmap.push_back(-1); }
        row = r0 + span;
    }
    if (nn == 0) {   // no cameras: one identity tile keeps the launch sequence well formed
        for (int r = 0; r < NBP; ++r) { P.padrows.push_back(r); P.rowmap.push_back(-1); }
        row = NBP;
    }
    P.npad = row;
    P.T = row / NBP;
}

void pattern(const std::vector<std::vector<int>>& g, FactorPlan& P) {
    const int T = P.T, C = P.C;
    std::vector<char>& nz = P.nz;
    nz.assign((size_t)T * T, 0);
    auto mark = [&](int r0, int r1, int c0, int c1) {   // rows [r0, r1) x cols [c0, c1), lower-normalised
        for (int I = r0 / NBP; I <= (r1 - 1) / NBP; ++I)
            for (int J = c0 / NBP; J <= (c1 - 1) / NBP; ++J) nz[(size_t)std::max(I, J) * T + std::min(I, J)] = 1;
    };
    for (int I = 0; I < T; ++I) nz[(size_t)I * T + I] = 1;
    for (int a = 0; a < C; ++a) {
        mark(P.camrow[a], P.camrow[a] + 6, P.camrow[a], P.camrow[a] + 6);
        for (int b : g[a])   // (the symmetric co-visibility lists; each pair marks the same lower tile twice)
            if (b > a) mark(P.camrow[a], P.camrow[a] + 6, P.camrow[b], P.camrow[b] + 6);
    }
    // symbolic fill of the block factorization in tile order
    for (int k = 0; k < T; ++k)
        for (int a = k + 1; a < T; ++a)
            if (nz[(size_t)a * T + k])
                for (int b = k + 1; b <= a; ++b)
                    if (nz[(size_t)b * T + k]) nz[(size_t)a * T + b] = 1;
    P.tiles_nz = 0;
    for (char v : nz) P.tiles_nz += v;
}

// latency model of one launch sequence (us): per launch its slowest task
// latency model of one level launch (us, r02q kernels): a task's sources run in parallel parts
// (chol_level_split), so a task costs one source update, plus the hand-off when it has several
// (64-row tiles measured; 32-row tiles: a quarter of the tile GEMM work, two of the four sweeps)
constexpr double LAT_LAUNCH = 6.0, LAT_LOAD = NBP == 64 ? 2.5 : 1.5, LAT_UPD = NBP == 64 ? 6.5 : 2.5,
                 LAT_INV = NBP == 64 ? 12.0 : 6.0, LAT_HANDOFF = 3.0;

void schedule(FactorPlan& P) {
    const int T = P.T;
    const std::vector<char>& nz = P.nz;
    P.parent.assign(T, -1);
    P.level.assign(T, 0);
    for (int k = 0; k < T; ++k) {
        for (int a = k + 1; a < T; ++a)
            if (nz[(size_t)a * T + k]) { P.parent[k] = a; break; }
        if (P.parent[k] >= 0) P.level[P.parent[k]] = std::max(P.level[P.parent[k]], P.level[k] + 1);
    }
    P.height = 0;
    for (int k = 0; k < T; ++k) P.height = std::max(P.height, P.level[k]);
    P.leaves.clear();
    for (int k = 0; k < T; ++k) if (P.level[k] == 0) P.leaves.push_back(k);
    P.task_start.assign(1, 0);
    P.ninv.clear();
    P.tasks.clear();
    P.src.clear();
    P.predicted_us = LAT_LAUNCH + LAT_LOAD + LAT_INV;
    for (int l = 0; l < P.height; ++l) {
        std::map<std::pair<int, int>, std::vector<int>> dst;   // (a, b) -> source panels, ascending
        for (int k = 0; k < T; ++k) {
            if (P.level[k] != l) continue;
            for (int a = k + 1; a < T; ++a) {
                if (!nz[(size_t)a * T + k]) continue;
                for (int b = k + 1; b <= a; ++b)
                    if (nz[(size_t)b * T + k]) dst[{a, b}].push_back(k);
            }
        }
        std::vector<PlanTask> inv, rest;
        double worst = 0.0;
        for (auto& kv : dst) {
            const int a = kv.first.first, b = kv.first.second;
            PlanTask t{a, b, (int)P.src.size(), 0};
            P.src.insert(P.src.end(), kv.second.begin(), kv.second.end());
            t.s1 = (int)P.src.size();
            const bool iv = a == b && P.level[a] == l + 1;
            (iv ? inv : rest).push_back(t);
            worst = std::max(worst, LAT_LOAD + LAT_UPD + (kv.second.size() > 1 ? LAT_HANDOFF : 0.0) + (iv ? LAT_INV : 0.0));
        }
        P.ninv.push_back((int)inv.size());
        P.tasks.insert(P.tasks.end(), inv.begin(), inv.end());
        P.tasks.insert(P.tasks.end(), rest.begin(), rest.end());
        P.task_start.push_back((int)P.tasks.size());
        P.predicted_us += LAT_LAUNCH + worst;
    }
    // back solve: per panel i its ancestors' upper tiles (i, k), k > i with nz(k, i)
    P.bs_start.assign(T + 1, 0);
    P.bs_k.clear();
    for (int i = 0; i < T; ++i) {
        P.bs_start[i] = (int)P.bs_k.size();
        for (int k = i + 1; k < T; ++k) if (nz[(size_t)k * T + i]) P.bs_k.push_back(k);
    }
    P.bs_start[T] = (int)P.bs_k.size();
    P.lvl_start.assign(P.height + 2, 0);
    P.lvl_panels.clear();
    for (int l = 0; l <= P.height; ++l) {
        P.lvl_start[l] = (int)P.lvl_panels.size();
        for (int k = 0; k < T; ++k) if (P.level[k] == l) P.lvl_panels.push_back(k);
    }
    P.lvl_start[P.height + 1] = (int)P.lvl_panels.size();
}

void build(int C, const std::vector<std::vector<int>>& g, const std::vector<std::vector<int>>& nodes, int order,
           int leaf_tiles, FactorPlan& P) {
    P = FactorPlan{};
    P.C = C;
    P.order = order;
    P.leaf_tiles = leaf_tiles;
    layout(C, nodes, P);
    pattern(g, P);
    schedule(P);
}

}  // namespace

void make_plan(int C, const std::vector<char>& adj, int order_mode, FactorPlan& out) {
    std::vector<std::vector<int>> g(C);   // co-visibility lists (either triangle of adj)
    for (int a = 0; a < C; ++a)
        for (int b = 0; b < C; ++b)
            if (a != b && (adj[(size_t)a * C + b] || adj[(size_t)b * C + a])) g[a].push_back(b);
    std::vector<std::vector<int>> natural;
    if (C > 0) {
        natural.emplace_back(C);
        for (int c = 0; c < C; ++c) natural[0][c] = c;
    }
    FactorPlan best;
    build(C, g, natural, 0, 0, best);
    if (order_mode == 0 || C == 0) {
        out = std::move(best);
        row_masks(out, adj, out.src_mask, out.pad_panels);
        return;
    }
    const int leaves_all[3] = {1, 2, 4};
    Nd nd(g, std::max(1, leaves_all[0] * NBP / 6));   // one dissection, the smallest leaf
    {
        std::vector<int> all(C);
        for (int c = 0; c < C; ++c) all[c] = c;
        nd.rec(all);
    }
    bool have_nd = false;
    for (int li = 0; li < 3; ++li) {
        const int lt = leaves_all[li];
        if (order_mode >= 2 && order_mode - 1 != li + 1) continue;
        std::vector<std::vector<int>> nodes;
        nd.derive(0, std::max(1, lt * NBP / 6), nodes);
        FactorPlan p;
        build(C, g, nodes, 1, lt, p);
        const bool forced = order_mode >= 1;
        if ((forced && !have_nd) || p.predicted_us < best.predicted_us ||
            (p.predicted_us == best.predicted_us && p.T < best.T)) {
            best = std::move(p);
            have_nd = true;
        }
    }
    out = std::move(best);
    row_masks(out, adj, out.src_mask, out.pad_panels);   // (r06: beside the plan, e.g. on the load's plan thread)
}


// Row-level symbolic structure of the block LDL^T (r06).  Each lower tile's 64 x 64
// pattern starts from the camera co-visibility (6 x 6 camera blocks; identity padding rows: their
// diagonal only) and is filled by the plan's tasks in schedule order: an update of (a, b) from panel k
// touches the rows of a that A_ak has nonzeros in times the rows of b that A_bk has.  The masks name,
// per (task, source), the 16-row strips and 4-column chunks where A_ak / A_bk are structurally nonzero,
// and per tile the 16-row panels that are pure padding; chol_factor skips the matrix-core steps and the
// sweeps whose operands are exact zeros (identity), so the values are unchanged (up to signed zeros).
void row_masks(const FactorPlan& P, const std::vector<char>& adj, std::vector<RowMask>& src_mask,
               std::vector<int>& pad_panels) {
    const int T = P.T, C = P.C;
    static_assert(NBP == 64, "row masks are 64-bit rows of 64-row tiles");
    std::vector<int> tid((size_t)T * T, -1);
    int ntiles = 0;
    for (int a = 0; a < T; ++a)
        for (int b = 0; b <= a; ++b)
            if (P.nz[(size_t)a * T + b] || a == b) tid[(size_t)a * T + b] = ntiles++;
    std::vector<uint64_t> pat((size_t)ntiles * NBP, 0);
    // per tile: its cameras and the row mask of each (a camera's 6 rows are contiguous, padding rows
    // are -1 in rowmap): the patterns are built camera by camera (C5: 66 tiles x ~11 x ~11 camera pairs
    // instead of 66 x 64 x 64 row pairs: this runs on every plan, i.e. every SfM call whose co-visibility
    // changed)
    std::vector<std::vector<std::pair<int, uint64_t>>> tcams(T);
    for (int a = 0; a < T; ++a)
        for (int i = 0; i < NBP; ++i) {
            const int m = P.rowmap[a * NBP + i];
            if (m < 0) continue;
            const int ci = m / 6;
            if (tcams[a].empty() || tcams[a].back().first != ci) tcams[a].push_back({ci, 0});
            tcams[a].back().second |= (uint64_t)1 << i;
        }
    for (int a = 0; a < T; ++a)
        for (int b = 0; b <= a; ++b) {
            const int id = tid[(size_t)a * T + b];
            if (id < 0) continue;
            uint64_t* pt = &pat[(size_t)id * NBP];
            for (const auto& ca : tcams[a]) {
                uint64_t m = 0;
                for (const auto& cb : tcams[b])
                    if (ca.first == cb.first || adj[(size_t)ca.first * C + cb.first]) m |= cb.second;
                for (int i = 0; i < NBP; ++i)
                    if ((ca.second >> i) & 1) pt[i] = m;
            }
            if (a == b)   // identity padding rows: their diagonal only
                for (int i = 0; i < NBP; ++i)
                    if (P.rowmap[a * NBP + i] < 0) pt[i] = (uint64_t)1 << i;
        }
    auto rows_of = [&](int id) { uint64_t r = 0; for (int i = 0; i < NBP; ++i) r |= (uint64_t)(pat[(size_t)id * NBP + i] != 0) << i; return r; };
    auto cols_of = [&](int id) { uint64_t c = 0; for (int i = 0; i < NBP; ++i) c |= pat[(size_t)id * NBP + i]; return c; };
    auto strips = [](uint64_t m) { int s = 0; for (int q = 0; q < NBP / 16; ++q) s |= ((m >> (16 * q)) & 0xffffu ? 1 : 0) << q; return s; };
    auto chunks = [](uint64_t m) { int s = 0; for (int q = 0; q < NBP / 4; ++q) s |= ((m >> (4 * q)) & 0xfu ? 1 : 0) << q; return s; };
    src_mask.assign(P.src.size(), RowMask{0xf, 0xf, 0xffff, 0xffff});
    for (int l = 0; l < P.height; ++l)
        for (int t = P.task_start[l]; t < P.task_start[l + 1]; ++t) {
            const PlanTask& tk = P.tasks[t];
            const int dst = tid[(size_t)tk.a * T + tk.b];
            for (int s = tk.s0; s < tk.s1; ++s) {
                const int k = P.src[s];
                const int ia = tid[(size_t)tk.a * T + k], ib = tid[(size_t)tk.b * T + k];
                if (ia < 0 || ib < 0 || dst < 0) continue;   // (never: a source tile of a task is nonzero)
                const uint64_t ra = rows_of(ia), rb = rows_of(ib);
                src_mask[s] = RowMask{strips(ra), strips(rb), chunks(cols_of(ia)), chunks(cols_of(ib))};
                for (int i = 0; i < NBP; ++i)
                    if ((ra >> i) & 1) pat[(size_t)dst * NBP + i] |= rb;
            }
        }
    pad_panels.assign(T, 0);
    for (int a = 0; a < T; ++a)
        for (int q = 0; q < NBP / 16; ++q) {
            bool pad = true;
            for (int i = 0; i < 16; ++i) pad = pad && P.rowmap[a * NBP + 16 * q + i] < 0;
            pad_panels[a] |= (pad ? 1 : 0) << q;
        }
}

}  // namespace ba
}  // namespace sfmx

extern "C" int sfmx_ba_plan(int32_t n_cams, const uint8_t* adj, int32_t order, sfmx_ba_plan_info* info,
                            int32_t* camrow, int32_t* leaves, int32_t leaves_cap, int32_t* tasks, int32_t tasks_cap,
                            int32_t* src, int32_t src_cap) {
    if (!info || n_cams < 0 || (n_cams > 0 && !adj) || order < -1 || order > 4) {
        sfmx::set_last_error("sfmx_ba_plan: invalid arguments");
        return SFMX_EINVAL;
    }
    const int C = n_cams;
    std::vector<char> a((size_t)C * C);
    for (size_t i = 0; i < a.size(); ++i) a[i] = adj[i] != 0;
    sfmx::ba::FactorPlan p;
    sfmx::ba::make_plan(C, a, order, p);
    info->order = p.order;
    info->leaf_tiles = p.leaf_tiles;
    info->npad = p.npad;
    info->tiles = p.T;
    info->tiles_nz = p.tiles_nz;
    info->height = p.height;
    info->leaves = (int32_t)p.leaves.size();
    info->tasks = (int32_t)p.tasks.size();
    info->src = (int32_t)p.src.size();
    info->predicted_us = p.predicted_us;
    if (camrow) for (int c = 0; c < C; ++c) camrow[c] = p.camrow[c];
    if ((leaves && leaves_cap < info->leaves) || (tasks && tasks_cap < info->tasks) || (src && src_cap < info->src)) {
        sfmx::set_last_error("sfmx_ba_plan: output capacity too small");
        return SFMX_ECAPACITY;
    }
    if (leaves) for (size_t i = 0; i < p.leaves.size(); ++i) leaves[i] = p.leaves[i];
    if (src) for (size_t i = 0; i < p.src.size(); ++i) src[i] = p.src[i];
    if (tasks)
        for (int l = 0; l < p.height; ++l)
            for (int t = p.task_start[l]; t < p.task_start[l + 1]; ++t) {
                int32_t* r = tasks + 6 * (size_t)t;
                r[0] = l; r[1] = p.tasks[t].a; r[2] = p.tasks[t].b; r[3] = t - p.task_start[l] < p.ninv[l];
                r[4] = p.tasks[t].s0; r[5] = p.tasks[t].s1;
            }
    return SFMX_OK;
}
