"""Factorization plan of the reduced camera system (host only, sfmx_ba_plan): the nested
dissection ordering + level schedule that the GPU solve (ba_chol.hpp) executes, checked by
executing the schedule in numpy on random SPD systems with the plan's tile pattern and
comparing with a dense solve.  The reference's Ceres DENSE_SCHUR factors the same matrix in
natural order (CeresUtils.cpp:43-50); only the rounding depends on the order."""
import numpy as np
import pytest

from sfmx import ba


def _tile():
    """The library's tile size (ba_kernels.hpp SFMX_BA_NB): npad / tiles of any plan."""
    p = ba.factor_plan(np.zeros((1, 1), np.uint8), ba.ORDER_NATURAL)
    return p["npad"] // p["tiles"]


NB = _tile()


def ring(C, w):
    a = np.zeros((C, C), np.uint8)
    for c in range(C):
        for d in range(1, w):
            a[c, (c + d) % C] = a[(c + d) % C, c] = 1
    return a


def clustered(C, k, seed):
    """k dense clusters chained by single links, plus random long links."""
    rng = np.random.default_rng(seed)
    a = np.zeros((C, C), np.uint8)
    lab = np.sort(rng.integers(0, k, C))
    for i in range(C):
        for j in range(i + 1, C):
            if lab[i] == lab[j] or (abs(lab[i] - lab[j]) == 1 and rng.random() < 0.02) or rng.random() < 0.002:
                a[i, j] = a[j, i] = 1
    return a


def simulate(adj, plan, seed=0):
    """Run the level schedule (block LDL^T, W_k = D_k^-1, forward solve with the rhs) and the back
    solve in numpy; -> (max relative error vs np.linalg.solve, tile-read conflicts within a level)."""
    rng = np.random.default_rng(seed)
    C, npad, T = adj.shape[0], plan["npad"], plan["tiles"]
    rows = plan["camrow"]
    # SPD S with the camera-block pattern of adj, identity padding
    S = np.eye(npad)
    B = {}
    for a in range(C):
        for b in range(a, C):
            if a == b or adj[a, b]:
                v = rng.normal(size=(6, 6))
                B[a, b] = 0.3 * v if a != b else v + v.T
    M = np.zeros((npad, npad))
    for (a, b), v in B.items():
        M[rows[a]:rows[a] + 6, rows[b]:rows[b] + 6] += v
        if a != b:
            M[rows[b]:rows[b] + 6, rows[a]:rows[a] + 6] += v.T
    pad = np.ones(npad, bool)
    for c in range(C):
        pad[rows[c]:rows[c] + 6] = False
    M[np.ix_(~pad, ~pad)] += np.eye((~pad).sum()) * (np.abs(M).sum(1).max() + 1.0)
    S = np.where(np.outer(pad, pad), np.eye(npad), M)
    b = np.where(pad, 0.0, rng.normal(size=npad))
    x_ref = np.linalg.solve(S, b)
    t = lambda i: slice(i * NB, (i + 1) * NB)   # noqa: E731
    A = S.copy()
    r = b.copy()
    W = {}
    U = {}
    for k in plan["leaves"]:
        W[k] = np.linalg.inv(A[t(k), t(k)])
        r[t(k)] = W[k] @ r[t(k)]
    conflicts = 0
    tasks, src = plan["tasks"], plan["src"]
    for lvl in range(plan["height"]):
        sel = tasks[tasks[:, 0] == lvl]
        dst = {(int(a), int(bb)) for _, a, bb, _, _, _ in sel}
        for _, a, bb, inv, s0, s1 in sel:
            for k in src[s0:s1]:
                if (a, k) in dst or (bb, k) in dst:
                    conflicts += 1
                G = A[t(a), t(k)] @ W[k]
                A[t(a), t(bb)] -= G @ A[t(bb), t(k)].T
                if a == bb:
                    r[t(a)] -= A[t(a), t(k)] @ r[t(k)]
                    U[k, a] = G.T
            if inv:
                assert a == bb
                W[a] = np.linalg.inv(A[t(a), t(a)])
                r[t(a)] = W[a] @ r[t(a)]
    assert set(W) == set(range(T)), "every panel's diagonal tile is inverted exactly once"
    for k in range(T - 1, -1, -1):   # back solve L~^T x = w in index order
        for (kk, a), u in U.items():
            if kk == k:
                r[t(k)] -= u @ r[t(a)]
    return float(np.max(np.abs(r - x_ref)) / np.max(np.abs(x_ref))), conflicts


@pytest.mark.parametrize("order", [ba.ORDER_NATURAL, ba.ORDER_ND, 2, 3, 4, ba.ORDER_AUTO])
@pytest.mark.parametrize("graph", ["ring40", "clusters", "dense12", "disconnected"])
def test_schedule_solves_system(graph, order):
    adj = {"ring40": lambda: ring(40, 4), "clusters": lambda: clustered(48, 4, 3),
           "dense12": lambda: np.ones((12, 12), np.uint8),
           "disconnected": lambda: np.kron(np.eye(3, dtype=np.uint8), ring(12, 3))}[graph]()
    plan = ba.factor_plan(adj, order)
    rows = plan["camrow"]
    assert len(set(rows.tolist())) == len(rows)
    assert rows.max() + 6 <= plan["npad"] and plan["npad"] == NB * plan["tiles"]
    spans = sorted((int(r), int(r) + 6) for r in rows)
    assert all(e0 <= s1 for (_, e0), (s1, _) in zip(spans, spans[1:])), "camera rows overlap"
    err, conflicts = simulate(adj, plan)
    assert conflicts == 0
    assert err < 1e-9


def test_ring_nested_dissection_is_shallow():
    """C5's camera graph (200 cameras on a ring, each point seen by 6 consecutive cameras): natural
    order is a chain of 19 panels of 64 rows (38 of 32); nested dissection has 5 levels (6 - 7)."""
    adj = ring(200, 6)
    nat = ba.factor_plan(adj, ba.ORDER_NATURAL)
    nd = ba.factor_plan(adj, ba.ORDER_AUTO)
    assert nat["order"] == 0 and nat["height"] == nat["tiles"] - 1 == (18 if NB == 64 else 37)
    assert nd["order"] == 1 and nd["height"] <= (5 if NB == 64 else 7)
    assert nd["predicted_us"] < 0.5 * nat["predicted_us"]


def test_dense_graph_keeps_natural_order():
    adj = np.ones((30, 30), np.uint8)
    p = ba.factor_plan(adj, ba.ORDER_AUTO)
    assert p["order"] == 0 and list(p["camrow"]) == [6 * c for c in range(30)]


def test_plan_deterministic_and_capacity():
    adj = clustered(60, 5, 7)
    a, b = ba.factor_plan(adj), ba.factor_plan(adj)
    for k in ("camrow", "leaves", "tasks", "src"):
        assert np.array_equal(a[k], b[k])
    from sfmx._lib import lib, sfmx_ba_plan_info
    import ctypes as C
    info = sfmx_ba_plan_info()
    tasks = np.zeros((1, 6), np.int32)
    rc = lib.sfmx_ba_plan(60, np.ascontiguousarray(adj).ctypes.data, -1, C.byref(info), None, None, 0,
                          tasks.ctypes.data_as(C.POINTER(C.c_int32)), 1, None, 0)
    assert rc == -4 and info.tasks == a["tasks"].shape[0]


def test_plans_equal_the_r03_library_on_random_graphs():
    """r04 records one nested dissection as a call tree and reads the leaf-size candidates off it
    (ba_plan.cpp Nd::derive) instead of dissecting once per candidate: the plans must be the ones the
    r03 library (lib/libsfmx_r03.so, built from the r03 tree) makes, field for field, every order mode."""
    import ctypes as C
    import os
    from sfmx import _lib
    path = os.path.join(os.path.dirname(_lib.LIB_PATH), "libsfmx_r03.so")
    if not os.path.exists(path):
        pytest.skip("lib/libsfmx_r03.so not built here")
    old = C.CDLL(path)
    for name, (res, args) in _lib.PROTOTYPES.items():
        if hasattr(old, name):
            f = getattr(old, name)
            f.restype, f.argtypes = res, args
    rng = np.random.default_rng(3)
    cur = ba.lib
    try:
        for it in range(60):
            n = int(rng.integers(1, 120))
            if it % 3 == 0:
                adj = (rng.random((n, n)) < rng.uniform(0.01, 0.3)).astype(np.uint8)
            elif it % 3 == 1:   # rings of bandwidth 1..5 (C5's shape)
                adj = np.zeros((n, n), np.uint8)
                for d in range(1, int(rng.integers(1, 6)) + 1):
                    adj[np.arange(n), (np.arange(n) + d) % n] = 1
            else:   # disconnected blocks
                adj = np.zeros((n, n), np.uint8)
                for s in range(0, n, 7):
                    e = min(n, s + 7)
                    adj[s:e, s:e] = rng.random((e - s, e - s)) < 0.5
            np.fill_diagonal(adj, 0)
            for order in (ba.ORDER_AUTO, 0, 1, 2, 3, 4):
                ba.lib = old
                a = ba.factor_plan(adj, order)
                ba.lib = cur
                b = ba.factor_plan(adj, order)
                for k in a:
                    assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), (it, order, k)
    finally:
        ba.lib = cur
