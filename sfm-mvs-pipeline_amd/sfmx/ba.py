"""Bundle adjustment: Python mirror of the reference's BA interface over the C ABI
(include/sfmx_ba.h, libsfmx.so).

Reference (brunothg/sfm-mvs-pipeline/src/photogrammetrie):
  * ``BundleAdjustment::doBundleAdjustment(Scene&) -> bool``  common/BundleAdjustment.h:97,
    returns ``termination_type == CONVERGENCE`` (BundleAdjustment.cpp:140)
  * ``CeresUtils::solve`` with ``defaultOptions`` (DENSE_SCHUR, 5000 iterations)   util/CeresUtils.cpp:38-56
  * ``CeresUtils::toCeresPose / toOpenCvPose``                                   util/CeresUtils.h:90-148
  * camera models and their intrinsics block layout                               common/*Camera.cpp

``BAProblem`` holds exactly the Ceres-problem data layout the reference builds
(point[3], angle-axis pose[6], one intrinsics block[k] per camera, one residual per
observation bound to its shot's camera, BundleAdjustment.cpp:45-48, 81-89); all
arithmetic runs in the HIP kernels.  One camera: ``cam_model`` / ``intr`` / ``cx, cy``.
Several cameras: ``intr_models`` (model per camera), ``pose_intr`` (camera of each
pose), ``centers`` ((cx, cy) per camera) and ``intr`` = the blocks back to back.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from ._lib import (lib, check, sfmx_ba_problem, sfmx_ba_options, sfmx_ba_summary, sfmx_ba_plan_info, ALLREDUCE_FN)

CAM_SIMPLE, CAM_SIMPLE_RADIAL, CAM_DISTORTION = 1, 3, 7      # value = intrinsics size k
CAMERA_MODELS = {"Simple": CAM_SIMPLE, "SimpleRadial": CAM_SIMPLE_RADIAL, "Distortion": CAM_DISTORTION}
CONVERGENCE, NO_CONVERGENCE, FAILURE = 0, 1, 2
TERMINATION_NAMES = {CONVERGENCE: "CONVERGENCE", NO_CONVERGENCE: "NO_CONVERGENCE", FAILURE: "FAILURE"}
REDUCE_SUM, REDUCE_MAX = 0, 1


@dataclass
class BAProblem:
    cam_model: int
    points: np.ndarray          # (P, 3) float64
    poses: np.ndarray           # (C, 6) float64 angle-axis | t
    intr: np.ndarray            # (k,)  float64
    obs_point: np.ndarray       # (O,)  int32
    obs_cam: np.ndarray         # (O,)  int32
    obs_xy: np.ndarray          # (O, 2) float64
    cx: float = 0.0
    cy: float = 0.0
    intr_models: Optional[np.ndarray] = None   # (M,) int32: several cameras (None: the one block)
    pose_intr: Optional[np.ndarray] = None     # (C,) int32: camera of each pose
    centers: Optional[np.ndarray] = None       # (M, 2) float64: (cx, cy) per camera

    @property
    def multi(self) -> bool:
        return self.intr_models is not None

    def __post_init__(self):
        # parameter blocks are owned (copied): solve() writes the result into them
        self.points = np.array(self.points, np.float64, copy=True).reshape(-1, 3)
        self.poses = np.array(self.poses, np.float64, copy=True).reshape(-1, 6)
        self.intr = np.array(self.intr, np.float64, copy=True).reshape(-1)
        self.obs_point = np.ascontiguousarray(self.obs_point, np.int32).reshape(-1)
        self.obs_cam = np.ascontiguousarray(self.obs_cam, np.int32).reshape(-1)
        self.obs_xy = np.ascontiguousarray(self.obs_xy, np.float64).reshape(-1, 2)
        models = (CAM_SIMPLE, CAM_SIMPLE_RADIAL, CAM_DISTORTION)
        if self.multi:
            self.intr_models = np.ascontiguousarray(self.intr_models, np.int32).reshape(-1)
            self.pose_intr = np.ascontiguousarray(self.pose_intr, np.int32).reshape(-1)
            self.centers = np.ascontiguousarray(self.centers if self.centers is not None
                                                else np.zeros((len(self.intr_models), 2)), np.float64).reshape(-1, 2)
            if not all(int(m) in models for m in self.intr_models):
                raise ValueError("intr_models entries must be CAM_SIMPLE, CAM_SIMPLE_RADIAL or CAM_DISTORTION")
            if len(self.intr) != int(self.intr_models.sum()) or len(self.pose_intr) != len(self.poses) or \
                    len(self.centers) != len(self.intr_models):
                raise ValueError("intr must hold every camera's block; pose_intr one entry per pose; centers one per camera")
            return
        if self.cam_model not in models:
            raise ValueError("cam_model must be CAM_SIMPLE, CAM_SIMPLE_RADIAL or CAM_DISTORTION")
        if len(self.intr) != self.cam_model:
            raise ValueError(f"intrinsics block must have {self.cam_model} entries")

    def copy(self) -> "BAProblem":
        return BAProblem(self.cam_model, self.points.copy(), self.poses.copy(), self.intr.copy(), self.obs_point,
                         self.obs_cam, self.obs_xy, self.cx, self.cy, self.intr_models, self.pose_intr, self.centers)

    def struct(self) -> sfmx_ba_problem:
        s = sfmx_ba_problem(len(self.points), len(self.poses), len(self.obs_point), self.cam_model,
                            self.points.ctypes.data, self.poses.ctypes.data, self.intr.ctypes.data,
                            self.obs_point.ctypes.data, self.obs_cam.ctypes.data, self.obs_xy.ctypes.data,
                            float(self.cx), float(self.cy))
        if self.multi:
            s.n_intr = len(self.intr_models)
            s.intr_model = self.intr_models.ctypes.data
            s.pose_intr = self.pose_intr.ctypes.data
            s.intr_center = self.centers.ctypes.data
        return s


def default_options(**kw) -> sfmx_ba_options:
    o = sfmx_ba_options()
    check(lib.sfmx_ba_default_options(C.byref(o)), "sfmx_ba_default_options")
    for k, v in kw.items():
        if not hasattr(o, k):
            raise ValueError(f"unknown option {k}")
        setattr(o, k, v)
    return o


def summary_dict(s: sfmx_ba_summary) -> dict:
    return {f: getattr(s, f) for f, _ in s._fields_}


def solve(problem: BAProblem, options: Optional[sfmx_ba_options] = None, trace_cap: int = 0):
    """In-place solve (problem.points/poses/intr updated) -> (summary dict, trace[n,3])."""
    opt = options or default_options()
    st = problem.struct()
    sm = sfmx_ba_summary()
    tr = np.zeros((max(trace_cap, 1), 3), np.float64)
    n = check(lib.sfmx_ba_solve(C.byref(st), C.byref(opt), C.byref(sm), tr.ctypes.data if trace_cap else None,
                                trace_cap), "sfmx_ba_solve")
    return summary_dict(sm), tr[:n]


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (ncclGetUniqueId) for sfmx_ba_set_comm."""
    buf = C.create_string_buffer(128)
    check(lib.sfmx_ba_comm_unique_id(buf), "sfmx_ba_comm_unique_id")
    return buf.raw


def release_cache():
    """Free the solver contexts sfmx_ba_solve keeps per device between calls."""
    check(lib.sfmx_ba_release_cache(), "sfmx_ba_release_cache")


def jacobian(problem: BAProblem, device: int = 0):
    """Device residuals + Jacobian blocks -> (r[O,2], Je[O,2,3], Jc[O,2,6], Ji[O,2,k])."""
    O, k = len(problem.obs_point), len(problem.intr)
    r = np.zeros((O, 2)); Je = np.zeros((O, 2, 3)); Jc = np.zeros((O, 2, 6)); Ji = np.zeros((O, 2, k))
    st = problem.struct()
    check(lib.sfmx_ba_jacobian(C.byref(st), device, r.ctypes.data, Je.ctypes.data, Jc.ctypes.data, Ji.ctypes.data),
          "sfmx_ba_jacobian")
    return r, Je, Jc, Ji


class BAContext:
    """HBM-resident problem (bench / multi-GPU).  ``allreduce(buf_ptr, count, op, stream)``
    (optional) sums the reduced camera system across point-sharded ranks."""

    def __init__(self, problem: BAProblem, options: Optional[sfmx_ba_options] = None, allreduce=None):
        self.problem = problem
        self.opt = options or default_options()
        h = C.c_void_p()
        st = problem.struct()
        check(lib.sfmx_ba_create(C.byref(st), C.byref(self.opt), C.byref(h)), "sfmx_ba_create")
        self._h = h
        self._cb = None
        if allreduce is not None:
            def _cb(buf, count, op, user, stream):
                try:
                    allreduce(int(buf), int(count), int(op), int(stream or 0))
                    return 0
                except Exception:   # pragma: no cover - surfaced as SFMX_EDEVICE
                    import traceback
                    traceback.print_exc()
                    return 1
            self._cb = ALLREDUCE_FN(_cb)
            check(lib.sfmx_ba_set_allreduce(self._h, self._cb, None), "sfmx_ba_set_allreduce")

    def set_comm(self, unique_id: bytes, nranks: int, rank: int):
        """Native RCCL collectives for the point-sharded solve (sfmx_ba_set_comm): every rank
        passes the same 128-byte id (from comm_unique_id() on rank 0)."""
        buf = C.create_string_buffer(bytes(unique_id), 128)
        check(lib.sfmx_ba_set_comm(self._h, buf, nranks, rank), "sfmx_ba_set_comm")

    def run(self, max_iterations: int = 0, trace_cap: int = 0):
        sm = sfmx_ba_summary()
        tr = np.zeros((max(trace_cap, 1), 3), np.float64)
        n = check(lib.sfmx_ba_run(self._h, max_iterations, C.byref(sm), tr.ctypes.data if trace_cap else None,
                                  trace_cap), "sfmx_ba_run")
        return summary_dict(sm), tr[:n]

    def update(self, problem: BAProblem):
        """Replace the problem (any topology, e.g. a grown scene), reusing the context's device
        buffers and, when the co-visibility is unchanged, its factorization plan."""
        st = problem.struct()
        check(lib.sfmx_ba_update(self._h, C.byref(st)), "sfmx_ba_update")
        self.problem = problem

    def setup_ms(self) -> dict:
        """Host-side setup of the last create / update (ms): ordering + groups (of the camera buckets
        that changed), device allocation, uploads, factorization plan, total; plus ``buckets_redone``
        (a count: the buckets an update re-ordered, include/sfmx_ba.h sfmx_ba_setup_ms)."""
        v = (C.c_double * len(SETUP_NAMES))()
        n = check(lib.sfmx_ba_setup_ms(self._h, v, len(SETUP_NAMES)), "sfmx_ba_setup_ms")
        return {k: v[i] for i, k in enumerate(SETUP_NAMES[:n])}

    def reset(self, problem: Optional[BAProblem] = None):
        st = (problem or self.problem).struct()
        check(lib.sfmx_ba_set(self._h, C.byref(st)), "sfmx_ba_set")

    def get(self, problem: Optional[BAProblem] = None) -> BAProblem:
        p = problem or self.problem.copy()
        st = p.struct()
        check(lib.sfmx_ba_get(self._h, C.byref(st)), "sfmx_ba_get")
        return p

    def set_phase_timing(self, on: bool = True):
        """Record per-phase device events in later runs (diagnostics; each costs GPU time)."""
        check(lib.sfmx_ba_set_phase_timing(self._h, 1 if on else 0), "sfmx_ba_set_phase_timing")

    def phase_ms(self):
        """Per-phase device ms of the last run, plus ``dag_fallbacks``: steps re-run with the
        per-level factorization launches after an in-launch dependency wait timed out."""
        v = (C.c_double * 5)()
        n = check(lib.sfmx_ba_phase_ms(self._h, v, 5), "sfmx_ba_phase_ms")
        return {k: v[i] for i, k in enumerate(["linearize", "schur", "cholesky_solve", "step_cost", "dag_fallbacks"][:n])}

    def close(self):
        if getattr(self, "_h", None):
            lib.sfmx_ba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


ORDER_AUTO, ORDER_NATURAL, ORDER_ND = -1, 0, 1
# include/sfmx_ba.h sfmx_ba_setup_ms: ms unless noted
SETUP_NAMES = ["order_groups", "alloc", "upload", "plan", "total", "host_setup", "buckets_redone", "validate",
               "h_view", "h_compare", "h_bucket_lists", "h_order_groups", "h_layout", "h_merge", "h_tasks", "h_shadows",
               "plan_host", "stream_wait", "params_upload", "topology_upload"]


def factor_plan(adj: np.ndarray, order: int = ORDER_AUTO) -> dict:
    """The solver's factorization plan for a camera co-visibility graph (host only): camera rows,
    tile counts, elimination-tree height and the level schedule (include/sfmx_ba.h sfmx_ba_plan)."""
    adj = np.ascontiguousarray(adj, np.uint8)
    n = adj.shape[0]
    info = sfmx_ba_plan_info()
    camrow = np.zeros(max(n, 1), np.int32)
    check(lib.sfmx_ba_plan(n, adj.ctypes.data, order, C.byref(info), camrow.ctypes.data_as(C.POINTER(C.c_int32)),
                           None, 0, None, 0, None, 0), "sfmx_ba_plan")
    leaves = np.zeros(max(info.leaves, 1), np.int32)
    tasks = np.zeros((max(info.tasks, 1), 6), np.int32)
    src = np.zeros(max(info.src, 1), np.int32)
    i32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))   # noqa: E731
    check(lib.sfmx_ba_plan(n, adj.ctypes.data, order, C.byref(info), i32(camrow), i32(leaves), len(leaves),
                           i32(tasks), len(tasks), i32(src), len(src)), "sfmx_ba_plan")
    out = {f: getattr(info, f) for f, _ in info._fields_}
    out.update(camrow=camrow[:n], leaves=leaves[:info.leaves], tasks=tasks[:info.tasks], src=src[:info.src])
    return out


def pose_to_ceres(Rt: np.ndarray) -> np.ndarray:
    """CeresUtils::toCeresPose: 3x4 [R|t] -> {angle-axis, t}."""
    Rt = np.ascontiguousarray(Rt, np.float64).reshape(3, 4)
    out = np.zeros(6)
    check(lib.sfmx_pose_to_ceres(Rt.ctypes.data_as(C.POINTER(C.c_double)), out.ctypes.data_as(C.POINTER(C.c_double))),
          "sfmx_pose_to_ceres")
    return out


def pose_from_ceres(pose: np.ndarray) -> np.ndarray:
    """CeresUtils::toOpenCvPose: {angle-axis, t} -> 3x4 [R|t]."""
    pose = np.ascontiguousarray(pose, np.float64).reshape(6)
    out = np.zeros((3, 4))
    check(lib.sfmx_pose_from_ceres(pose.ctypes.data_as(C.POINTER(C.c_double)), out.ctypes.data_as(C.POINTER(C.c_double))),
          "sfmx_pose_from_ceres")
    return out


class BundleAdjustment:
    """``BundleAdjustment::doBundleAdjustment(scene)``: solve the scene's problem in
    place and return ``termination_type == CONVERGENCE``."""

    @staticmethod
    def doBundleAdjustment(problem: BAProblem, options: Optional[sfmx_ba_options] = None) -> bool:
        summary, _ = solve(problem, options)
        BundleAdjustment.last_summary = summary
        return summary["termination_type"] == CONVERGENCE
