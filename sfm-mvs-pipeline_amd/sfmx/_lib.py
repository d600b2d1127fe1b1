"""ctypes binding of libsfmx.so (the C ABI declared in include/sfmx.h).

The shared library is built in-tree by ``make -C sfm-mvs-pipeline_amd`` (or
``__graft_entry__.build()``).  There is no Python or CPU fallback for any
numeric step: if the library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SFMX_LIB_NAME: another in-tree build under lib/ (A/B timing of two builds in one run, tools/ab_build.sh)
LIB_PATH = os.path.join(PKG_ROOT, "lib", os.path.basename(os.environ.get("SFMX_LIB_NAME", "libsfmx.so")))

SFMX_OK, SFMX_EINVAL, SFMX_ENOMEM, SFMX_EDEVICE, SFMX_ECAPACITY, SFMX_ESTATE, SFMX_EINTERNAL = 0, -1, -2, -3, -4, -5, -6
SFMX_NORM_L2, SFMX_NORM_HAMMING = 4, 6
SFMX_8U, SFMX_32F = 0, 5

ERROR_NAMES = {
    SFMX_EINVAL: "SFMX_EINVAL",
    SFMX_ENOMEM: "SFMX_ENOMEM",
    SFMX_EDEVICE: "SFMX_EDEVICE",
    SFMX_ECAPACITY: "SFMX_ECAPACITY",
    SFMX_ESTATE: "SFMX_ESTATE",
    SFMX_EINTERNAL: "SFMX_EINTERNAL",
}


class sfmx_desc(C.Structure):
    _fields_ = [("data", C.c_void_p), ("rows", C.c_int32), ("cols", C.c_int32),
                ("type", C.c_int32), ("_pad", C.c_int32)]


class sfmx_dmatch(C.Structure):
    _fields_ = [("queryIdx", C.c_int32), ("trainIdx", C.c_int32), ("imgIdx", C.c_int32),
                ("distance", C.c_float)]


class sfmx_ba_problem(C.Structure):
    _fields_ = [("n_points", C.c_int32), ("n_cams", C.c_int32), ("n_obs", C.c_int32), ("cam_model", C.c_int32),
                ("points", C.c_void_p), ("poses", C.c_void_p), ("intr", C.c_void_p),
                ("obs_point", C.c_void_p), ("obs_cam", C.c_void_p), ("obs_xy", C.c_void_p),
                ("cx", C.c_double), ("cy", C.c_double),
                ("n_intr", C.c_int32), ("_reserved", C.c_int32), ("intr_model", C.c_void_p),
                ("pose_intr", C.c_void_p), ("intr_center", C.c_void_p)]


class sfmx_ba_options(C.Structure):
    _fields_ = [("max_num_iterations", C.c_int32), ("max_num_consecutive_invalid_steps", C.c_int32),
                ("jacobi_scaling", C.c_int32), ("device", C.c_int32),
                ("function_tolerance", C.c_double), ("gradient_tolerance", C.c_double),
                ("parameter_tolerance", C.c_double), ("initial_trust_region_radius", C.c_double),
                ("max_trust_region_radius", C.c_double), ("min_trust_region_radius", C.c_double),
                ("min_lm_diagonal", C.c_double), ("max_lm_diagonal", C.c_double),
                ("min_relative_decrease", C.c_double), ("max_group_points", C.c_int32), ("_reserved_opt", C.c_int32)]


class sfmx_ba_plan_info(C.Structure):
    _fields_ = [("order", C.c_int32), ("leaf_tiles", C.c_int32), ("npad", C.c_int32), ("tiles", C.c_int32),
                ("tiles_nz", C.c_int32), ("height", C.c_int32), ("leaves", C.c_int32), ("tasks", C.c_int32),
                ("src", C.c_int32), ("predicted_us", C.c_double)]


class sfmx_ba_summary(C.Structure):
    _fields_ = [("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("num_successful_steps", C.c_int32), ("num_unsuccessful_steps", C.c_int32),
                ("num_invalid_steps", C.c_int32), ("termination_type", C.c_int32),
                ("total_ms", C.c_double), ("ms_per_iteration", C.c_double),
                ("final_gradient_max_norm", C.c_double), ("final_radius", C.c_double)]


class sfmx_cli_config(C.Structure):
    """include/sfmx_cli.h"""
    _fields_ = [(n, C.c_int32) for n in ("run", "loglevel", "omp_cpu_threads", "force_colored_output", "help",
                                         "n_images", "camera_model", "feature_detector", "feature_limit",
                                         "sift_n_octave_layers")] + \
               [("sift_contrast_threshold", C.c_double)] + \
               [(n, C.c_int32) for n in ("feature_matcher", "norm", "strategy", "feature_sequence",
                                         "feature_gridlength", "omp_feature_threads", "match_threshold",
                                         "baseline_homography_threshold", "distinct_matches")] + \
               [(n, C.c_double) for n in ("ransac_matching_threshold", "ransac_baseline_threshold",
                                          "ransac_pose_threshold", "homography_inlier_ratio_threshold",
                                          "pose_inlier_ratio_threshold", "reprojection_error_threshold",
                                          "pointcloud_feature_merge_distance", "pointcloud_point_merge_distance")] + \
               [(n, C.c_int32) for n in ("colored", "dense", "sgm", "mesh", "no_decimate", "refine_mesh", "stats",
                                         "artifacts", "n_warnings")] + \
               [("out", C.c_char * 1024)]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p)

# Every symbol include/sfmx.h (and include/sfmx_ba.h, sfmx_homography.h, sfmx_scene.h) declares, with its ctypes prototype.
_P = C.POINTER
_i32p, _i64p, _vp = _P(C.c_int32), _P(C.c_int64), C.c_void_p
PROTOTYPES = {
    "sfmx_pairs_unordered": (C.c_int64, [C.c_int32, _i32p, C.c_int64]),
    "sfmx_pairs_video": (C.c_int64, [C.c_int32, C.c_int32, _i32p, C.c_int64]),
    "sfmx_pairs_grid": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, _i32p, C.c_int64]),
    "sfmx_matcher_create": (C.c_int, [C.c_int32, _P(_vp)]),
    "sfmx_matcher_destroy": (C.c_int, [_vp]),
    "sfmx_matcher_set_images": (C.c_int, [_vp, _P(sfmx_desc), C.c_int32, C.c_int32, _vp]),
    "sfmx_matcher_set_images_device": (C.c_int, [_vp, _P(sfmx_desc), C.c_int32, C.c_int32, _vp]),
    "sfmx_matcher_run": (C.c_int, [_vp, _i32p, C.c_int32, C.c_double, C.c_int32, C.c_int32, _vp]),
    "sfmx_matcher_fetch": (C.c_int, [_vp, _vp, C.c_int64, _i64p, _i64p, _i32p, _vp]),
    "sfmx_matcher_device_results": (C.c_int, [_vp, _P(_vp), _P(_vp), _P(_vp)]),
    "sfmx_matcher_stats": (C.c_int, [_vp, _i64p, _i64p, _vp]),
    "sfmx_matcher_timing": (C.c_int, [_vp, _P(C.c_float), _P(C.c_float)]),
    "sfmx_matcher_pass_timing": (C.c_int, [_vp, _P(C.c_float), _P(C.c_float)]),
    "sfmx_matcher_timing_history": (C.c_int, [_vp, _P(C.c_float), _P(C.c_float), C.c_int32]),
    "sfmx_match_pairs": (C.c_int, [_P(sfmx_desc), C.c_int32, _i32p, C.c_int32, C.c_int32, C.c_double,
                                   C.c_int32, C.c_int32, C.c_int32, _vp, C.c_int64, _i64p, _i64p, _i32p]),
    "sfmx_device_count": (C.c_int, []),
    "sfmx_version": (C.c_char_p, []),
    "sfmx_last_error": (C.c_char_p, []),
    "sfmx_selftest_sqrt": (C.c_int, [C.c_int32, C.c_int64, _P(C.c_uint32)]),
    "sfmx_ba_default_options": (C.c_int, [_P(sfmx_ba_options)]),
    "sfmx_ba_solve": (C.c_int, [_P(sfmx_ba_problem), _P(sfmx_ba_options), _P(sfmx_ba_summary), _vp, C.c_int32]),
    "sfmx_ba_create": (C.c_int, [_P(sfmx_ba_problem), _P(sfmx_ba_options), _P(_vp)]),
    "sfmx_ba_set_allreduce": (C.c_int, [_vp, ALLREDUCE_FN, _vp]),
    "sfmx_ba_comm_unique_id": (C.c_int, [_vp]),
    "sfmx_ba_set_comm": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32]),
    "sfmx_ba_run": (C.c_int, [_vp, C.c_int32, _P(sfmx_ba_summary), _vp, C.c_int32]),
    "sfmx_ba_get": (C.c_int, [_vp, _P(sfmx_ba_problem)]),
    "sfmx_ba_set": (C.c_int, [_vp, _P(sfmx_ba_problem)]),
    "sfmx_ba_phase_ms": (C.c_int, [_vp, _P(C.c_double), C.c_int32]),
    "sfmx_ba_set_phase_timing": (C.c_int, [_vp, C.c_int32]),
    "sfmx_ba_destroy": (C.c_int, [_vp]),
    "sfmx_ba_update": (C.c_int, [_vp, _P(sfmx_ba_problem)]),
    "sfmx_ba_setup_ms": (C.c_int, [_vp, _P(C.c_double), C.c_int32]),
    "sfmx_ba_release_cache": (C.c_int, []),
    "sfmx_ba_debug_check_topology": (C.c_int, [_P(sfmx_ba_problem), C.c_int32, _P(C.c_double)]),   # diagnostic library only
    "sfmx_ba_debug_adjacency": (C.c_int, [_P(sfmx_ba_problem), C.c_int32, _vp]),   # diagnostic library only
    "sfmx_ba_debug_incremental_check": (C.c_int, [_P(sfmx_ba_problem), _P(sfmx_ba_problem), C.c_int32, _i32p,
                                                  _P(C.c_double)]),   # diagnostic library only
    "sfmx_ba_debug_occupancy": (C.c_int, [C.c_int32, _i32p]),   # diagnostic library only
    "sfmx_ba_jacobian": (C.c_int, [_P(sfmx_ba_problem), C.c_int32, _vp, _vp, _vp, _vp]),
    "sfmx_ba_plan": (C.c_int, [C.c_int32, _vp, C.c_int32, _P(sfmx_ba_plan_info), _i32p, _i32p, C.c_int32, _i32p,
                               C.c_int32, _i32p, C.c_int32]),
    "sfmx_pose_to_ceres": (C.c_int, [_P(C.c_double), _P(C.c_double)]),
    "sfmx_pose_from_ceres": (C.c_int, [_P(C.c_double), _P(C.c_double)]),
    "sfmx_homography_ratios": (C.c_int, [_P(_vp), _i32p, C.c_int32, _i32p, _i32p, C.c_int32, _vp, _vp, C.c_double,
                                         C.c_int32, C.c_double, C.c_int32, C.c_int32, _vp, _P(C.c_double)]),
    "sfmx_homography_last_kernel_ms": (C.c_float, []),
    "sfmx_find_3d2d_matches": (C.c_int, [_P(_vp), _i32p, C.c_int32, _i32p, C.c_int32, _vp, _vp, _vp, C.c_int32,
                                         _vp, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp, _vp]),
    "sfmx_find_3d2d_last_kernel_ms": (C.c_float, []),
    "sfmx_ba_observations_from_origins": (C.c_int, [_i64p, C.c_int32, _i32p, _P(C.c_double), C.c_int32, _i32p, _i32p,
                                                    _P(C.c_double), _i32p, _i32p, _i32p]),
    "sfmx_undistort_images": (C.c_int, [_vp, C.c_int32, C.c_int32, C.c_int32, _vp]),
    "sfmx_sift_default_params": (None, [_vp]),
    "sfmx_sift_detect_compute": (C.c_int, [_vp, C.c_int32, C.c_int32, C.c_int64, _vp, C.c_int32, C.c_int32, _vp, _vp,
                                           _vp, C.c_int32, _i32p]),
    "sfmx_sift_detect_compute_batch": (C.c_int, [_vp, C.c_int32, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, _vp,
                                                 _i32p, _i32p, _i32p]),
    "sfmx_sift_last_kernel_ms": (C.c_float, []),
    "sfmx_orb_default_params": (None, [_vp]),
    "sfmx_orb_detect_compute": (C.c_int, [_vp, C.c_int32, C.c_int32, C.c_int64, _vp, C.c_int32, C.c_int32, _vp, _vp,
                                          _vp, C.c_int32, _i32p]),
    "sfmx_orb_detect_compute_batch": (C.c_int, [_vp, C.c_int32, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, _vp,
                                                _i32p, _i32p, _i32p]),
    "sfmx_orb_last_kernel_ms": (C.c_float, []),
    "sfmx_undistort_last_kernel_ms": (C.c_float, []),
    "sfmx_openmvs_serialize": (C.c_int, [C.c_uint32, _vp, C.c_int32, _vp, C.c_int32, _P(C.c_double), C.c_int32,
                                         _i64p, _i32p, _vp, C.c_int64, _i64p, _i32p, _i32p]),
    "sfmx_openmvs_write": (C.c_int, [C.c_char_p, C.c_uint32, _vp, C.c_int32, _vp, C.c_int32, _P(C.c_double),
                                     C.c_int32, _i64p, _i32p, _i32p, _i32p]),
    "sfmx_args_parse": (C.c_int, [C.c_int32, _P(C.c_char_p), _P(_vp)]),
    "sfmx_args_destroy": (C.c_int, [_vp]),
    "sfmx_args_get": (C.c_int64, [_vp, C.c_char_p, C.c_char_p, _vp, C.c_int64]),
    "sfmx_args_count": (C.c_int32, [_vp, C.c_char_p]),
    "sfmx_args_get_at": (C.c_int64, [_vp, C.c_char_p, C.c_int32, _vp, C.c_int64]),
    "sfmx_args_is_flag": (C.c_int32, [_vp, C.c_char_p]),
    "sfmx_args_to_string": (C.c_int64, [_vp, _vp, C.c_int64]),
    "sfmx_cli_configure": (C.c_int, [_vp, _P(sfmx_cli_config), _vp, C.c_int64, _i64p]),
    "sfmx_cli_usage": (C.c_int64, [C.c_char_p, C.c_int32, _vp, C.c_int64]),
}


def _bind_runtime_like_torch() -> None:
    """PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7).  If
    libsfmx is loaded first, the system ROCm runtime is mapped and torch later
    maps a second copy (and sees no GPU).  Importing torch first makes
    libsfmx's DT_NEEDED resolve to torch's already-loaded runtime, so device
    pointers and streams can be shared.  Set SFMX_NO_TORCH=1 to skip."""
    if os.environ.get("SFMX_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def _load() -> C.CDLL:
    _bind_runtime_like_torch()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"sfmx native library not found at {LIB_PATH}; build it with "
            "`make -C sfm-mvs-pipeline_amd` (hipcc, gfx950). There is no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in PROTOTYPES.items():
        if not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class SfmxError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = (lib.sfmx_last_error() or b"").decode(errors="replace")
        super().__init__(f"{where}: {ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


def check(code: int, where: str) -> int:
    if code < 0:
        if code == SFMX_EINVAL:
            err = SfmxError(code, where)
            raise ValueError(str(err))   # reference: std::invalid_argument
        raise SfmxError(code, where)
    return code
