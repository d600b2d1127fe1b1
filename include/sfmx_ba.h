/* SPDX-License-Identifier: MIT
 *
 * sfmx bundle adjustment — C ABI.
 *
 * Replaces, for the reference (brunothg/sfm-mvs-pipeline, paths under src/photogrammetrie):
 *   - BundleAdjustment::doBundleAdjustment(Scene&)                 common/BundleAdjustment.h:97
 *     (problem build :29-91, write-back :97-138)
 *   - CeresUtils::solve(ceres::Problem&, ceres::Solver::Summary&)  util/CeresUtils.h:69, .cpp:38-56
 *     with DENSE_SCHUR, max_num_iterations = 5000 and Ceres 1.14 defaults otherwise
 *   - the three AutoDiff reprojection functors                      common/SimpleRadialCamera.cpp:69-124,
 *                                                                   common/SimpleCamera.cpp:63-112,
 *                                                                   common/DistortionCamera.cpp:62-117
 * The parameter-block layout is the reference's Ceres problem layout:
 *   point double[3] (CeresPCE::coordinates, BundleAdjustment.h:28-45),
 *   pose  double[6] = angle-axis + translation (CeresCameraShot::pose, :47-64),
 *   one intrinsics block double[k] per camera (ICamera::ceresCameraParameters, ICamera.h:171;
 *   BundleAdjustment.cpp:45-48 registers every scene camera, :81-89 binds each residual to
 *   shot->getCamera()'s block):
 *     SIMPLE k=1 [f], SIMPLE_RADIAL k=3 [f,k1,k2], DISTORTION k=7 [f,cx,cy,k1,k2,p1,p2].
 * One residual block (2 residuals) per observation, squared loss, no
 * constant blocks (BundleAdjustment.cpp:83-89).  A camera no residual references is not a
 * parameter of the problem (Ceres only knows blocks that AddResidualBlock named): its values
 * are left as they are.
 */
#ifndef SFMX_BA_H
#define SFMX_BA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { SFMX_CAM_SIMPLE = 1, SFMX_CAM_SIMPLE_RADIAL = 3, SFMX_CAM_DISTORTION = 7 };   /* value = k */
/* ceres::TerminationType subset */
enum { SFMX_BA_CONVERGENCE = 0, SFMX_BA_NO_CONVERGENCE = 1, SFMX_BA_FAILURE = 2 };

typedef struct sfmx_ba_problem {
    int32_t n_points, n_cams, n_obs, cam_model;   /* cam_model = SFMX_CAM_* (n_intr == 0)     */
    double* points;                 /* 3*n_points, in/out                                      */
    double* poses;                  /* 6*n_cams (angle-axis rx,ry,rz, tx,ty,tz), in/out        */
    double* intr;                   /* in/out: n_intr == 0: the one block of k = cam_model;
                                       else the n_intr blocks back to back (block m starts at
                                       the sum of the k of blocks 0 .. m-1)                    */
    const int32_t* obs_point;       /* n_obs                                                   */
    const int32_t* obs_cam;         /* n_obs: the pose (shot) of the observation               */
    const double* obs_xy;           /* 2*n_obs observed pixel (cv::Point2f promoted to double) */
    double cx, cy;                  /* principal point, SIMPLE / SIMPLE_RADIAL only, n_intr == 0
                                       (per-residual constant, SimpleRadialCamera.cpp:118-124) */
    /* Several cameras (scene.getCameras(), BundleAdjustment.cpp:45-48).  n_intr = 0 (a
     * zero-initialised struct): every pose uses the single block above.  n_intr >= 1: */
    int32_t n_intr;                 /* number of intrinsics blocks (cameras)                   */
    int32_t _reserved;
    const int32_t* intr_model;      /* n_intr: SFMX_CAM_* of each block (models may be mixed)  */
    const int32_t* pose_intr;       /* n_cams: the block of each pose (shot->getCamera())      */
    const double* intr_center;      /* 2*n_intr: (cx, cy) of each block, read for SIMPLE /
                                       SIMPLE_RADIAL (ICamera::getCenter, ICamera.h:90)        */
} sfmx_ba_problem;
/* Capacity: the referenced blocks hold at most SFMX_BA_MAX_INTR parameters in total (e.g. one
 * DISTORTION camera, two SIMPLE_RADIAL cameras, or seven SIMPLE ones); a larger problem fails
 * with SFMX_ECAPACITY. */
enum { SFMX_BA_MAX_INTR = 7 };

typedef struct sfmx_ba_options {     /* defaults = CeresUtils::defaultOptions + Ceres 1.14 */
    int32_t max_num_iterations;              /* 5000 (CeresUtils.cpp:45)  */
    int32_t max_num_consecutive_invalid_steps;/* 5                        */
    int32_t jacobi_scaling;                  /* 1                         */
    int32_t device;                          /* HIP device index          */
    double function_tolerance;               /* 1e-6  */
    double gradient_tolerance;               /* 1e-10 */
    double parameter_tolerance;              /* 1e-8  */
    double initial_trust_region_radius;      /* 1e4   */
    double max_trust_region_radius;          /* 1e16  */
    double min_trust_region_radius;          /* 1e-32 */
    double min_lm_diagonal;                  /* 1e-6  */
    double max_lm_diagonal;                  /* 1e32  */
    double min_relative_decrease;            /* 1e-3  */
    /* sfmx only (no Ceres counterpart; 0 = automatic): at most this many points per point group of
     * the Schur kernels (1 .. 128).  Automatic sizing fills the device's workgroup slots; a small cap
     * gives many tiny groups (tests of that regime run on the product library). */
    int32_t max_group_points;
    int32_t _reserved_opt;
} sfmx_ba_options;

typedef struct sfmx_ba_summary {
    double initial_cost, final_cost;         /* 1/2 sum ||r||^2 (Ceres convention) */
    int32_t num_successful_steps;            /* Ceres counting: iteration 0 counts as successful */
    int32_t num_unsuccessful_steps;
    int32_t num_invalid_steps;
    int32_t termination_type;                /* SFMX_BA_* */
    double total_ms;                         /* minimizer wall time */
    double ms_per_iteration;                 /* total_ms / (successful + unsuccessful) */
    double final_gradient_max_norm;
    double final_radius;
} sfmx_ba_summary;

int sfmx_ba_default_options(sfmx_ba_options* opt);

/* Solve in place (the reference's doBundleAdjustment + write-back).  trace
 * (optional) receives 3 doubles per iteration: cost, trust-region radius,
 * step accepted (1/0); returns the number of trace rows written (>= 0) or a
 * negative SFMX_E* code.  The library keeps one solver context per device between
 * calls (the reference adjusts a growing scene after every registered camera,
 * SfM.cpp:235 / :371): its HIP stream, pinned memory and device buffers are reused
 * and the factorization plan too while the camera co-visibility is unchanged.
 * Calls are serialised by a lock; sfmx_ba_release_cache frees the contexts. */
int sfmx_ba_solve(sfmx_ba_problem* problem, const sfmx_ba_options* opt, sfmx_ba_summary* summary,
                  double* trace, int32_t trace_cap);
int sfmx_ba_release_cache(void);

/* ---- context API (bench / multi-GPU) --------------------------------------
 * A context keeps the problem resident in HBM.  For point-sharded multi-GPU
 * BA every rank creates a context over ITS points' observations (all cameras
 * and the intrinsics replicated) and installs an all-reduce callback; the
 * solver calls it once per linear solve on the reduced camera system and
 * gradient (device buffer of `count` doubles, sum across ranks), on the
 * camera/intrinsics column norms once per linearization, and on a few scalars
 * per iteration.  Residual costs and the point part of every norm are summed
 * over ranks; camera and intrinsics parameters are replicated.  Without a callback the context is single-GPU. */
typedef struct sfmx_ba_ctx sfmx_ba_ctx;
/* op: SFMX_REDUCE_SUM or SFMX_REDUCE_MAX; in place on a device buffer of this
 * context's device, ordered on `stream`; returns 0 on success. */
enum { SFMX_REDUCE_SUM = 0, SFMX_REDUCE_MAX = 1 };
typedef int (*sfmx_allreduce_fn)(double* device_buf, int64_t count, int32_t op, void* user, void* stream);

int sfmx_ba_create(const sfmx_ba_problem* problem, const sfmx_ba_options* opt, sfmx_ba_ctx** out);
int sfmx_ba_set_allreduce(sfmx_ba_ctx* ctx, sfmx_allreduce_fn fn, void* user);
/* Native collectives (RCCL over xGMI, one process per GPU): rank 0 calls
 * sfmx_ba_comm_unique_id (128 bytes, ncclUniqueId) and hands it to every rank (any
 * transport), then every rank calls sfmx_ba_set_comm with it.  The solver's all-reduces
 * are then ncclAllReduce on its own HIP stream, with no host callback in the LM loop; a
 * communicator takes precedence over a callback.  RCCL is loaded at run time
 * (librccl.so.1: the copy the process already has, e.g. PyTorch's). */
int sfmx_ba_comm_unique_id(void* unique_id_out);
int sfmx_ba_set_comm(sfmx_ba_ctx* ctx, const void* unique_id, int32_t nranks, int32_t rank);
/* Run the LM minimizer from the context's current parameters for at most
 * max_iterations iterations (<= 0: options.max_num_iterations). */
int sfmx_ba_run(sfmx_ba_ctx* ctx, int32_t max_iterations, sfmx_ba_summary* summary,
                double* trace, int32_t trace_cap);
/* Replace the context's problem by another one of any topology (a grown scene,
 * BundleAdjustment after every registered camera, SfM.cpp:235 / :371): the scene stays
 * resident.  Points are ordered and grouped in buckets of their smallest camera; for a
 * point-major problem (the reference's residual order) only the buckets holding points whose
 * observations (count, cameras, pixels) changed since the last load are redone on the host,
 * the others keep their order and groups and their observation data moves on the device
 * (no upload).  The result is bit-identical to a fresh context on the same problem.  Device
 * buffers are reused when large enough and the factorization plan when the camera
 * co-visibility is unchanged (single rank).  Options and the all-reduce callback stay.  Then
 * sfmx_ba_run / sfmx_ba_get as after sfmx_ba_create.  A refused problem (SFMX_EINVAL,
 * SFMX_ECAPACITY) leaves the loaded one intact; a later failure leaves the context unloaded:
 * run / get / set return SFMX_ESTATE until an update succeeds. */
int sfmx_ba_update(sfmx_ba_ctx* ctx, const sfmx_ba_problem* problem);
/* Host-side setup of the last create / update: [0] point ordering + groups (ms), [1] device
 * allocation (ms), [2] uploads (pinned staging, incl. the parameters; ms), [3] the
 * factorization plan (built at the next run; 0 when reused; ms), [4] total (ms), [5] the host
 * ordering / grouping pass alone (ms), [6] the number of camera buckets it redid, [7] the problem's
 * validation (ms), [8 .. 15] the phases of [5] (ms: point-major view, change detection, bucket
 * lists, ordering + groups of the redone buckets, layout arrays, merge, assembly tasks, shadows),
 * [16] the plan's host computation, [17] the load's final stream wait, [18] the parameters'
 * staging and copies, [19] the topology arrays' (ms).  n = entries (up to 20). */
int sfmx_ba_setup_ms(sfmx_ba_ctx* ctx, double* ms, int32_t n);
/* Copy the current parameters back into problem->points/poses/intr. */
int sfmx_ba_get(sfmx_ba_ctx* ctx, sfmx_ba_problem* problem);
/* Reset the parameters from problem->points/poses/intr (same topology). */
int sfmx_ba_set(sfmx_ba_ctx* ctx, const sfmx_ba_problem* problem);
/* Per-phase device time of the last run (ms, summed over its iterations):
 * [0] linearize (residuals + Jacobians), [1] Schur assembly, [2] Cholesky + solves,
 * [3] step / candidate cost; [4] (n >= 5) the number of steps this context re-ran with the
 * per-level factorization launches because an in-launch dependency wait saw no progress for
 * 20 ms (a preempted queue), after which the context stays on them.  n = entries written.  [1]..[3] are recorded only while
 * phase timing is on (sfmx_ba_set_phase_timing; off by default: each event costs GPU time). */
int sfmx_ba_phase_ms(sfmx_ba_ctx* ctx, double* ms, int32_t n);
/* Diagnostics: record the per-phase events of sfmx_ba_phase_ms in later runs (on != 0). */
int sfmx_ba_set_phase_timing(sfmx_ba_ctx* ctx, int32_t on);
int sfmx_ba_destroy(sfmx_ba_ctx* ctx);

/* Residuals and Jacobian blocks (device-computed) of every observation at the
 * problem's current parameters: r[2*O], Je[6*O] (d r / d point, row-major 2x3),
 * Jc[12*O] (2x6 pose), Ji[2*k*O] (2xk intrinsics; with n_intr >= 1, k = the length of the
 * whole intr array and an observation's columns outside its camera's block are 0).  For the
 * autodiff tests. */
int sfmx_ba_jacobian(const sfmx_ba_problem* problem, int32_t device, double* r, double* Je, double* Jc,
                     double* Ji);

/* The factorization plan of the reduced camera system (host only, no device work): for a
 * camera co-visibility graph adj (n_cams x n_cams, row-major, nonzero = the two cameras share a
 * point) the ordering and level schedule the solver uses (SFMX_BA_ORDER in the solver):
 * order -1 automatic (latency model), 0 natural, 1 nested dissection, 2/3/4 nested dissection
 * with leaves of 1/2/4 tiles.  Optional outputs: camrow[n_cams] (first row of each camera's 6
 * in S_cc), leaves[info.leaves], tasks[6 * info.tasks] rows (level, a, b, invert, s0, s1: tile
 * (a, b) updated from the panels src[s0 .. s1), then inverted if `invert`), src[info.src].
 * Returns SFMX_ECAPACITY (info filled) when a capacity is short.  The tiles are 64 x 64. */
typedef struct sfmx_ba_plan_info {
    int32_t order, leaf_tiles, npad, tiles, tiles_nz, height, leaves, tasks, src;
    double predicted_us;
} sfmx_ba_plan_info;
int sfmx_ba_plan(int32_t n_cams, const uint8_t* adj, int32_t order, sfmx_ba_plan_info* info, int32_t* camrow,
                 int32_t* leaves, int32_t leaves_cap, int32_t* tasks, int32_t tasks_cap, int32_t* src, int32_t src_cap);

/* Pose conversions of CeresUtils (util/CeresUtils.h:90-148): 3x4 [R|t]
 * row-major <-> Ceres pose {angle-axis, t}, via ceres::RotationMatrixToAngleAxis /
 * AngleAxisToRotationMatrix semantics.  Host-side. */
int sfmx_pose_to_ceres(const double* Rt12, double* pose6);
int sfmx_pose_from_ceres(const double* pose6, double* Rt12);

#ifdef __cplusplus
}
#endif
#endif /* SFMX_BA_H */
