/* SPDX-License-Identifier: MIT
 *
 * sfmx CLI layer — the reference's command-line grammar and the flag -> pipeline
 * configuration mapping, as a C ABI so any host (the `Photogrammetrie` driver in
 * sfm-mvs-pipeline_amd/bin, a C++ caller, a ctypes stub) reads flags exactly the
 * way the reference does.  Pure host code: no device is touched.
 *
 * Reference interfaces replaced (paths relative to brunothg/sfm-mvs-pipeline):
 *   - AppArgs::parseArgs / getArg / getArgs / getArgCount / isFlag / toString
 *                                              src/cli/util/AppArgs.cpp:29-97, AppArgs.h:33-96
 *   - App::main's global flags (-Prun, -Ploglevel, -Pomp-cpu-threads, --forceColoredOutput)
 *                                              src/cli/App.cpp:31-58
 *   - PhotogrammetrieCli's flag -> SfM configuration
 *       runSfM setters                         src/cli/PhotogrammetrieCli.cpp:83-113
 *       (and their validation                  src/photogrammetrie/sfm/SfM.cpp:42-143)
 *       configureFeatureMatcherStrategy        src/cli/PhotogrammetrieCli.cpp:320-340
 *       configureFeatureDetector               src/cli/PhotogrammetrieCli.cpp:342-357
 *       configureFeatureMatcher                src/cli/PhotogrammetrieCli.cpp:359-392
 *       prepareScene's camera model            src/cli/PhotogrammetrieCli.cpp:288-299
 *       init / checkImageParam / getWorkingDir src/cli/PhotogrammetrieCli.cpp:394-420
 */
#ifndef SFMX_CLI_H
#define SFMX_CLI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- AppArgs -----------------------------------------------------------
 * A multimap<string,string> filled from argv (the caller passes argv + 1, as
 * App.cpp:34 does):
 *   - an argument shorter than 3 characters or not starting with '-' is an
 *     unnamed parameter stored under the key "";
 *   - otherwise type = its first two characters, key = the text after them up
 *     to the first '=' (or to the end), value = the text after that '=' (or "");
 *   - type "-P" stores key -> value, type "--" stores key -> "1", any other
 *     type (e.g. "-X...") is dropped.
 * Values for one key keep their command-line order. */
typedef struct sfmx_args sfmx_args;

int sfmx_args_parse(int32_t argc, const char* const* argv, sfmx_args** out);
int sfmx_args_destroy(sfmx_args* a);

/* String results: the value is copied NUL-terminated into buf (truncated to
 * cap-1 bytes; buf may be NULL with cap 0) and its full length is returned
 * (>= 0), so a caller can size the buffer with a first call. */

/* getArg: the first value stored for key, or default_value (NULL = "") if none. */
int64_t sfmx_args_get(const sfmx_args* a, const char* key, const char* default_value, char* buf, int64_t cap);
/* getArgCount */
int32_t sfmx_args_count(const sfmx_args* a, const char* key);
/* getArgs()[index]; SFMX_EINVAL if index is out of range. */
int64_t sfmx_args_get_at(const sfmx_args* a, const char* key, int32_t index, char* buf, int64_t cap);
/* isFlag: getArg(key, "0") == "1" (so "-Pkey=1" also sets a flag). */
int32_t sfmx_args_is_flag(const sfmx_args* a, const char* key);
/* toString: "key -> value" lines in key order. */
int64_t sfmx_args_to_string(const sfmx_args* a, char* buf, int64_t cap);

/* ---- PhotogrammetrieCli configuration ------------------------------------ */
enum { SFMX_RUN_HELP = 0, SFMX_RUN_PHOTOGRAMMETRIE = 1, SFMX_RUN_PCL_STATS = 2 };
enum { SFMX_DETECTOR_SIFT = 0, SFMX_DETECTOR_ORB = 1 };
/* FLANN is recorded as requested; sfmx executes every matcher as exact BF
 * (the FLANN forests are approximate and rebuilt per pair). */
enum { SFMX_MATCHER_BF = 0, SFMX_MATCHER_FLANN = 1 };
enum { SFMX_STRATEGY_UNORDERED = 0, SFMX_STRATEGY_VIDEO = 1, SFMX_STRATEGY_GRID = 2 };
/* Log levels of AppLogger (util/AppLogger.h:55-59). */
enum { SFMX_LOG_TRACE = 0, SFMX_LOG_DEBUG = 1, SFMX_LOG_INFO = 2, SFMX_LOG_WARN = 3, SFMX_LOG_ERROR = 4 };

typedef struct sfmx_cli_config {
    /* App.cpp:34-50 */
    int32_t run;                        /* -Prun: SFMX_RUN_* ("help" and unknown -> HELP)        */
    int32_t loglevel;                   /* -Ploglevel = 2                                          */
    int32_t omp_cpu_threads;            /* -Pomp-cpu-threads = hardware threads                    */
    int32_t force_colored_output;       /* --forceColoredOutput                                    */
    int32_t help;                       /* --help (the reference prints usage and exits)           */
    int32_t n_images;                   /* getArgCount("image"); 0 -> usage + exit in reference   */
    /* prepareScene :289-299 */
    int32_t camera_model;               /* -Pcamera-model: SFMX_CAM_* (sfmx_ba.h) = SimpleRadial  */
    /* configureFeatureDetector :342-357 */
    int32_t feature_detector;           /* -Pfeature-detector: SFMX_DETECTOR_* = SIFT             */
    int32_t feature_limit;              /* -Pfeature-limit = 10000 (ORB nfeatures / SIFT nfeatures) */
    int32_t sift_n_octave_layers;       /* 3 (SIFT::create(limit, 3, 0.09))                        */
    double  sift_contrast_threshold;    /* 0.09                                                    */
    /* configureFeatureMatcher :359-392 */
    int32_t feature_matcher;            /* -Pfeature-matcher: SFMX_MATCHER_* = BF                 */
    int32_t norm;                       /* SFMX_NORM_L2 (SIFT) / SFMX_NORM_HAMMING (ORB)           */
    /* configureFeatureMatcherStrategy :320-340 */
    int32_t strategy;                   /* SFMX_STRATEGY_*                                          */
    int32_t feature_sequence;           /* -Pfeature-sequence = 0                                   */
    int32_t feature_gridlength;         /* -Pfeature-gridlength = 0                                 */
    /* runSfM setters :94-112 (after SfM.cpp's setter normalisation) */
    int32_t omp_feature_threads;        /* -Pomp-feature-threads = 0 -> hardware threads, >= 1     */
    int32_t match_threshold;            /* -Pmatch-threshold = 20 (>= 4)                           */
    int32_t baseline_homography_threshold; /* -Pbaseline-homography-threshold = 100 (>= 4)        */
    int32_t distinct_matches;           /* --distinct-matches                                       */
    double  ransac_matching_threshold;  /* -Pransac-matching-threshold = 0.006, in [0,1]           */
    double  ransac_baseline_threshold;  /* -Pransac-baseline-threshold = -1, != 0 and <= 1         */
    double  ransac_pose_threshold;      /* -Pransac-pose-threshold = -8.0, != 0 and <= 1           */
    double  homography_inlier_ratio_threshold; /* = 0.4, in [0,1]                                  */
    double  pose_inlier_ratio_threshold;       /* = 0.4, in [0,1]                                  */
    double  reprojection_error_threshold;      /* = 10, >= 0                                       */
    double  pointcloud_feature_merge_distance; /* = 20                                             */
    double  pointcloud_point_merge_distance;   /* = 0.01                                           */
    /* output / stage flags (main :55-80, runSfM :115-136, runMVS :221-247) */
    int32_t colored, dense, sgm, mesh, no_decimate, refine_mesh, stats, artifacts;
    int32_t n_warnings;                 /* warnings written to the log                             */
    char    out[1024];                  /* -Pout = "./reconstruction"                              */
} sfmx_cli_config;

/* Reads every flag the reference reads, in the reference's order (camera model,
 * detector, matcher, strategy, then the SfM setters), applying its defaults and
 * normalisation.  The reference's warnings (unknown camera model / detector /
 * matcher, invalid sequence length) are appended to `log` as lines
 * "<level>\t<message>\n" (level = SFMX_LOG_*), NUL-terminated and truncated to
 * log_cap; *log_len (may be NULL) receives the full length.  A value the
 * reference rejects — std::stoi/std::stod failing, or an SfM setter throwing
 * std::invalid_argument — returns SFMX_EINVAL with an SFMX_LOG_ERROR line naming
 * the flag; the config then holds the values read before it. */
int sfmx_cli_configure(const sfmx_args* a, sfmx_cli_config* cfg, char* log, int64_t log_cap, int64_t* log_len);

/* Usage text of App (which = 0) or of the photogrammetrie sub-program (1), with
 * the defaults the code applies.  String result as above. */
int64_t sfmx_cli_usage(const char* exec_name, int32_t which, char* buf, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* SFMX_CLI_H */
