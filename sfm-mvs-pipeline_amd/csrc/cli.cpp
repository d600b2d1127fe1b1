// SPDX-License-Identifier: MIT
// sfmx CLI layer (VERDICT r01 ★ row: "keeping the pipeline's CLI flags"), host side.
//
//   sfmx_args_*          AppArgs (src/cli/util/AppArgs.cpp:29-97): the -P / -- grammar
//   sfmx_cli_configure   App.cpp:31-58 + PhotogrammetrieCli.cpp:83-113, 288-299, 320-420:
//                        every flag the reference reads, its default, its warning and the
//                        validation SfM's setters apply (SfM.cpp:42-143)
//   sfmx_cli_usage       App::printUsage / PhotogrammetrieCli::printUsage, with the
//                        defaults the code actually applies (the reference's
//                        usage text disagrees with its code on two defaults)
//
// Numbers are read with std::stoi / std::stod, the same functions the reference calls,
// so "12abc", " 7", "1e-3", "inf" and friends parse exactly as there; where the
// reference would die on an uncaught std::invalid_argument / std::out_of_range we
// return SFMX_EINVAL with the flag's name instead.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sfmx.h"
#include "../../include/sfmx_ba.h"
#include "../../include/sfmx_cli.h"
#include "match_common.hpp"

struct sfmx_args {
    std::multimap<std::string, std::string> kv;   // equal keys keep insertion order

    // AppArgs::getArg: first value of key, else the default
    std::string get(const std::string& key, const std::string& dflt = "") const {
        auto it = kv.find(key);
        return it == kv.end() ? dflt : it->second;
    }
    bool flag(const std::string& key) const { return get(key, "0") == "1"; }
};

namespace {

int64_t put_string(const std::string& s, char* buf, int64_t cap) {
    if (buf && cap > 0) {
        const size_t k = std::min<size_t>(s.size(), (size_t)(cap - 1));
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (int64_t)s.size();
}

int hardware_threads() { return std::max(1, (int)std::thread::hardware_concurrency()); }

struct Log {
    std::string text;
    int warnings = 0;
    void add(int level, const std::string& msg) {
        text += std::to_string(level);
        text += '\t';
        text += msg;
        text += '\n';
        if (level == SFMX_LOG_WARN) warnings++;
    }
};

struct Rejected {           // a value the reference would throw on
    std::string msg;
};

int read_int(const sfmx_args& a, const char* key, const char* dflt) {
    const std::string v = a.get(key, dflt);
    try {
        return std::stoi(v);
    } catch (const std::exception&) {
        throw Rejected{std::string("-P") + key + "=" + v + ": not an int (std::stoi)"};
    }
}

double read_double(const sfmx_args& a, const char* key, const char* dflt) {
    const std::string v = a.get(key, dflt);
    try {
        return std::stod(v);
    } catch (const std::exception&) {
        throw Rejected{std::string("-P") + key + "=" + v + ": not a number (std::stod)"};
    }
}

void require(bool ok, const char* key, const char* rule) {
    if (!ok) throw Rejected{std::string("-P") + key + ": " + rule};
}

void defaults(sfmx_cli_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->run = SFMX_RUN_HELP;
    c->loglevel = SFMX_LOG_INFO;
    c->omp_cpu_threads = hardware_threads();
    c->camera_model = SFMX_CAM_SIMPLE_RADIAL;
    c->feature_detector = SFMX_DETECTOR_SIFT;
    c->feature_limit = 10000;
    c->sift_n_octave_layers = 3;
    c->sift_contrast_threshold = 0.09;
    c->feature_matcher = SFMX_MATCHER_BF;
    c->norm = SFMX_NORM_L2;
    c->strategy = SFMX_STRATEGY_UNORDERED;
    c->omp_feature_threads = hardware_threads();
    c->match_threshold = 20;
    c->baseline_homography_threshold = 100;
    c->ransac_matching_threshold = 0.006;
    c->ransac_baseline_threshold = -1.0;
    c->ransac_pose_threshold = -8.0;
    c->homography_inlier_ratio_threshold = 0.4;
    c->pose_inlier_ratio_threshold = 0.4;
    c->reprojection_error_threshold = 10.0;
    c->pointcloud_feature_merge_distance = 20.0;
    c->pointcloud_point_merge_distance = 0.01;
    std::strcpy(c->out, "./reconstruction");
}

// PhotogrammetrieCli::prepareScene's model choice (:289-299)
void read_camera_model(const sfmx_args& a, sfmx_cli_config* c, Log& log) {
    const std::string m = a.get("camera-model", "SimpleRadial");
    if (m == "SimpleRadial") c->camera_model = SFMX_CAM_SIMPLE_RADIAL;
    else if (m == "Distortion") c->camera_model = SFMX_CAM_DISTORTION;
    else if (m == "Simple") c->camera_model = SFMX_CAM_SIMPLE;
    else {
        log.add(SFMX_LOG_WARN, "unknown camera model: " + m + " -> using SimpleRadial");
        c->camera_model = SFMX_CAM_SIMPLE_RADIAL;
    }
}

// configureFeatureDetector (:342-357): only the exact string "ORB" selects ORB; an
// empty or "SIFT" value is silent, anything else warns; both read feature-limit.
void read_detector(const sfmx_args& a, sfmx_cli_config* c, Log& log) {
    const std::string d = a.get("feature-detector");
    c->feature_limit = read_int(a, "feature-limit", "10000");
    if (d == "ORB") {
        c->feature_detector = SFMX_DETECTOR_ORB;
    } else {
        if (!d.empty() && d != "SIFT") log.add(SFMX_LOG_WARN, "unknown feature detector: " + d + " -> using SIFT");
        c->feature_detector = SFMX_DETECTOR_SIFT;
    }
}

// configureFeatureMatcher (:359-392): the norm follows the detector; "FLANN" selects the
// (approximate) FLANN index, an empty or "BF" value is silent, anything else warns.
void read_matcher(const sfmx_args& a, sfmx_cli_config* c, Log& log) {
    const std::string m = a.get("feature-matcher");
    c->norm = a.get("feature-detector") == "ORB" ? SFMX_NORM_HAMMING : SFMX_NORM_L2;
    if (m == "FLANN") {
        c->feature_matcher = SFMX_MATCHER_FLANN;
    } else {
        if (!m.empty() && m != "BF") log.add(SFMX_LOG_WARN, "unknown feature matcher: " + m + " -> using BF");
        c->feature_matcher = SFMX_MATCHER_BF;
    }
}

// configureFeatureMatcherStrategy (:320-340)
void read_strategy(const sfmx_args& a, sfmx_cli_config* c, Log& log) {
    c->feature_sequence = read_int(a, "feature-sequence", "0");
    c->feature_gridlength = read_int(a, "feature-gridlength", "0");
    if (c->feature_sequence >= 2) {
        c->strategy = c->feature_gridlength >= 1 ? SFMX_STRATEGY_GRID : SFMX_STRATEGY_VIDEO;
    } else {
        if (c->feature_sequence != 0)
            log.add(SFMX_LOG_WARN, "invalid sequence length: " + std::to_string(c->feature_sequence) +
                                       " -> using the default (unordered)");
        c->strategy = SFMX_STRATEGY_UNORDERED;
    }
}

// runSfM's setter calls, in order (:94-112), each with its SfM.cpp validation
void read_sfm(const sfmx_args& a, sfmx_cli_config* c) {
    int t = read_int(a, "omp-feature-threads", "0");                    // SfM.cpp:66-71
    if (t == 0) t = hardware_threads();
    c->omp_feature_threads = std::max(1, t);

    c->match_threshold = read_int(a, "match-threshold", "20");
    require(c->match_threshold >= 4, "match-threshold", "the minimum match count must not be < 4");   // :73-78
    c->baseline_homography_threshold = read_int(a, "baseline-homography-threshold", "100");
    require(c->baseline_homography_threshold >= 4, "baseline-homography-threshold",
            "the minimum match count must not be < 4");                  // :80-85

    double v = read_double(a, "ransac-matching-threshold", "0.006");
    require(!(v < 0 || v > 1), "ransac-matching-threshold", "must be in [0, 1]");                 // :110-115
    c->ransac_matching_threshold = v;
    v = read_double(a, "ransac-baseline-threshold", "-1");
    require(!(v == 0 || v > 1), "ransac-baseline-threshold", "must not be 0 and not > 1");        // :117-122
    c->ransac_baseline_threshold = v;
    v = read_double(a, "ransac-pose-threshold", "-8.0");
    require(!(v == 0 || v > 1), "ransac-pose-threshold", "must not be 0 and not > 1");            // :124-129
    c->ransac_pose_threshold = v;
    v = read_double(a, "homography-inlier-ratio-threshold", "0.4");
    require(!(v < 0 || v > 1), "homography-inlier-ratio-threshold", "must be in [0, 1]");         // :87-93
    c->homography_inlier_ratio_threshold = v;
    v = read_double(a, "pose-inlier-ratio-threshold", "0.4");
    require(!(v < 0 || v > 1), "pose-inlier-ratio-threshold", "must be in [0, 1]");               // :95-100
    c->pose_inlier_ratio_threshold = v;
    v = read_double(a, "reprojection-error-threshold", "10");
    require(!(v < 0), "reprojection-error-threshold", "must not be < 0");                         // :102-107
    c->reprojection_error_threshold = v;
    c->pointcloud_feature_merge_distance = read_double(a, "pointcloud-feature-merge-distance", "20");
    c->pointcloud_point_merge_distance = read_double(a, "pointcloud-point-merge-distance", "0.01");
    c->distinct_matches = a.flag("distinct-matches");
}

}  // namespace

extern "C" {

int sfmx_args_parse(int32_t argc, const char* const* argv, sfmx_args** out) {
    if (!out || argc < 0 || (argc > 0 && !argv)) {
        sfmx::set_last_error("sfmx_args_parse: bad argument");
        return SFMX_EINVAL;
    }
    auto* a = new (std::nothrow) sfmx_args;
    if (!a) return SFMX_ENOMEM;
    for (int i = 0; i < argc; i++) {
        const std::string arg = argv[i] ? argv[i] : "";
        if (arg.size() < 3 || arg[0] != '-') {          // unnamed parameter
            a->kv.emplace("", arg);
            continue;
        }
        const size_t eq = arg.find('=');
        const std::string type = arg.substr(0, 2);
        const std::string key = eq == std::string::npos ? arg.substr(2) : arg.substr(2, eq - 2);
        if (type == "-P") a->kv.emplace(key, eq == std::string::npos ? std::string() : arg.substr(eq + 1));
        else if (type == "--") a->kv.emplace(key, "1");
    }
    *out = a;
    return SFMX_OK;
}

int sfmx_args_destroy(sfmx_args* a) {
    delete a;
    return SFMX_OK;
}

int64_t sfmx_args_get(const sfmx_args* a, const char* key, const char* default_value, char* buf, int64_t cap) {
    if (!a || !key) { sfmx::set_last_error("sfmx_args_get: null argument"); return SFMX_EINVAL; }
    return put_string(a->get(key, default_value ? default_value : ""), buf, cap);
}

int32_t sfmx_args_count(const sfmx_args* a, const char* key) {
    if (!a || !key) { sfmx::set_last_error("sfmx_args_count: null argument"); return SFMX_EINVAL; }
    return (int32_t)a->kv.count(key);
}

int64_t sfmx_args_get_at(const sfmx_args* a, const char* key, int32_t index, char* buf, int64_t cap) {
    if (!a || !key) { sfmx::set_last_error("sfmx_args_get_at: null argument"); return SFMX_EINVAL; }
    auto r = a->kv.equal_range(key);
    int32_t i = 0;
    for (auto it = r.first; it != r.second; ++it, ++i)
        if (i == index) return put_string(it->second, buf, cap);
    sfmx::set_last_error("sfmx_args_get_at: index out of range");
    return SFMX_EINVAL;
}

int32_t sfmx_args_is_flag(const sfmx_args* a, const char* key) {
    if (!a || !key) { sfmx::set_last_error("sfmx_args_is_flag: null argument"); return SFMX_EINVAL; }
    return a->flag(key) ? 1 : 0;
}

int64_t sfmx_args_to_string(const sfmx_args* a, char* buf, int64_t cap) {
    if (!a) { sfmx::set_last_error("sfmx_args_to_string: null argument"); return SFMX_EINVAL; }
    std::string s;
    for (const auto& kv : a->kv) {
        if (!s.empty()) s += '\n';
        s += kv.first + " -> " + kv.second;
    }
    return put_string(s, buf, cap);
}

int sfmx_cli_configure(const sfmx_args* a, sfmx_cli_config* cfg, char* log_buf, int64_t log_cap, int64_t* log_len) {
    if (!a || !cfg) { sfmx::set_last_error("sfmx_cli_configure: null argument"); return SFMX_EINVAL; }
    defaults(cfg);
    Log log;
    int rc = SFMX_OK;
    try {
        // App::main (App.cpp:34-50)
        cfg->loglevel = read_int(*a, "loglevel", "2");
        cfg->force_colored_output = a->flag("forceColoredOutput");
        cfg->omp_cpu_threads = read_int(*a, "omp-cpu-threads", std::to_string(hardware_threads()).c_str());
        const std::string run = a->get("run", "help");
        cfg->run = run == "photogrammetrie" ? SFMX_RUN_PHOTOGRAMMETRIE
                 : run == "pcl-stats"       ? SFMX_RUN_PCL_STATS
                                            : SFMX_RUN_HELP;
        // PhotogrammetrieCli::init / checkImageParam (:404-420): the reference prints the
        // usage and exits before reading anything else, so nothing else is read here either.
        cfg->help = a->flag("help");
        cfg->n_images = (int32_t)a->kv.count("image");
        const std::string out = a->get("out", "./reconstruction");
        if (out.size() >= sizeof(cfg->out)) throw Rejected{"-Pout: path longer than 1023 bytes"};
        std::memcpy(cfg->out, out.c_str(), out.size() + 1);
        if (cfg->run == SFMX_RUN_PHOTOGRAMMETRIE && !cfg->help && cfg->n_images > 0) {
            read_camera_model(*a, cfg, log);       // prepareScene runs before runSfM (:66-67)
            read_detector(*a, cfg, log);           // runSfM :86-88
            read_matcher(*a, cfg, log);
            read_strategy(*a, cfg, log);
            read_sfm(*a, cfg);                     // :94-112
            cfg->colored = a->flag("colored");
            cfg->dense = a->flag("dense");
            cfg->sgm = a->flag("sgm");
            cfg->mesh = a->flag("mesh");
            cfg->no_decimate = a->flag("no-decimate");
            cfg->refine_mesh = a->flag("refine-mesh");
            cfg->stats = a->flag("stats");
            cfg->artifacts = a->flag("artifacts");
        }
    } catch (const Rejected& r) {
        log.add(SFMX_LOG_ERROR, r.msg);
        sfmx::set_last_error(r.msg.c_str());
        rc = SFMX_EINVAL;
    } catch (const std::bad_alloc&) {
        rc = SFMX_ENOMEM;
    }
    cfg->n_warnings = log.warnings;
    const int64_t n = put_string(log.text, log_buf, log_cap);
    if (log_len) *log_len = n;
    return rc;
}

int64_t sfmx_cli_usage(const char* exec_name, int32_t which, char* buf, int64_t cap) {
    const std::string exe = exec_name ? exec_name : "Photogrammetrie";
    std::string s;
    if (which == 0) {
        s = "usage: " + exe +
            "\n\t -Prun=[sub-program: photogrammetrie | pcl-stats]"
            "\n\t -Ploglevel=[0 (trace) .. 4 (error)] = 2"
            "\n\t -Pomp-cpu-threads=[max OpenMP threads] = " + std::to_string(hardware_threads()) +
            "\n\t --forceColoredOutput (colour log output even into a pipe)"
            "\n\t --help (this text, or the sub-program's)";
    } else if (which == 1) {
        s = "usage: " + exe + " -Prun=photogrammetrie"
            "\n\t -Pimage*=[image file or directory; repeatable]"
            "\n\t -Pout=[working / output directory] = ./reconstruction"
            "\n\t -Pcamera-model=[SimpleRadial | Distortion | Simple] = SimpleRadial"
            "\n\t -Pfeature-detector=[SIFT | ORB] = SIFT"
            "\n\t -Pfeature-limit=[max features per image] = 10000"
            "\n\t -Pfeature-matcher=[BF | FLANN] = BF   (sfmx runs both as exact BF on the GPU)"
            "\n\t -Pfeature-sequence=[pairing sequence length: 0 (unordered) or >= 2] = 0"
            "\n\t -Pfeature-gridlength=[grid row length, with -Pfeature-sequence (>= 1)] = 0"
            "\n\t -Pmatch-threshold=[min matches per image pair (>= 4)] = 20"
            "\n\t -Pbaseline-homography-threshold=[min matches for the baseline homography (>= 4)] = 100"
            "\n\t -Phomography-inlier-ratio-threshold=[0..1] = 0.4"
            "\n\t -Ppose-inlier-ratio-threshold=[0..1] = 0.4"
            "\n\t -Pransac-matching-threshold=[0..1; > 0: x * max(width, height) px] = 0.006"
            "\n\t -Pransac-baseline-threshold=[<= 1, != 0; > 0: x * max(width, height) px, < 0: -x px] = -1"
            "\n\t -Pransac-pose-threshold=[<= 1, != 0; > 0: x * max(width, height) px, < 0: -x px] = -8.0"
            "\n\t -Preprojection-error-threshold=[max reprojection error (>= 0)] = 10"
            "\n\t -Ppointcloud-feature-merge-distance=[max feature merge distance] = 20"
            "\n\t -Ppointcloud-point-merge-distance=[max point merge distance] = 0.01"
            "\n\t -Pomp-feature-threads=[feature extraction workers, 0 = auto] = 0"
            "\n\t --distinct-matches (keep only matches with a unique train feature)"
            "\n\t --colored --dense --sgm --mesh --no-decimate --refine-mesh (densification stages)"
            "\n\t --stats (write run statistics)"
            "\n\t --artifacts (write intermediate artefacts)"
            "\n\t --help (this text)";
    } else {
        sfmx::set_last_error("sfmx_cli_usage: which must be 0 or 1");
        return SFMX_EINVAL;
    }
    return put_string(s, buf, cap);
}

}  // extern "C"
