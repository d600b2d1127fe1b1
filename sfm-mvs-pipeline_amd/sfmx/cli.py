"""The reference's command line, kept (VERDICT r01 ★ row).

``Photogrammetrie -Prun=photogrammetrie -Pimage=./images -Pfeature-detector=SIFT ...``
(sfm-mvs-pipeline_amd/bin/Photogrammetrie, or ``python -m sfmx.cli``) accepts the
run-scripts' flag sets unchanged and drives the sfmx hot path with them:

    prepareScene        image files / directories, first image's resolution, initial camera
                        (PhotogrammetrieCli.cpp:249-318)
    extractFeatures     SIFT(limit, 3, 0.09) / ORB(limit) on the GPU (SfM.cpp:577-597)
    calculateShotMatches  strategy pairs -> exact 2-NN + ratio 0.7 -> --distinct-matches ->
                        -Pmatch-threshold (SfM.cpp:542-575), all on the GPU
    calculateHomography per-pair RANSAC inlier ratio with -Pransac-matching-threshold
                        (SfM.cpp:599-637), on the GPU

Parsing and the flag -> configuration mapping (defaults, warnings, the SfM setters'
validation) are native: include/sfmx_cli.h, csrc/cli.cpp.  This module is the host
driver around them.  Stages after the match graph that sfmx does not accelerate
(incremental registration / triangulation, MVS densify, mesh; SURVEY.md §8 marks
them out of scope) are reported and skipped; ``--sfmx-plan`` (an sfmx-only flag)
prints the resolved plan and stops before any device work.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import re
import shutil
import sys
import time
from typing import List, Optional, Sequence

import numpy as np

from ._lib import lib, check, sfmx_cli_config

RUN_HELP, RUN_PHOTOGRAMMETRIE, RUN_PCL_STATS = 0, 1, 2
DETECTOR_SIFT, DETECTOR_ORB = 0, 1
MATCHER_BF, MATCHER_FLANN = 0, 1
STRATEGY_UNORDERED, STRATEGY_VIDEO, STRATEGY_GRID = 0, 1, 2
LOG_TRACE, LOG_DEBUG, LOG_INFO, LOG_WARN, LOG_ERROR = 0, 1, 2, 3, 4
CAMERA_MODELS = {1: "Simple", 3: "SimpleRadial", 7: "Distortion"}
STRATEGY_NAMES = {STRATEGY_UNORDERED: "Unordered", STRATEGY_VIDEO: "Video", STRATEGY_GRID: "Grid"}
EXIT_USAGE = 255          # the reference's exit(-1)



def prepare_working_dir(workdir: str, log) -> None:
    """PhotogrammetrieCli::prepareWorkingDir (PhotogrammetrieCli.cpp:399-402): remove_all(-Pout),
    then create it.  The reference's semantics are kept, but a -Pout that is the filesystem root,
    the home directory, the current directory or one of its ancestors is refused (that would wipe
    the caller's tree), and the path being cleared is logged."""
    target = os.path.realpath(workdir)
    cwd = os.path.realpath(os.getcwd())
    home = os.path.realpath(os.path.expanduser("~"))
    if target in (os.path.realpath(os.sep), home) or cwd == target or cwd.startswith(target.rstrip(os.sep) + os.sep):
        raise ValueError(f"-Pout={workdir}: refusing to clear {target} (the filesystem root, the home directory, "
                         "or the current directory or one of its ancestors)")
    if os.path.exists(target):
        log.info(f"clearing working directory {target}")
    shutil.rmtree(target, ignore_errors=True)
    os.makedirs(target, exist_ok=True)

def _string(call, *args) -> str:
    n = call(*args, None, 0)
    if n < 0:
        check(int(n), call.__name__)
    buf = C.create_string_buffer(int(n) + 1)
    call(*args, buf, len(buf))
    return buf.value.decode("utf-8", errors="surrogateescape")


class AppArgs:
    """AppArgs (cli/util/AppArgs.h:33-96) over sfmx_args_*: parseArgs / getArg /
    getArgs / getArgCount / isFlag / toString with the reference's semantics."""

    def __init__(self, argv: Sequence[str] = ()):
        self._h = None
        self.parseArgs(argv)

    def parseArgs(self, argv: Sequence[str]) -> None:
        self.close()
        enc = [a.encode("utf-8", errors="surrogateescape") for a in argv]
        arr = (C.c_char_p * max(len(enc), 1))(*enc)
        h = C.c_void_p()
        check(lib.sfmx_args_parse(len(enc), arr, C.byref(h)), "sfmx_args_parse")
        self._h = h

    def close(self) -> None:
        if self._h is not None and self._h.value:
            lib.sfmx_args_destroy(self._h)
        self._h = None

    __del__ = close

    def getArg(self, key: str, defaultValue: str = "") -> str:
        return _string(lib.sfmx_args_get, self._h, key.encode(), defaultValue.encode())

    def getArgCount(self, key: str) -> int:
        return int(check(lib.sfmx_args_count(self._h, key.encode()), "sfmx_args_count"))

    def getArgs(self, key: str) -> List[str]:
        return [_string(lib.sfmx_args_get_at, self._h, key.encode(), i) for i in range(self.getArgCount(key))]

    def isFlag(self, key: str) -> bool:
        return bool(check(lib.sfmx_args_is_flag(self._h, key.encode()), "sfmx_args_is_flag"))

    def toString(self) -> str:
        return _string(lib.sfmx_args_to_string, self._h)


class ConfigError(ValueError):
    """A flag value the reference rejects (std::stoi/std::stod or an SfM setter throwing)."""


def configure(args: AppArgs):
    """sfmx_cli_configure -> (sfmx_cli_config, [(level, message)]).  Raises ConfigError
    (carrying the log) for a value the reference would throw on."""
    cfg = sfmx_cli_config()
    n = C.c_int64(0)
    buf = C.create_string_buffer(1 << 16)
    rc = lib.sfmx_cli_configure(args._h, C.byref(cfg), buf, len(buf), C.byref(n))
    log = []
    for line in buf.value.decode("utf-8", errors="replace").splitlines():
        lvl, _, msg = line.partition("\t")
        log.append((int(lvl), msg))
    if rc == -1:
        err = ConfigError(log[-1][1] if log else "invalid flag value")
        err.log = log
        raise err
    check(rc, "sfmx_cli_configure")
    return cfg, log


def config_dict(cfg: sfmx_cli_config) -> dict:
    d = {}
    for name, _ in cfg._fields_:
        v = getattr(cfg, name)
        d[name] = v.decode() if isinstance(v, bytes) else v
    return d


def usage(exec_name: str, which: int) -> str:
    return _string(lib.sfmx_cli_usage, exec_name.encode(), int(which))


class AppLogger:
    """AppLogger's record layout (util/AppLogger.cpp:40-93): level, seconds since
    start, wall time, logger name, message; colour only on a tty or when forced."""
    start = time.time()
    loglevel = LOG_INFO
    always_colored = False
    NAMES = {LOG_ERROR: "ERROR", LOG_WARN: "WARN", LOG_INFO: "INFO", LOG_DEBUG: "DEBUG", LOG_TRACE: "TRACE"}

    def __init__(self, name: str, stream=None):
        self.name = name
        self.stream = stream

    def log(self, message: str, level: int, force: bool = False) -> None:
        if not force and level < AppLogger.loglevel:
            return
        out = self.stream or sys.stdout
        lvl = self.NAMES.get(level, f"Custom-{level}")
        head = (f"[{lvl}][{int(time.time() - AppLogger.start)}]"
                f"[{time.ctime()}: {lib.sfmx_version().decode()}: {self.name}]")
        if AppLogger.always_colored or out.isatty():
            out.write(f"\n\033[1;35m{head}\033[0;34m \n{message}\033[0m\n\n")
        else:
            out.write(f"\n{head} \n{message}\n\n")
        out.flush()

    def trace(self, m): self.log(m, LOG_TRACE)
    def debug(self, m): self.log(m, LOG_DEBUG)
    def info(self, m): self.log(m, LOG_INFO)
    def warn(self, m): self.log(m, LOG_WARN)
    def error(self, m): self.log(m, LOG_ERROR)


# ---- images (CameraShot::loadMImage, CameraShot.cpp:37-48) -----------------------

def image_paths(specs: Sequence[str], logger: AppLogger) -> List[str]:
    """prepareScene's expansion (:252-280): a file as is, a directory's non-directory
    entries sorted by file name; a missing path warns and is skipped."""
    out = []
    for spec in specs:
        if not os.path.exists(spec):
            logger.warn(f"image or image directory '{spec}' not found")
            continue
        if os.path.isdir(spec):
            subs = [os.path.join(spec, e) for e in os.listdir(spec)]
            subs = [p for p in subs if not os.path.isdir(p)]
            out += sorted(subs, key=lambda p: os.path.basename(p).encode("utf-8", errors="surrogateescape"))
        else:
            out.append(spec)
    return out


def image_size(path: str):
    """(width, height) of cv::imread(path) -- EXIF orientation applied, as imread does."""
    from PIL import Image, ImageOps
    with Image.open(path) as im:
        w, h = im.size
        if ImageOps.exif_transpose(im, in_place=False).size != (w, h):
            w, h = h, w
    return w, h


def load_gray(path: str, resolution=None) -> np.ndarray:
    """cv::imread(path, IMREAD_GRAYSCALE) (+ cv::resize to the scene resolution when it
    differs).  JPEG: the decoder's own grayscale output (libjpeg JCS_GRAYSCALE = the Y
    plane, as OpenCV's JPEG decoder requests it); 8-bit gray files as stored; other
    colour files: OpenCV's fixed-point RGB->gray (4899 R + 9617 G + 1868 B + 2^13) >> 14.
    Decoder builds can differ in their IDCT, so decoded pixels are 'parity unpinned'
    against an OpenCV build; everything downstream of the pixels is pinned."""
    from PIL import Image, ImageOps
    with Image.open(path) as im:
        if im.format == "JPEG":
            im.draft("L", im.size)
        im = ImageOps.exif_transpose(im)
        if im.mode == "L":
            g = np.asarray(im, np.uint8)
        else:
            rgb = np.asarray(im.convert("RGB"), np.uint32)
            g = ((rgb[..., 0] * 4899 + rgb[..., 1] * 9617 + rgb[..., 2] * 1868 + (1 << 13)) >> 14).astype(np.uint8)
    if resolution is not None and (g.shape[1], g.shape[0]) != tuple(resolution):
        # cv::resize(INTER_LINEAR) stand-in (bilinear); only hit by mixed-size image sets
        g = np.asarray(Image.fromarray(g).resize(tuple(resolution), Image.BILINEAR), np.uint8)
    return np.ascontiguousarray(g)


# ---- the photogrammetrie sub-program --------------------------------------------

def strategy_pairs(cfg) -> "callable":
    from . import matching
    if cfg.strategy == STRATEGY_GRID:
        return lambda n: matching.GridFeatureMatchingStrategy(cfg.feature_sequence, cfg.feature_gridlength).pairs(n)
    if cfg.strategy == STRATEGY_VIDEO:
        return lambda n: matching.VideoFeatureMatchingStrategy(cfg.feature_sequence).pairs(n)
    return lambda n: matching.UnorderedFeatureMatchingStrategy().pairs(n)


def make_detector(cfg):
    """configureFeatureDetector (:342-357) -> object with detectAndCompute(gray)."""
    from . import features
    if cfg.feature_detector == DETECTOR_ORB:
        if not hasattr(features, "ORB"):
            raise RuntimeError("ORB extraction is not built into this sfmx (features.ORB missing)")
        return features.ORB.create(cfg.feature_limit)
    return features.SIFT.create(cfg.feature_limit, cfg.sift_n_octave_layers, cfg.sift_contrast_threshold)


class PhotogrammetrieCli:
    logger = AppLogger("PhotogrammetrieCli")

    def __init__(self, args: AppArgs, exec_name: str = "Photogrammetrie"):
        self.args = args
        self.exec_name = exec_name
        self.timings = {}

    def _time(self, name, t0):
        self.timings[name] = (time.perf_counter() - t0) * 1e3

    def main(self) -> int:
        args, log = self.args, self.logger
        if args.isFlag("help"):                                    # init (:412-420)
            log.log("help\n" + usage(self.exec_name, 1), LOG_INFO, True)
            return EXIT_USAGE
        if args.getArgCount("image") <= 0:                         # checkImageParam (:404-410)
            log.log("no images given\n" + usage(self.exec_name, 1), LOG_INFO, True)
            return EXIT_USAGE
        try:
            cfg, msgs = configure(args)
        except ConfigError as e:
            for lvl, m in e.log:
                log.log(m, lvl)
            return EXIT_USAGE
        plan_only = args.isFlag("sfmx-plan")

        paths = image_paths(args.getArgs("image"), log)            # prepareScene (:249-318)
        log.debug(f"{len(paths)} images found")
        if len(paths) < 2:
            log.error("at least two images must be given")
            return EXIT_USAGE
        for lvl, m in msgs:                                        # camera-model warning first (:297)
            if m.startswith("unknown camera model"):
                log.log(m, lvl)
        w, h = image_size(paths[0])
        camera = {"model": CAMERA_MODELS[cfg.camera_model], "focal_length": float(max(w, h)) * 1.2,
                  "cx": w / 2.0, "cy": h / 2.0, "resolution": [w, h]}
        log.info("initial camera: " + json.dumps(camera))
        for lvl, m in msgs:                                        # detector / matcher / strategy (:86-88)
            if not m.startswith("unknown camera model"):
                log.log(m, lvl)
        pairs = strategy_pairs(cfg)(len(paths))
        plan = {"images": paths, "camera": camera, "config": config_dict(cfg),
                "strategy": STRATEGY_NAMES[cfg.strategy], "n_pairs": int(len(pairs)),
                "pairs": pairs.tolist()}
        workdir = cfg.out.decode()
        if plan_only:
            sys.stdout.write(json.dumps(plan) + "\n")
            return 0

        prepare_working_dir(workdir, log)                          # prepareWorkingDir (:399-402)
        if cfg.feature_matcher == MATCHER_FLANN:
            log.info("-Pfeature-matcher=FLANN: matching runs as exact brute force on the GPU "
                     "(exact 2-NN: FLANN's approximate search is randomised, so its lists are not reproducible)")

        from .matching import BFMatcher, LOWE_RATIO
        from .homography import homography_ratios

        # SfM::extractFeatures (SfM.cpp:577-597)
        t0 = time.perf_counter()
        det = make_detector(cfg)
        feats = []
        for i, p in enumerate(paths):
            k, d = det.detectAndCompute(load_gray(p, (w, h)))
            feats.append((k, d))
            log.info(f"features computed: {i + 1} of {len(paths)} ({int(100.0 / len(paths) * (i + 1))}%)")
        self._time("extract_features", t0)

        # SfM::calculateShotMatches (SfM.cpp:542-575)
        t0 = time.perf_counter()
        m = BFMatcher(cfg.norm)
        try:
            m.set_images([d for _, d in feats])
            m.run(pairs, LOWE_RATIO, bool(cfg.distinct_matches), int(cfg.match_threshold))
            matches, off, keep = m.fetch()
        finally:
            m.close()
        self._time("match", t0)
        kept = [p for p in range(len(pairs)) if keep[p]]
        log.info(f"{len(kept)} of {len(pairs)} image pairs kept (>= {cfg.match_threshold} matches)")

        # SfM::calculateHomography (SfM.cpp:599-637) over the kept pairs
        t0 = time.perf_counter()
        kpairs = pairs[kept].reshape(-1, 2)
        kcounts = (off[1:] - off[:-1])[kept]
        koff = np.concatenate([[0], np.cumsum(kcounts)]).astype(np.int64)
        kmatches = np.concatenate([matches[off[p]:off[p + 1]] for p in kept]) if kept else matches[:0]
        ratios = homography_ratios([np.stack([k["x"], k["y"]], 1) for k, _ in feats], [(w, h)] * len(paths),
                                   kpairs, kmatches, koff, cfg.ransac_matching_threshold)
        self._time("homography", t0)

        self._write(workdir, cfg, plan, paths, feats, kpairs, kmatches, koff, ratios)
        skipped = [f for f in ("dense", "mesh", "sgm", "refine_mesh", "no_decimate", "colored") if getattr(cfg, f)]
        log.info("match graph done; registration / triangulation"
                 + (", " + ", ".join("--" + s.replace("_", "-") for s in skipped) if skipped else "")
                 + " are outside the sfmx hot path and were not run (SURVEY.md §8)")
        return 0

    def _write(self, workdir, cfg, plan, paths, feats, pairs, matches, off, ratios):
        with open(os.path.join(workdir, "shot_matches.csv"), "w") as f:
            f.write("left,right,left_image,right_image,matches,homography_inlier_ratio\n")
            for p, (l, r) in enumerate(pairs):
                f.write(f"{l},{r},{os.path.basename(paths[l])},{os.path.basename(paths[r])},"
                        f"{int(off[p + 1] - off[p])},{ratios[p]!r}\n")
        summary = dict(plan, n_features=[int(len(k)) for k, _ in feats], kept_pairs=pairs.tolist(),
                       match_counts=[int(off[p + 1] - off[p]) for p in range(len(pairs))],
                       homography_inlier_ratios=[float(r) for r in ratios], timings_ms=self.timings)
        with open(os.path.join(workdir, "sfmx_pipeline.json"), "w") as f:
            json.dump(summary, f, indent=1)
        if cfg.stats:                                              # --stats (:126-132)
            with open(os.path.join(workdir, "app.stat.csv"), "w") as f:
                f.write("stage,ms\n")
                for k, v in self.timings.items():
                    f.write(f"{k},{v:.3f}\n")
        if cfg.artifacts:                                          # --artifacts (:139-219): raw data, not drawings
            os.makedirs(os.path.join(workdir, "features"), exist_ok=True)
            os.makedirs(os.path.join(workdir, "matches"), exist_ok=True)
            for i, (k, d) in enumerate(feats):
                np.savez(os.path.join(workdir, "features", f"{i}{os.path.basename(paths[i])}.npz"),
                         keypoints=k, descriptors=d)
            for p, (l, r) in enumerate(pairs):
                np.save(os.path.join(workdir, "matches", f"{p}{os.path.basename(paths[l])}-"
                                                         f"{os.path.basename(paths[r])}.npy"),
                        matches[off[p]:off[p + 1]])


class App:
    logger = AppLogger("App")

    @staticmethod
    def main(argv: Sequence[str]) -> int:
        """App::main (App.cpp:31-58): global flags, then the sub-program."""
        exec_name = argv[0] if argv else "Photogrammetrie"
        args = AppArgs(list(argv[1:]))
        m = re.match(r"\s*([+-]?\d+)", args.getArg("loglevel", str(LOG_INFO)))   # std::stoi
        if not m:
            App.logger.error(f"-Ploglevel={args.getArg('loglevel')}: not an int (std::stoi)")
            return EXIT_USAGE
        AppLogger.loglevel = int(m.group(1))
        AppLogger.always_colored = args.isFlag("forceColoredOutput")
        App.logger.debug("arguments:\n" + args.toString())
        run = args.getArg("run", "help")
        if run == "photogrammetrie":
            rc = PhotogrammetrieCli(args, exec_name).main()
        elif run == "pcl-stats":
            App.logger.error("-Prun=pcl-stats (point-cloud statistics) is outside the sfmx hot path")
            return EXIT_USAGE
        else:
            App.logger.log("help\n" + usage(exec_name, 0), LOG_INFO, True)
            return EXIT_USAGE
        if rc == 0:
            App.logger.info("EOL")
        return rc


def main(argv: Optional[Sequence[str]] = None) -> int:
    return App.main(list(sys.argv if argv is None else argv))


if __name__ == "__main__":
    sys.exit(main())
