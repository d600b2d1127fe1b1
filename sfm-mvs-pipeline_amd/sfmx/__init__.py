"""sfmx — MI355X-native SfM matching + bundle-adjustment hot path.

Python host layer over the C ABI in ``include/sfmx.h`` (libsfmx.so).  The
package directory is ``sfm-mvs-pipeline_amd/``; add it to ``sys.path`` and
``import sfmx``.
"""
from . import _lib  # noqa: F401  (fails loudly if libsfmx.so is missing)
from .matching import (  # noqa: F401
    BFMatcher, NORM_L2, NORM_HAMMING, LOWE_RATIO, DMATCH_DTYPE, Scene, Shot, ShotMatches,
    IFeatureMatchingStrategy, UnorderedFeatureMatchingStrategy, VideoFeatureMatchingStrategy,
    GridFeatureMatchingStrategy, calculate_shot_matches, match_pairs, pairs_unordered, pairs_video, pairs_grid,
)

from . import homography, scene, mvs, features  # noqa: F401,E402

__version__ = "0.1.0"
