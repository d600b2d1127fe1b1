"""Debug harness (not product): run kat_orb_ties through the ORB 32x32 kernel variant given
in SFMX_ORB_VARIANT with the printf-instrumented build (SFMX_LIB_NAME=libsfmx_dbg.so)."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd"), os.path.join(REPO, "tests")]
import numpy as np
import sfmx
import fixtures
d = fixtures.load("kat_orb_ties")
m = sfmx.BFMatcher(sfmx.NORM_HAMMING)
m.set_images(d["imgs"])
m.run(d["pairs"], d["ratio"])
got, off, _ = m.fetch()
m.close()
print("variant", os.environ.get("SFMX_ORB_VARIANT"), "got", got.tolist(), "expected", d["matches"].tolist(), flush=True)
