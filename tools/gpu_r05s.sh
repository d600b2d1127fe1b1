#!/bin/bash
# r05s: packed FAST scores vs r04's score map (diagnostic SFMX_ORB_SCORE_MAP), each with the blur fused or
# separate: ORB GPU tests (product, then the diagnostic library with the score map), one-stream traces x 2.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05s_pytest_orb.log 2>&1 || exit 2
SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_SCORE_MAP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05s_pytest_orb_smap.log 2>&1 || exit 3
prof() { tag=$1; shift; (cd /tmp && env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05s_$tag -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05s_prof_$tag.log 2>&1); }
for i in 1 2; do
  prof packed_fused_$i SFMX_X=0 || exit 4
  prof packed_sep_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_BLUR_SEPARATE=1 || exit 5
  prof smap_fused_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_SCORE_MAP=1 || exit 6
  prof smap_sep_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_SCORE_MAP=1 SFMX_ORB_BLUR_SEPARATE=1 || exit 7
done
echo done
