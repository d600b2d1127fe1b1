#!/bin/bash
# r05r: FAST + NMS with 8 consecutive rows per wave (scalar prefix, one barrier fewer): ORB GPU tests,
# one-stream traces of the product (fused blur, plain grid), the separate blur (diagnostic) and the
# fused pass with whole images per XCD (diagnostic, SFMX_ORB_XCD_FAST=-1), twice in alternation.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05r_pytest_orb.log 2>&1 || exit 2
prof() { tag=$1; shift; (cd /tmp && env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05r_$tag -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05r_prof_$tag.log 2>&1); }
for i in 1 2; do
  prof fused_$i SFMX_X=0 || exit 3
  prof sep_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_BLUR_SEPARATE=1 || exit 4
  prof xcdm1_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_XCD_FAST=-1 || exit 5
done
echo done
