#!/bin/bash
# r05t: FAST + NMS with the score map (kept pixels only) and the fused blur; strips of 1 (product) / 2 / 4
# tiles per workgroup (diagnostic SFMX_ORB_FAST_STRIP): ORB GPU tests, one-stream traces x 2, the ORB leg's
# FETCH_SIZE / WRITE_SIZE (product) and FETCH_SIZE with strips of 4.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05t_pytest_orb.log 2>&1 || exit 2
SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_FAST_STRIP=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05t_pytest_orb_strip4.log 2>&1 || exit 3
prof() { tag=$1; shift; (cd /tmp && env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05t_$tag -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05t_prof_$tag.log 2>&1); }
for i in 1 2; do
  prof s1_$i SFMX_X=0 || exit 4
  prof s2_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_FAST_STRIP=2 || exit 5
  prof s4_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_FAST_STRIP=4 || exit 6
done
OUT=gpurun_out/pmc_feat_r05t
mkdir -p $OUT
run() { name=$1; shift; ctr=$1; shift; env "$@" timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-include-regex "orb_" --output-format csv -d $OUT -o $name -- python3 bench.py --only-orb-features --no-cpu-baseline --steps 10 > $OUT/$name.log 2>&1; }
run orb_f FETCH_SIZE SFMX_X=0 && run orb_w WRITE_SIZE SFMX_X=0 && run orb_f_s4 FETCH_SIZE SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_FAST_STRIP=4 || exit 7
echo done
