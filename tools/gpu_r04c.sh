#!/bin/bash
# r04c: A/Bs after r04a -- the diagonal-tile inverse (r03 LDS inner sweep vs the r04 cross-lane form,
# tools/micro/chol_tile[_r03]), the BA factorization chol_factor vs chol_factor_w (diagnostic library,
# SFMX_BA_WIDE), the C2 matching leg with the one-launch default vs the overlapped batches, and a
# kernel trace of the batched ORB extraction leg.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 60 tools/micro/chol_tile > gpurun_out/r04c_chol_tile_new_$i.txt 2>&1 || exit 1
  timeout -k 10 60 tools/micro/chol_tile_r03 > gpurun_out/r04c_chol_tile_r03_$i.txt 2>&1 || exit 2
done
B="--only-ba --no-cpu-baseline --no-ba-calls"
for i in 1 2; do
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_BA_WIDE=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r04c_ba_wide1_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_BA_WIDE=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r04c_ba_wide0_$i.log 2>&1 || exit 4
done
M="--no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $M > gpurun_out/r04c_c2_b1_$i.log 2>&1 || exit 5
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_MATCH_BATCHES=2 timeout -k 10 300 python -u bench.py $M > gpurun_out/r04c_c2_b2_$i.log 2>&1 || exit 6
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04c_orbf -o orbf -- python3 $GRAFT_REPO_ROOT/bench.py --only-orb-features --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r04c_prof_orbf.log 2>&1 || exit 7
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04c_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py $M > $GRAFT_REPO_ROOT/gpurun_out/r04c_prof_c2.log 2>&1 || exit 8
echo done
