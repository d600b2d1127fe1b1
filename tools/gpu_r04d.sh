#!/bin/bash
# r04d: the LDS inner sweep restored + chol_factor_w, the persistent (ticket-fed) SIFT / ORB screens:
# BA / match / full-size / ORB GPU tests, the fixed chol tile micro (step gate open) vs r03's, the BA leg
# vs the r03 library, the C2 leg persistent vs per-item screens (diagnostic library), the C4 leg.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_match.py tests/test_gpu_fullsize.py tests/test_gpu_orb.py -m gpu > gpurun_out/r04d_pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 60 tools/micro/chol_tile > gpurun_out/r04d_chol_tile_new_$i.txt 2>&1 || exit 2
  timeout -k 10 60 tools/micro/chol_tile_r03 > gpurun_out/r04d_chol_tile_r03_$i.txt 2>&1 || exit 3
done
B="--only-ba --no-cpu-baseline --no-ba-calls"
M="--no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/r04d_ba_new_$i.log 2>&1 || exit 4
  SFMX_LIB_NAME=libsfmx_r03.so timeout -k 10 300 python -u bench.py $B > gpurun_out/r04d_ba_r03_$i.log 2>&1 || exit 5
  timeout -k 10 300 python -u bench.py $M > gpurun_out/r04d_c2_persist_$i.log 2>&1 || exit 6
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_SCREEN_PERSIST=0 timeout -k 10 300 python -u bench.py $M > gpurun_out/r04d_c2_items_$i.log 2>&1 || exit 7
done
timeout -k 10 300 python -u bench.py --workload orb $M > gpurun_out/r04d_c4_persist.log 2>&1 || exit 8
SFMX_LIB_NAME=libsfmx_diag.so SFMX_SCREEN_PERSIST=0 timeout -k 10 300 python -u bench.py --workload orb $M > gpurun_out/r04d_c4_items.log 2>&1 || exit 9
echo done
