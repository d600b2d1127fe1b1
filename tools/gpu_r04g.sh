#!/bin/bash
# r04g: ORB extraction with padded level rows and the fused FAST + NMS tile pass (GPU parity first, then
# the A/B vs the r03 library and a one-stream kernel trace); then the rest of r04e: per-XCD persistent
# screens vs the one-item-per-workgroup screens (C2, C4) and their GPU parity test.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r04g_pytest_orb.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04g_orbf_new_$i.log 2>&1 || exit 2
  SFMX_LIB_NAME=libsfmx_r03.so timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04g_orbf_r03_$i.log 2>&1 || exit 3
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04g_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r04g_prof_orb1.log 2>&1) || exit 4
M="--no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $M > $R/gpurun_out/r04g_c2_items_$i.log 2>&1 || exit 5
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_SCREEN_PERSIST=1 timeout -k 10 300 python -u bench.py $M > $R/gpurun_out/r04g_c2_xcd_$i.log 2>&1 || exit 6
done
timeout -k 10 300 python -u bench.py --workload orb $M > $R/gpurun_out/r04g_c4_items.log 2>&1 || exit 7
SFMX_LIB_NAME=libsfmx_diag.so SFMX_SCREEN_PERSIST=1 timeout -k 10 300 python -u bench.py --workload orb $M > $R/gpurun_out/r04g_c4_xcd.log 2>&1 || exit 8
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_match.py -m gpu -k persistent > $R/gpurun_out/r04g_pytest_persist.log 2>&1 || exit 9
echo done
