#!/bin/bash
# r04f: the rest of r04e (whose run stopped at a relative path after a cd /tmp): ORB extraction A/B vs
# the r03 library (64 x 32 blur tiles, NMS keep bits), its one-stream kernel trace, per-XCD persistent
# screens vs the one-item-per-workgroup screens (C2, C4) and their GPU parity test.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04f_orbf_new_$i.log 2>&1 || exit 6
  SFMX_LIB_NAME=libsfmx_r03.so timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04f_orbf_r03_$i.log 2>&1 || exit 7
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04f_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r04f_prof_orb1.log 2>&1) || exit 8
M="--no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $M > $R/gpurun_out/r04f_c2_items_$i.log 2>&1 || exit 9
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_SCREEN_PERSIST=1 timeout -k 10 300 python -u bench.py $M > $R/gpurun_out/r04f_c2_xcd_$i.log 2>&1 || exit 10
done
timeout -k 10 300 python -u bench.py --workload orb $M > $R/gpurun_out/r04f_c4_items.log 2>&1 || exit 11
SFMX_LIB_NAME=libsfmx_diag.so SFMX_SCREEN_PERSIST=1 timeout -k 10 300 python -u bench.py --workload orb $M > $R/gpurun_out/r04f_c4_xcd.log 2>&1 || exit 12
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_match.py -m gpu -k persistent > $R/gpurun_out/r04f_pytest_persist.log 2>&1 || exit 13
echo done
