#!/bin/bash
# r04e: S_cc's pattern from the points' co-visibility (no group-union pairs: C5 plan height 6 -> 5,
# 82 -> 66 nonzero tiles), 4-camera buckets + 2048-point topology segments: the BA GPU suite + the
# C5 full test, the BA leg vs the r03 library (alternating), the BA leg's kernel trace, the call replay;
# ORB extraction: 64 x 32 blur tiles with sliding windows, NMS keep bits (GPU tests, A/B vs r03, one-stream trace).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_fullsize.py tests/test_gpu_orb.py -m gpu -k "not c2 and not c3 and not c4" > gpurun_out/r04e_pytest.log 2>&1 || exit 1
B="--only-ba --no-cpu-baseline --no-ba-calls"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/r04e_ba_new_$i.log 2>&1 || exit 2
  SFMX_LIB_NAME=libsfmx_r03.so timeout -k 10 300 python -u bench.py $B > gpurun_out/r04e_ba_r03_$i.log 2>&1 || exit 3
done
timeout -k 10 600 python -u bench.py --only-ba --no-cpu-baseline > gpurun_out/r04e_ba_calls.log 2>&1 || exit 4
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04e_ba -o ba -- python3 $GRAFT_REPO_ROOT/bench.py $B > $GRAFT_REPO_ROOT/gpurun_out/r04e_prof_ba.log 2>&1 || exit 5
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > gpurun_out/r04e_orbf_new_$i.log 2>&1 || exit 6
  SFMX_LIB_NAME=libsfmx_r03.so timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > gpurun_out/r04e_orbf_r03_$i.log 2>&1 || exit 7
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04e_orb1 -o orb1 -- python3 $GRAFT_REPO_ROOT/tools/orb_prof.py 32 > $GRAFT_REPO_ROOT/gpurun_out/r04e_prof_orb1.log 2>&1 || exit 8
M="--no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $M > gpurun_out/r04e_c2_items_$i.log 2>&1 || exit 9
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_SCREEN_PERSIST=1 timeout -k 10 300 python -u bench.py $M > gpurun_out/r04e_c2_xcd_$i.log 2>&1 || exit 10
done
timeout -k 10 300 python -u bench.py --workload orb $M > gpurun_out/r04e_c4_items.log 2>&1 || exit 11
SFMX_LIB_NAME=libsfmx_diag.so SFMX_SCREEN_PERSIST=1 timeout -k 10 300 python -u bench.py --workload orb $M > gpurun_out/r04e_c4_xcd.log 2>&1 || exit 12
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_match.py -m gpu -k persistent > gpurun_out/r04e_pytest_persist.log 2>&1 || exit 13
echo done
