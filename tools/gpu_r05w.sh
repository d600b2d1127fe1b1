#!/bin/bash
# r05w: (as r05v, the RNG walk in scalar registers) homography RANSAC with getSubset's attempts speculated 64 at a time on wave 0: the homography
# and CLI GPU tests (product; the serial draw on the diagnostic library, SFMX_HOMOG_SERIAL=1), then the
# C2 + homography legs x 2 in alternation with the serial draw.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_homography.py tests/test_gpu_cli.py > $R/gpurun_out/r05w_pytest.log 2>&1 || exit 2
SFMX_LIB_NAME=libsfmx_diag.so SFMX_HOMOG_SERIAL=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_homography.py > $R/gpurun_out/r05w_pytest_serial.log 2>&1 || exit 3
B="--no-ba --no-orb --no-c3 --no-f4 --no-mvs --no-features --no-orb-features"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B > $R/gpurun_out/r05w_bench_spec_$i.log 2>&1 || exit 4
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_HOMOG_SERIAL=1 timeout -k 10 300 python -u bench.py $B --no-cpu-baseline > $R/gpurun_out/r05w_bench_serial_$i.log 2>&1 || exit 5
done
echo done
