#!/bin/bash
# r05zb: homography: resume state from LDS, 4 correspondences in flight per lane in the counts: GPU tests,
# draws, the C2 + homography legs x 2 against the serial draw.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_homography.py tests/test_gpu_cli.py > $R/gpurun_out/r05zb_pytest.log 2>&1 || exit 2
(cd tools/micro && timeout -k 5 60 ./homog_stamps_diag > $R/gpurun_out/r05zb_stamps_spec.txt 2>&1 && SFMX_HOMOG_SERIAL=1 timeout -k 5 60 ./homog_stamps_diag > $R/gpurun_out/r05zb_stamps_serial.txt 2>&1) || exit 3
B="--no-ba --no-orb --no-c3 --no-f4 --no-mvs --no-features --no-orb-features --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B > $R/gpurun_out/r05zb_bench_spec_$i.log 2>&1 || exit 4
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_HOMOG_SERIAL=1 timeout -k 10 300 python -u bench.py $B > $R/gpurun_out/r05zb_bench_serial_$i.log 2>&1 || exit 5
done
echo done
