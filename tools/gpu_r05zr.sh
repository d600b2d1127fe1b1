#!/bin/bash
# r05zr: BA set / get permute the points on the device (caller-order memcpys on the host, pieces of the
# get's D2H copied as they land): BA GPU suite + C5 oracle test, then the BA leg (call replay) alternating
# with the previous library (lib/libsfmx_prev.so), twice; the diagnostic library at 1 / 4 / 8 get pieces.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py "tests/test_gpu_fullsize.py::test_c5_full_ba_matches_oracle" > $R/gpurun_out/r05zr_pytest_ba.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r05zr_ba_new_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_prev.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r05zr_ba_prev_$i.log 2>&1 || exit 4
done
for g in 1 4 8; do
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_BA_GET_PIECES=$g timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r05zr_ba_diag_g$g.log 2>&1 || exit 5
done
echo done
