#!/bin/bash
# r05zu: ba_camred stages each camera's slot list in LDS (one dependent load level, 8 loads in flight; the adds
# keep their order): BA GPU suite + C5 oracle test, the BA leg alternating with the previous library
# (lib/libsfmx_prev.so; final costs must agree bit for bit), one BA kernel trace each.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py "tests/test_gpu_fullsize.py::test_c5_full_ba_matches_oracle" > $R/gpurun_out/r05zu_pytest_ba.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r05zu_ba_new_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_prev.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r05zu_ba_prev_$i.log 2>&1 || exit 4
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zu_new -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r05zu_prof_new.log 2>&1) || exit 5
(cd /tmp && SFMX_LIB_NAME=libsfmx_prev.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zu_prev -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r05zu_prof_prev.log 2>&1) || exit 6
echo done
