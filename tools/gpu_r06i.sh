#!/bin/bash
# r06i: masked tile products spread over the four waves (chol_factor)
# leaf sizes nd1 / nd2 / nd4 (diagnostic library, SFMX_BA_ORDER) to re-pick the plan under the r06 masks
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py "tests/test_gpu_fullsize.py::test_c5_full_ba_matches_oracle" -m gpu > $R/gpurun_out/r06i_pytest_ba.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06i_ba.log 2>&1 || exit 3
for o in nd4; do
  SFMX_BA_ORDER=$o SFMX_LIB_NAME=libsfmx_diag.so timeout -k 10 300 python -u tools/chol_trace.py > $R/gpurun_out/r06i_chol_trace_$o.txt 2>&1 || exit 4
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06i_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06i_prof_ba.log 2>&1) || exit 5
tail -3 $R/gpurun_out/r06i_pytest_ba.log
echo done
