#!/bin/bash
# r06k: (+ the C2 line with the per-run kernel events of the timed steps) ba_add_cam folded into ba_assemble (one rank), padding identity from ba_gschur
# leaf sizes nd1 / nd2 / nd4 (diagnostic library, SFMX_BA_ORDER) to re-pick the plan under the r06 masks
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_scene.py "tests/test_gpu_fullsize.py::test_c5_full_ba_matches_oracle" -m gpu > $R/gpurun_out/r06k_pytest_ba.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06k_ba.log 2>&1 || exit 3
for o in nd4; do
  SFMX_BA_ORDER=$o SFMX_LIB_NAME=libsfmx_diag.so timeout -k 10 300 python -u tools/chol_trace.py > $R/gpurun_out/r06k_chol_trace_$o.txt 2>&1 || exit 4
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06k_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06k_prof_ba.log 2>&1) || exit 5
timeout -k 10 300 python -u bench.py --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features --no-cpu-baseline > $R/gpurun_out/r06k_c2.log 2>&1 || exit 6
tail -3 $R/gpurun_out/r06k_pytest_ba.log
echo done
