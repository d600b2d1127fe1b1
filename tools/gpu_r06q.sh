#!/bin/bash
# r06q: ba_finalize loads batched (fold, rows): BA suite, BA leg, BA kernel trace

set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_scene.py "tests/test_gpu_fullsize.py::test_c5_full_ba_matches_oracle" -m gpu > $R/gpurun_out/r06q_pytest_ba.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r06q_ba.log 2>&1 || exit 3
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06q_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06q_prof_ba.log 2>&1) || exit 5
tail -3 $R/gpurun_out/r06q_pytest_ba.log
echo done
