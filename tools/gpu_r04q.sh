#!/bin/bash
# r04q: the BA GPU suite after draining the stream before the staging arena restarts on a load; the ORB
# suite after draining a failed chunk's stream; the BA leg with the call replay.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_fullsize.py -m gpu -k "not c2 and not c3 and not c4" > $R/gpurun_out/r04q_pytest_ba.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r04q_pytest_orb.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04q_ba_calls.log 2>&1 || exit 3
echo done
