#!/bin/bash
# r04p: the BA GPU suite with the ring-sharded 2-rank case (plan dropped when the all-reduce callback is set).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py -m gpu > $R/gpurun_out/r04p_pytest_ba.log 2>&1 || exit 1
echo done
