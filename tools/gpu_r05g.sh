#!/bin/bash
# r05g: BA suite + the BA leg's call replay with uninitialised topology resizes and 1024-point change blocks.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py -m gpu > $R/gpurun_out/r05g_pytest_ba.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r05g_bench_ba.log 2>&1 || exit 3
echo done
