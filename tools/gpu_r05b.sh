#!/bin/bash
# r05b: BA suite on the parallel host setup (product-library tiny groups included), the BA leg with the
# call replay (setup phases), and the host phase tool on the box's CPU.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r05b_pytest_ba.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r05b_bench_ba.log 2>&1 || exit 3
timeout -k 10 120 python -u tools/ba_host_phases.py 20 > $R/gpurun_out/r05b_host_phases.txt 2>&1 || exit 4
echo done
