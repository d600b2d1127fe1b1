#!/bin/bash
# r05zn: ORB edge thresholds below 19 (reads outside a level from OpenCV's bordered pyramid): the ORB GPU
# tests (new edge-threshold sweep vs the oracle) and the ORB leg once (the default parameters unchanged).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05zn_pytest_orb.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05zn_orbf.log 2>&1 || exit 3
echo done
