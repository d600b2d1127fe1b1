#!/bin/bash
# r05k: homography host driver (persistent per-device scratch/staging): its GPU tests, the matcher's,
# then the default bench line (homography leg step vs kernel time).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_homography.py tests/test_gpu_match.py > $R/gpurun_out/r05k_pytest.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > $R/gpurun_out/r05k_bench.log 2>&1 || exit 3
echo done
