#!/bin/bash
# r05zc: the whole GPU suite, smoke and the default bench line after the ORB tile-pass fusion and the
# homography speculation.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $R/gpurun_out/r05zc_pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r05zc_smoke.log 2>&1 || exit 3
SFMX_BENCH_DETAIL=$R/gpurun_out/r05zc_bench_detail.json timeout -k 10 600 python -u bench.py > $R/gpurun_out/r05zc_bench.log 2>&1 || exit 4
tail -c 4000 $R/gpurun_out/r05zc_bench.log
echo done
