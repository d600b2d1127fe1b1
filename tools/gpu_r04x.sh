#!/bin/bash
# r04x: ba_gupdate held at 4 workgroups per CU (4 waves per SIMD) by an unused 33 KB dynamic LDS request
# (r04u: 5 by its VGPRs; r04w: 6 was slower): the BA GPU suite, the BA leg twice and its kernel trace.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py -m gpu > $R/gpurun_out/r04x_pytest_ba.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04x_ba1.log 2>&1 || exit 2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04x_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r04x_prof_ba.log 2>&1) || exit 3
echo done
