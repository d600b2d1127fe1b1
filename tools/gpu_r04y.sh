#!/bin/bash
# r04y: ba_gupdate held at 3 workgroups per CU (3 waves per SIMD) by an unused 47 KB dynamic LDS request
# (r04x: 4 was faster than r04u's 5): the BA GPU suite, the BA leg twice and its kernel trace.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py -m gpu > $R/gpurun_out/r04y_pytest_ba.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04y_ba1.log 2>&1 || exit 2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04y_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r04y_prof_ba.log 2>&1) || exit 3
echo done
