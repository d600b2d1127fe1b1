#!/bin/bash
# r04r: ba_glin's observation records (jer) at an 80-B row stride (K < 7) against the LDS bank conflicts
# of the 64-B rows: the BA GPU suite, the BA leg twice, its kernel trace and PMC.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_fullsize.py -m gpu -k "not c2 and not c3 and not c4" > $R/gpurun_out/r04r_pytest_ba.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04r_ba1.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04r_ba2.log 2>&1 || exit 3
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04r_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r04r_prof_ba.log 2>&1) || exit 4
timeout -k 10 600 bash tools/pmc_ba.sh r04r > $R/gpurun_out/r04r_pmc_ba.log 2>&1 || exit 5
echo done
