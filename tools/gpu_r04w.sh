#!/bin/bash
# r04w: ba_gupdate at 6 waves per SIMD (launch bounds: 79 VGPRs, 1536 workgroup slots for its 2028 groups;
# r04u: 88 VGPRs, 5 waves): the BA GPU suite, the BA leg twice and
# its kernel trace; then the whole GPU suite, smoke and the default bench line on these libraries.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_fullsize.py -m gpu -k "not c2 and not c3 and not c4" > $R/gpurun_out/r04w_pytest_ba.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04w_ba1.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04w_ba2.log 2>&1 || exit 3
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04w_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r04w_prof_ba.log 2>&1) || exit 4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $R/gpurun_out/r04w_pytest_gpu.log 2>&1 || exit 5
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r04w_smoke.log 2>&1 || exit 6
timeout -k 10 600 python -u bench.py > $R/gpurun_out/r04w_bench.log 2>&1 || exit 7
echo done
