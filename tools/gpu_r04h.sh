#!/bin/bash
# r04h: BA host setup reads the caller's arrays in caller order (radix-sorted bucket keys) and builds the
# factorization plan while the load's copies run: the BA GPU suite, the C5 call replay (setup_frac),
# the BA leg; ORB Harris / angle on aligned 4-byte window loads (GPU ORB suite, features_orb, one-stream
# trace), then the ORB extraction kernels' instruction / wait counters (PMC, one stream).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_fullsize.py -m gpu -k "not c2 and not c3 and not c4" > $R/gpurun_out/r04h_pytest_ba.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04h_ba_calls.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04h_ba_calls_2.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r04h_pytest_orb.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04h_orbf.log 2>&1 || exit 6
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04h_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r04h_prof_orb1.log 2>&1) || exit 7
timeout -k 10 600 bash tools/pmc_orb_kernels.sh r04h > $R/gpurun_out/r04h_pmc_orbk.log 2>&1 || exit 4
echo done
