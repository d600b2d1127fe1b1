#!/bin/bash
# r04j: ORB -- the FAST pre-test with compacted candidates, the border test / kept places before the angles
# (no compaction kernel), chunks filling whole stream rounds: GPU ORB suite, features_orb, one-stream trace,
# kernel PMC; fresh extraction and BA traffic PMC for the bench line (the BA plan from the co-visibility and
# the r04 ORB kernels changed both); the BA GPU suite.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r04j_pytest_orb.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04j_orbf.log 2>&1 || exit 2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04j_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r04j_prof_orb1.log 2>&1) || exit 3
timeout -k 10 600 bash tools/pmc_orb_kernels.sh r04j > $R/gpurun_out/r04j_pmc_orbk.log 2>&1 || exit 4
timeout -k 10 800 bash tools/pmc_feat.sh r04j > $R/gpurun_out/r04j_pmc_feat.log 2>&1 || exit 5
timeout -k 10 600 bash tools/pmc_ba.sh r04j > $R/gpurun_out/r04j_pmc_ba.log 2>&1 || exit 6
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py -m gpu > $R/gpurun_out/r04j_pytest_ba.log 2>&1 || exit 7
echo done
