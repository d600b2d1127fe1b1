#!/bin/bash
# r04k: ORB -- dense kept-keypoint records for the angle kernel (two keypoints per wave), resize table
# prefetch, rBRIEF window stride: GPU ORB suite, features_orb twice, one-stream trace, kernel PMC.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r04k_pytest_orb.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04k_orbf_$i.log 2>&1 || exit 2
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04k_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r04k_prof_orb1.log 2>&1) || exit 3
timeout -k 10 600 bash tools/pmc_orb_kernels.sh r04k > $R/gpurun_out/r04k_pmc_orbk.log 2>&1 || exit 4
echo done
