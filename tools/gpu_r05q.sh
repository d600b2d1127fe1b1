#!/bin/bash
# r05q: the fused blur's interior rows as LDS loads (r05n-p compiled them as flat loads): ORB GPU tests,
# one-stream traces fused (product) vs separate (diagnostic, SFMX_ORB_BLUR_SEPARATE=1) x 2, then the
# instruction / wait counters of both (tools/pmc_orb_kernels.sh).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05q_pytest_orb.log 2>&1 || exit 2
for i in 1 2; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05q_fused_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05q_prof_fused_$i.log 2>&1) || exit 3
  (cd /tmp && SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_BLUR_SEPARATE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05q_sep_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05q_prof_sep_$i.log 2>&1) || exit 4
done
bash tools/pmc_orb_kernels.sh r05q_fused | grep -q "pmc_rc=0" || exit 5
SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_BLUR_SEPARATE=1 bash tools/pmc_orb_kernels.sh r05q_sep | grep -q "pmc_rc=0" || exit 6
echo done
