#!/bin/bash
# r05m: XCD run length of the ORB tile passes (diagnostic library, SFMX_ORB_XCD_RUN: 0 plain grid,
# -1 a contiguous 1/8 per XCD, else runs of that many blocks): one-stream kernel traces of each,
# twice in alternation; the ORB GPU tests on the product library first.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05m_pytest_orb.log 2>&1 || exit 2
export SFMX_LIB_NAME=libsfmx_diag.so
for i in 1 2; do
  for run in 0 8 32 128 -1; do
    (cd /tmp && SFMX_ORB_XCD_RUN=$run timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05m_${run}_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05m_prof_${run}_$i.log 2>&1) || exit 3
  done
done
echo done
