#!/bin/bash
# r05i: ORB angle / rBRIEF walked in row order per workgroup (orb_sort_kernel): GPU ORB suite, features_orb
# twice, one-stream kernel trace, extraction traffic PMC.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r05i_pytest_orb.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05i_orbf_$i.log 2>&1 || exit 2
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05i_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05i_prof_orb1.log 2>&1) || exit 3
timeout -k 10 800 bash tools/pmc_feat.sh r05i > $R/gpurun_out/r05i_pmc_feat.log 2>&1 || exit 4
echo done
