#!/bin/bash
# r04l: ORB resize on 128 x 16 tiles (GPU ORB suite, features_orb twice, one-stream trace); BA: the plan's
# leaf size forced (diagnostic library, SFMX_BA_ORDER nd1 / nd2 / nd4) vs the product's automatic choice.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r04l_pytest_orb.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04l_orbf_$i.log 2>&1 || exit 2
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04l_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r04l_prof_orb1.log 2>&1) || exit 3
B="--only-ba --no-cpu-baseline --no-ba-calls"
timeout -k 10 300 python -u bench.py $B > $R/gpurun_out/r04l_ba_auto.log 2>&1 || exit 4
for o in nd1 nd2 nd4; do
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_BA_ORDER=$o timeout -k 10 300 python -u bench.py $B > $R/gpurun_out/r04l_ba_$o.log 2>&1 || exit 5
done
echo done
