#!/bin/bash
# r05zp: ORB edge-regime instantiations (the default edgeThreshold runs r04's register budget): ORB GPU tests,
# one-stream traces against the previous library (lib/libsfmx_prev.so), alternating, twice.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_orb.py tests/test_gpu_cli.py > $R/gpurun_out/r05zp_pytest.log 2>&1 || exit 2
for i in 1 2; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zp_new_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05zp_prof_new_$i.log 2>&1) || exit 3
  (cd /tmp && SFMX_LIB_NAME=libsfmx_prev.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zp_prev_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05zp_prof_prev_$i.log 2>&1) || exit 4
done
echo done
