#!/bin/bash
# r05zx: diagnostic ba_camred_wide (1024 threads per camera / intrinsics field; SFMX_BA_CRED_WIDE, libsfmx_diag.so
# only) against ba_camred in the same diagnostic library: the BA leg twice each (ms per LM iteration, iterations,
# final cost), one kernel trace each.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
export SFMX_LIB_NAME=libsfmx_diag.so
B="bench.py --only-ba --no-cpu-baseline --no-ba-calls"
for i in 1 2; do
  SFMX_BA_CRED_WIDE=1 timeout -k 10 300 python -u $B > $R/gpurun_out/r05zx_ba_wide_$i.log 2>&1 || exit 3
  timeout -k 10 300 python -u $B > $R/gpurun_out/r05zx_ba_base_$i.log 2>&1 || exit 4
done
(cd /tmp && SFMX_BA_CRED_WIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zx_wide -o ba -- python3 $R/$B > $R/gpurun_out/r05zx_prof_wide.log 2>&1) || exit 5
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zx_base -o ba -- python3 $R/$B > $R/gpurun_out/r05zx_prof_base.log 2>&1) || exit 6
echo done
