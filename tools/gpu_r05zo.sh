#!/bin/bash
# r05zo: A/B of the ORB bordered-pyramid reads (product) against the previous library (lib/libsfmx_prev.so,
# the same tree before the change): one-stream traces and the ORB leg, alternating, twice.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zo_new_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05zo_prof_new_$i.log 2>&1) || exit 2
  (cd /tmp && SFMX_LIB_NAME=libsfmx_prev.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zo_prev_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05zo_prof_prev_$i.log 2>&1) || exit 3
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05zo_orbf_new_$i.log 2>&1 || exit 4
  SFMX_LIB_NAME=libsfmx_prev.so timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05zo_orbf_prev_$i.log 2>&1 || exit 5
done
echo done
