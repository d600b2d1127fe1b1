#!/bin/bash
# r05j: A/B on one box, alternating, of the ORB angle / rBRIEF processing order (diagnostic library both
# sides): row-bucket order per workgroup (r05 default) vs the kept order strided over the grid (r04,
# SFMX_ORB_KEPT_ORDER=1); features_orb x 3 each, then one-stream kernel traces of both.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
export SFMX_LIB_NAME=libsfmx_diag.so
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05j_orbf_sorted_$i.log 2>&1 || exit 2
  SFMX_ORB_KEPT_ORDER=1 timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05j_orbf_kept_$i.log 2>&1 || exit 3
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05j_sorted -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05j_prof_sorted.log 2>&1) || exit 4
(cd /tmp && SFMX_ORB_KEPT_ORDER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05j_kept -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05j_prof_kept.log 2>&1) || exit 5
echo done
