#!/bin/bash
# r05l: ORB tile passes with XCD-contiguous grids and the per-tile packed FAST scores (no score map):
# the ORB GPU tests, features_orb on the product library x 2, the XCD A/B on the diagnostic library
# (SFMX_ORB_XCD_OFF=1: the plain grids), then FETCH_SIZE / WRITE_SIZE passes over the ORB leg.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05l_pytest_orb.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05l_orbf_prod_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_diag.so timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05l_orbf_diag_$i.log 2>&1 || exit 4
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_XCD_OFF=1 timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05l_orbf_xoff_$i.log 2>&1 || exit 5
done
OUT=gpurun_out/pmc_feat_r05l
mkdir -p $OUT
run() { name=$1; shift; timeout -s KILL 180 rocprofv3 --pmc $1 --kernel-include-regex "orb_" --output-format csv -d $OUT -o $name -- python3 bench.py --only-orb-features --no-cpu-baseline --steps 10 > $OUT/$name.log 2>&1; }
run orb_f FETCH_SIZE && run orb_w WRITE_SIZE || exit 6
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05l_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05l_prof_orb1.log 2>&1) || exit 7
echo done
