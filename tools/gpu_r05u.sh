#!/bin/bash
# r05u: FAST + NMS (score map of the kept pixels, fused blur) on XCD-contiguous ranges: ORB GPU tests,
# one-stream traces vs the plain grids (diagnostic SFMX_ORB_XCD_RUN=0) x 2, features_orb x 2, the ORB
# leg's FETCH_SIZE / WRITE_SIZE.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05u_pytest_orb.log 2>&1 || exit 2
prof() { tag=$1; shift; (cd /tmp && env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05u_$tag -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05u_prof_$tag.log 2>&1); }
for i in 1 2; do
  prof xcd_$i SFMX_X=0 || exit 3
  prof plain_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_XCD_RUN=0 || exit 4
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05u_orbf_$i.log 2>&1 || exit 5
done
OUT=gpurun_out/pmc_feat_r05u
mkdir -p $OUT
run() { name=$1; shift; ctr=$1; shift; timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-include-regex "orb_" --output-format csv -d $OUT -o $name -- python3 bench.py --only-orb-features --no-cpu-baseline --steps 10 > $OUT/$name.log 2>&1; }
run orb_f FETCH_SIZE && run orb_w WRITE_SIZE || exit 7
echo done
