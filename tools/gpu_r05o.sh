#!/bin/bash
# r05o: as r05n, every global store of the FAST + NMS tile after its last barrier:
# the ORB GPU tests, one-stream kernel traces fused (product) vs separate blur (diagnostic library,
# SFMX_ORB_BLUR_SEPARATE=1) twice in alternation, features_orb x 2, FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py > $R/gpurun_out/r05o_pytest_orb.log 2>&1 || exit 2
for i in 1 2; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05o_fused_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05o_prof_fused_$i.log 2>&1) || exit 3
  (cd /tmp && SFMX_LIB_NAME=libsfmx_diag.so SFMX_ORB_BLUR_SEPARATE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05o_sep_$i -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r05o_prof_sep_$i.log 2>&1) || exit 4
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05o_orbf_$i.log 2>&1 || exit 5
done
OUT=gpurun_out/pmc_feat_r05o
mkdir -p $OUT
run() { name=$1; shift; timeout -s KILL 180 rocprofv3 --pmc $1 --kernel-include-regex "orb_" --output-format csv -d $OUT -o $name -- python3 bench.py --only-orb-features --no-cpu-baseline --steps 10 > $OUT/$name.log 2>&1; }
run orb_f FETCH_SIZE && run orb_w WRITE_SIZE || exit 6
echo done
