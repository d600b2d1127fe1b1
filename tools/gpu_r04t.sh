#!/bin/bash
# r04t (second run: two-way selects in place of indexed reads): the diagonal-tile inverse's inner 16 x 16 sweep on 4 x 4 pivot blocks (4 steps instead of 8):
# chol_tile micro A/B against the r04r header (tools/micro/chol_tile_r04r), the BA GPU suite, the BA leg
# twice and its kernel trace.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 60 tools/micro/chol_tile > gpurun_out/r04t_chol_tile_new_$i.txt 2>&1 || exit 1
  timeout -k 10 60 tools/micro/chol_tile_r04r > gpurun_out/r04t_chol_tile_r04r_$i.txt 2>&1 || exit 2
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_fullsize.py -m gpu -k "not c2 and not c3 and not c4" > $R/gpurun_out/r04t_pytest_ba.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04t_ba1.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r04t_ba2.log 2>&1 || exit 5
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04t_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r04t_prof_ba.log 2>&1) || exit 6
echo done
