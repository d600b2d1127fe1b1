#!/bin/bash
# r03g: point update fused into the candidate's ba_glin (UPD) vs the separate ba_gupdate (diag
# SFMX_BA_FUSE=0); kernel stats.  One GPU box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py > gpurun_out/r03g_ba.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03g_bench_fused_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_BA_FUSE=0 timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03g_bench_unfused_$i.log 2>&1 || exit 4
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03g -o ba -- python3 $GRAFT_REPO_ROOT/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $GRAFT_REPO_ROOT/gpurun_out/r03g_prof.log 2>&1 || exit 8
echo done
