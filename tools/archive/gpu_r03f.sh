#!/bin/bash
# r03f: BA on W_o / point records (no Jacobian rows in the step kernels) vs the r03 base build;
# 32-row tiles (base code) A/B; kernel stats of the new build.  One GPU box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py > gpurun_out/r03f_ba.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03f_bench_new_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_base.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03f_bench_base_$i.log 2>&1 || exit 4
  SFMX_LIB_NAME=libsfmx_nb32.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03f_bench_nb32_$i.log 2>&1 || exit 5
done
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > gpurun_out/r03f_bench_calls.log 2>&1 || exit 6
SFMX_BENCH_BA_AR1=1 timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03f_bench_rccl1.log 2>&1 || exit 7
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03f -o ba -- python3 $GRAFT_REPO_ROOT/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $GRAFT_REPO_ROOT/gpurun_out/r03f_prof.log 2>&1 || exit 8
echo done
