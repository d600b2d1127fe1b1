#!/bin/bash
# r03m: point groups sized to the device's workgroup slots (group_points) + parallel radix ordering:
# BA parity, A/B vs full-size groups (diag SFMX_BA_SLOTS=0), call pattern
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py > gpurun_out/r03m_ba.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03m_bench_slots_$i.log 2>&1 || exit 2
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_BA_SLOTS=0 timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03m_bench_full_$i.log 2>&1 || exit 3
done
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > gpurun_out/r03m_bench_calls.log 2>&1 || exit 4
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03m -o ba -- python3 $GRAFT_REPO_ROOT/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $GRAFT_REPO_ROOT/gpurun_out/r03m_prof.log 2>&1 || exit 5
echo done
