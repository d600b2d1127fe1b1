#!/bin/bash
# r03h: BA on W_o / point records, point sums on two wave halves: parity, A/B vs the r03 base build,
# PMC traffic passes, kernel stats.  One GPU box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py > gpurun_out/r03h_ba.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03h_bench_new_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_base.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03h_bench_base_$i.log 2>&1 || exit 4
done
bash tools/pmc_ba.sh r03h > gpurun_out/r03h_pmc.log 2>&1 || exit 5
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03h -o ba -- python3 $GRAFT_REPO_ROOT/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $GRAFT_REPO_ROOT/gpurun_out/r03h_prof.log 2>&1 || exit 8
echo done
