#!/bin/bash
# r03e: BA context reuse / native RCCL / 32-row tiles (A/B vs 64), one GPU box
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py > gpurun_out/r03e_ba.log 2>&1 || exit 1
SFMX_LIB_NAME=libsfmx_nb32.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_fullsize.py -k "not c2 and not c3 and not c4 and not sharded" > gpurun_out/r03e_ba_nb32.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > gpurun_out/r03e_bench_ba_nb64_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_nb32.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03e_bench_ba_nb32_$i.log 2>&1 || exit 4
done
SFMX_BENCH_BA_AR1=1 timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03e_bench_ba_rccl1.log 2>&1 || exit 5
echo done
