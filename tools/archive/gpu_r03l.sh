#!/bin/bash
# r03l: BA setup with a persistent host pool + presized staging (call pattern), BA parity, speculative-LM A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py > gpurun_out/r03l_ba.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > gpurun_out/r03l_bench_calls.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03l_bench_host_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_BA_SPEC=1 timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03l_bench_spec_$i.log 2>&1 || exit 4
done
echo done
