#!/bin/bash
# r03k: full GPU suite + smoke, BA A/B vs the r03 base build, BA call pattern (setup split timers)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r03k_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03k_smoke.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03k_bench_new_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_base.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03k_bench_base_$i.log 2>&1 || exit 4
done
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > gpurun_out/r03k_bench_calls.log 2>&1 || exit 5
echo done
