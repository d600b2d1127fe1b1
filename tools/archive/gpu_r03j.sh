#!/bin/bash
# r03j: glin scale loads before stores, one-pass finalize (1024 threads): parity, A/B vs r03 base, stamps, kernel stats
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py > gpurun_out/r03j_ba.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03j_bench_new_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_base.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03j_bench_base_$i.log 2>&1 || exit 4
done
timeout -k 10 300 python -u tools/ba_stamps.py > gpurun_out/r03j_stamps_new.txt 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > gpurun_out/r03j_bench_calls.log 2>&1 || exit 6
bash tools/pmc_feat.sh r03j > gpurun_out/r03j_pmc_feat.log 2>&1 || exit 7
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03j -o ba -- python3 $GRAFT_REPO_ROOT/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $GRAFT_REPO_ROOT/gpurun_out/r03j_prof.log 2>&1 || exit 8
echo done
