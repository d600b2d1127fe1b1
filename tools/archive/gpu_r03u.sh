#!/bin/bash
# r03u: the inner 16x16 pivot sweep by cross-lane moves (no LDS round trip per step): chol tile
# phase stamps, BA parity suite, C5 bench (final cost must stay 224576.80906871753-identical), stats
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/micro/chol_tile > gpurun_out/r03u_chol_tile.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py > gpurun_out/r03u_ba.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r03u_bench_$i.log 2>&1 || exit 3
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03u -o ba -- python3 $GRAFT_REPO_ROOT/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $GRAFT_REPO_ROOT/gpurun_out/r03u_prof.log 2>&1 || exit 4
echo done
