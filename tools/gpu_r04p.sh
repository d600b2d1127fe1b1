#!/bin/bash
# r04p: the BA GPU suite with the ring-sharded 2-rank case (plan dropped when the all-reduce callback is set),
# then the whole GPU suite, smoke and the default bench line on the round's final libraries.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py -m gpu > $R/gpurun_out/r04p_pytest_ba.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $R/gpurun_out/r04p_pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r04p_smoke.log 2>&1 || exit 3
timeout -k 10 600 python -u bench.py > $R/gpurun_out/r04p_bench.log 2>&1 || exit 4
echo done
