#!/bin/bash
# r04u: the whole GPU suite, smoke and the default bench line on the round's final libraries (r04s + the
# ba_glin LDS helper; the 4x4 inner sweep reverted).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $R/gpurun_out/r04u_pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r04u_smoke.log 2>&1 || exit 3
timeout -k 10 600 python -u bench.py > $R/gpurun_out/r04u_bench.log 2>&1 || exit 4
echo done
