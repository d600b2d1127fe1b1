#!/bin/bash
# r04z: the whole GPU suite, smoke and the default bench line on the round's final libraries (ba_gupdate held at
# 4 workgroups per CU), then the BA leg's kernel trace.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $R/gpurun_out/r04z_pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r04z_smoke.log 2>&1 || exit 3
timeout -k 10 600 python -u bench.py > $R/gpurun_out/r04z_bench.log 2>&1 || exit 4
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04z_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r04z_prof_ba.log 2>&1) || exit 5
echo done
