#!/bin/bash
# r06y: closing checkpoint of the final r06 libraries (ba_gschur LDS-only combine barriers): the whole GPU suite, smoke, the default bench line, the C2 and BA kernel traces
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $R/gpurun_out/r06y_pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r06y_smoke.log 2>&1 || exit 3
SFMX_BENCH_DETAIL=$R/gpurun_out/r06y_bench_detail.json timeout -k 10 600 python -u bench.py > $R/gpurun_out/r06y_bench.log 2>&1 || exit 4
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06y_c2 -o c2 -- python3 $R/bench.py --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features --no-cpu-baseline > $R/gpurun_out/r06y_prof_c2.log 2>&1) || exit 5
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06y_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06y_prof_ba.log 2>&1) || exit 6
tail -c 3000 $R/gpurun_out/r06y_bench.log
echo done
