#!/bin/bash
# r06z: LDS-only block sums at the ends of ba_glin / ba_gupdate: BA suite, stamps, BA leg, trace
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_scene.py "tests/test_gpu_fullsize.py::test_c5_full_ba_matches_oracle" -m gpu > $R/gpurun_out/r06z_pytest_ba.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/ba_stamps.py > $R/gpurun_out/r06z_ba_stamps.txt 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r06z_ba.log 2>&1 || exit 3
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06z_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06z_prof_ba.log 2>&1) || exit 5
tail -3 $R/gpurun_out/r06z_pytest_ba.log
cat $R/gpurun_out/r06z_ba_stamps.txt
echo done
