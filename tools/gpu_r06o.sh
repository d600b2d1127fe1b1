#!/bin/bash
# r06o: row masks built in make_plan; ba_camred stamps (stamp library): BA suite + adapters + scene + C5 parity, BA leg with the calls replay
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py tests/test_gpu_scene.py "tests/test_gpu_fullsize.py::test_c5_full_ba_matches_oracle" -m gpu > $R/gpurun_out/r06o_pytest_ba.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r06o_ba.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/ba_stamps.py > $R/gpurun_out/r06o_ba_stamps.txt 2>&1 || exit 4
tail -3 $R/gpurun_out/r06o_pytest_ba.log
cat $R/gpurun_out/r06o_ba_stamps.txt
echo done
