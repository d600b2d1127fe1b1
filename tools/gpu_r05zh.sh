#!/bin/bash
# r05zh: SIFT extrema scan with 8 rows per thread: SIFT + CLI GPU tests, homography tests (new speculation
# edge cases), a one-stream kernel trace of the features leg, the features leg x 2.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sift.py tests/test_gpu_cli.py tests/test_gpu_homography.py > $R/gpurun_out/r05zh_pytest.log 2>&1 || exit 2
(cd /tmp && SFMX_FEAT_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zh_feat -o feat -- python3 $R/bench.py --only-features --no-cpu-baseline --steps 4 > $R/gpurun_out/r05zh_prof_feat.log 2>&1) || exit 3
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-features --no-cpu-baseline > $R/gpurun_out/r05zh_feat_$i.log 2>&1 || exit 4
done
echo done
