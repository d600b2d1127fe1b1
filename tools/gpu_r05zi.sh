#!/bin/bash
# r05zi: SIFT extrema rows per thread only on the big launches (octave 0): SIFT GPU tests, one-stream
# traces of the product (8 rows) and of 2 / 4 rows (diagnostic SFMX_SIFT_EX_ROWS), the features leg x 2.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sift.py > $R/gpurun_out/r05zi_pytest.log 2>&1 || exit 2
prof() { tag=$1; shift; (cd /tmp && env SFMX_FEAT_STREAMS=1 "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zi_$tag -o feat -- python3 $R/bench.py --only-features --no-cpu-baseline --steps 4 > $R/gpurun_out/r05zi_prof_$tag.log 2>&1); }
prof r8 SFMX_X=0 && prof r4 SFMX_LIB_NAME=libsfmx_diag.so SFMX_SIFT_EX_ROWS=4 && prof r2 SFMX_LIB_NAME=libsfmx_diag.so SFMX_SIFT_EX_ROWS=2 || exit 3
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-features --no-cpu-baseline > $R/gpurun_out/r05zi_feat_$i.log 2>&1 || exit 4
done
echo done
