#!/bin/bash
# r05zd: SIFT tile blurs and extrema scan on XCD-contiguous block ranges: the SIFT GPU tests (product),
# the features leg x 2 against the plain grids (diagnostic, SFMX_SIFT_XCD=0), FETCH_SIZE / WRITE_SIZE of
# both, and the ORB tests (xcd.hpp moved).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sift.py tests/test_gpu_orb.py > $R/gpurun_out/r05zd_pytest.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-features --no-cpu-baseline > $R/gpurun_out/r05zd_feat_xcd_$i.log 2>&1 || exit 3
  SFMX_LIB_NAME=libsfmx_diag.so SFMX_SIFT_XCD=0 timeout -k 10 300 python -u bench.py --only-features --no-cpu-baseline > $R/gpurun_out/r05zd_feat_plain_$i.log 2>&1 || exit 4
done
OUT=gpurun_out/pmc_feat_r05zd
mkdir -p $OUT
SIFT_RE="up2_kernel|to_float_kernel|blur_|small_octaves|half_nn|dog_kernel|extrema_kernel|refine_kernel|orient_kernel|descriptor_kernel"
run() { name=$1; shift; ctr=$1; shift; env "$@" timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-include-regex "$SIFT_RE" --output-format csv -d $OUT -o $name -- python3 bench.py --only-features --no-cpu-baseline --steps 10 > $OUT/$name.log 2>&1; }
run sift_f FETCH_SIZE SFMX_X=0 && run sift_w WRITE_SIZE SFMX_X=0 && run sift_plain_f FETCH_SIZE SFMX_LIB_NAME=libsfmx_diag.so SFMX_SIFT_XCD=0 || exit 5
echo done
