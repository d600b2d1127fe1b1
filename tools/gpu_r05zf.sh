#!/bin/bash
# r05zf: the product's SIFT order (tile blurs XCD-contiguous, extrema on the plain grid): SIFT GPU tests,
# features leg x 2, FETCH_SIZE / WRITE_SIZE of the leg.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sift.py > $R/gpurun_out/r05zf_pytest.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-features --no-cpu-baseline > $R/gpurun_out/r05zf_feat_$i.log 2>&1 || exit 3
done
OUT=gpurun_out/pmc_feat_r05zf
mkdir -p $OUT
SIFT_RE="up2_kernel|to_float_kernel|blur_|small_octaves|half_nn|dog_kernel|extrema_kernel|refine_kernel|orient_kernel|descriptor_kernel"
run() { name=$1; shift; ctr=$1; shift; timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-include-regex "$SIFT_RE" --output-format csv -d $OUT -o $name -- python3 bench.py --only-features --no-cpu-baseline --steps 10 > $OUT/$name.log 2>&1; }
run sift_f FETCH_SIZE && run sift_w WRITE_SIZE || exit 5
echo done
