#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter per rocprofv3 run, no trace domains with --pmc) over the
# SIFT and ORB extraction legs of bench.py -> gpurun_out/pmc_feat_<tag>/; summarise with tools/pmc_feat_json.py
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_feat_${1:-r03}
mkdir -p $OUT
SIFT_RE="up2_kernel|to_float_kernel|blur_|small_octaves|half_nn|dog_kernel|extrema_kernel|refine_kernel|orient_kernel|descriptor_kernel"
run() { name=$1; re=$2; shift 2; timeout -s KILL 180 rocprofv3 --pmc "$1" --kernel-include-regex "$re" --output-format csv -d $OUT -o $name -- python3 bench.py "${@:2}" --no-cpu-baseline --steps 10 > $OUT/$name.log 2>&1; }
run sift_f "$SIFT_RE" FETCH_SIZE --only-features && \
run sift_w "$SIFT_RE" WRITE_SIZE --only-features && \
run orb_f "orb_" FETCH_SIZE --only-orb-features && \
run orb_w "orb_" WRITE_SIZE --only-orb-features
echo pmc_rc=$?
