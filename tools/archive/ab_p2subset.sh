#!/bin/bash
# r02: subset-restricted pass 2 (SFMX_SIFT_P2=10) -- parity (match tests + C2 all pairs vs oracle),
# then the config-2 two-pass launch A/B against the default pass 2, 2 rounds.
set -o pipefail
OUT=gpurun_out/ab_p2subset
mkdir -p $OUT
SFMX_SIFT_P2=10 timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 --timeout-method thread -k "not c5 and not c4_all" > $OUT/parity.log 2>&1 || { echo parity_failed; exit 1; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for r in 1 2; do for v in 0 10; do
  SFMX_SIFT_P2=$v timeout -k 10 200 $B > $OUT/p${v}_$r.log 2>&1 || exit 1
done; done
echo ab_done
