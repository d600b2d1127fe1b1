#!/bin/bash
# r02: screen fold-pipelining A/B (SFMX_SIFT_VARIANT 109/110/111 vs 0): parity of each variant on
# the KATs + oracle cases, then the config-2 two-pass launch (screen / pass-2 split), 2 rounds.
set -o pipefail
OUT=gpurun_out/ab_screen2
mkdir -p $OUT
for v in ${VARIANTS:-109 110 111}; do
  SFMX_SIFT_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/parity_$v.log 2>&1 || exit 1
done
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for r in 1 2; do for v in 0 ${VARIANTS:-109 110 111}; do
  SFMX_SIFT_VARIANT=$v timeout -k 10 200 $B > $OUT/v${v}_$r.log 2>&1 || exit 1
done; done
echo ab_done
