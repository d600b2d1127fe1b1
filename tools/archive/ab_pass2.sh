#!/bin/bash
# Pass-2 item-size A/B (r01g): parity per variant, then kernel ms on config 2 (2 rounds).
set -o pipefail
mkdir -p gpurun_out/ab2
for p in ${P2:-1 2 3}; do
  SFMX_SIFT_P2=$p timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2/parity_$p.log 2>&1 || exit 1
done
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features"
for r in 1 2; do for p in 0 ${P2:-1 2 3}; do
  SFMX_SIFT_P2=$p timeout -k 10 200 $B > gpurun_out/ab2/p${p}_$r.log 2>&1 || exit 1
done; done
echo ab_done
