#!/bin/bash
# Screening-pass shape A/B (r01g): parity of the 16x16x64 variants, then kernel ms of
# each variant on config 2 (2 rounds), then the operand-bit probe (SFMX_PROBE_XOR80).
set -o pipefail
mkdir -p gpurun_out/ab
for v in 106 107 108; do
  SFMX_SIFT_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/parity_$v.log 2>&1 || exit 1
done
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features"
for r in 1 2; do for v in ${VARIANTS:-0 106 107 108}; do
  SFMX_SIFT_VARIANT=$v timeout -k 10 200 $B > gpurun_out/ab/v${v}_$r.log 2>&1 || exit 1
done; done
for v in 0 106; do
  SFMX_PROBE_XOR80=1 SFMX_SIFT_VARIANT=$v timeout -k 10 200 $B > gpurun_out/ab/xor_v${v}.log 2>&1 || exit 1
done
echo ab_done
