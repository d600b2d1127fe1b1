#!/bin/bash
# parity + A/B timing of SIFT kernel variants (SFMX_SIFT_VARIANT)
for v in 20 21; do
SFMX_SIFT_VARIANT=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py -k "sift or l2" > gpurun_out/pipe_t_$v.log 2>&1 || { echo "parity_fail $v"; exit 1; }
done
for r in 1 2; do for v in 0 20 21 22 23; do
SFMX_SIFT_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs > gpurun_out/pipe_${v}_$r.log 2>&1 || exit 1
done; done
echo ab_done
