#!/bin/bash
# Correctness + timing of each SIFT kernel variant (SFMX_SIFT_VARIANT), one process each.
mkdir -p gpurun_out/tune
for v in ${VARIANTS:-0 1 2 3 4}; do
  SFMX_SIFT_VARIANT=$v timeout -k 10 200 python -m pytest tests/test_gpu_match.py -q -x -k "golden or ragged or full_size_sift" > gpurun_out/tune/pytest_v$v.log 2>&1 || { echo "pytest v$v failed"; exit 1; }
  SFMX_SIFT_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ba > gpurun_out/tune/bench_v$v.log 2>&1 || { echo "bench v$v failed"; exit 1; }
done
echo done
