#!/bin/bash
# A/B of two in-tree builds on the openMVS-export (undistortion) leg, alternating, one box:
# lib/libsfmx_prev.so (built from an earlier commit by the caller) vs lib/libsfmx.so.
set -o pipefail
F="--steps 20 --warmup 3 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-features"
for r in 1 2 3; do
  for lib in ${LIBS:-libsfmx_prev.so libsfmx.so}; do
    SFMX_LIB_NAME=$lib timeout -k 10 200 python -u bench.py $F > gpurun_out/abm_${lib%.so}_$r.log 2>&1 || exit 1
    python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/abm_${lib%.so}_$r.log') if l.startswith('{')][-1]['mvs']; print('$lib', $r, round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_per_launch'],3), round(d['distinct_cameras']['kernel_ms_per_launch'],3), d.get('bit_exact_vs_oracle'))"
  done
done
