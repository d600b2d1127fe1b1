#!/bin/bash
# A/B of two in-tree builds on the config-2 matching step, alternating, one box:
# lib/libsfmx_prev.so (built from an earlier commit by the caller) vs lib/libsfmx.so.
set -o pipefail
F="--steps 10 --warmup 3 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features"
for r in 1 2 3; do
  for lib in libsfmx_prev.so libsfmx.so; do
    SFMX_LIB_NAME=$lib timeout -k 10 200 python -u bench.py $F > gpurun_out/ab_${lib%.so}_$r.log 2>&1 || exit 1
    python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/ab_${lib%.so}_$r.log') if l.startswith('{')][-1]; print('$lib', $r, round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_per_launch'],3))"
  done
done
