#!/bin/bash
# A/B of two in-tree builds on the SIFT extraction leg, alternating, one box:
# lib/libsfmx_prev.so (built from an earlier commit by the caller) vs lib/libsfmx.so.
set -o pipefail
F="--steps 3 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs"
for r in 1 2 3; do
  for lib in ${LIBS:-libsfmx_prev.so libsfmx.so}; do
    SFMX_LIB_NAME=$lib timeout -k 10 200 python -u bench.py $F > gpurun_out/abx_${lib%.so}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/abx_${lib%.so}_$r.log') if l.startswith('{')][-1]['features']; print('$lib', $r, round(d['value'],1), 'images/s', round(d['kernel_ms_per_image'],3), 'kernel ms/image')"
  done
done
