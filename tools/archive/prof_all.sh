#!/bin/bash
# Kernel-trace + stats of the full bench (SIFT C2 + BA C5) -> gpurun_out/prof_<tag>/
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG/bench.log 2>&1
echo prof_rc=$?
