#!/bin/bash
export TMPDIR=/tmp
TAG=${1:-ba}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python bench.py --only-ba --no-cpu-baseline > gpurun_out/prof_$TAG/bench.log 2>&1
echo prof_rc=$?
