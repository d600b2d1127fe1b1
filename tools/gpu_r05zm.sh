#!/bin/bash
# r05zm: extraction legs against the worker-stream count (SFMX_FEAT_STREAMS 4 / 8 / 16), twice each.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for s in 4 8 16; do
    SFMX_FEAT_STREAMS=$s timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r05zm_orbf_s${s}_$i.log 2>&1 || exit 2
    SFMX_FEAT_STREAMS=$s timeout -k 10 300 python -u bench.py --only-features --no-cpu-baseline > $R/gpurun_out/r05zm_sift_s${s}_$i.log 2>&1 || exit 3
  done
done
echo done
