#!/bin/bash
# r05ze: kernel traces of the SIFT features leg, XCD-contiguous (product) vs plain grids (diagnostic,
# SFMX_SIFT_XCD=0), twice in alternation; one stream (SFMX_FEAT_STREAMS=1) so the durations are the kernels'.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
prof() { tag=$1; shift; (cd /tmp && env SFMX_FEAT_STREAMS=1 "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05ze_$tag -o feat -- python3 $R/bench.py --only-features --no-cpu-baseline --steps 4 > $R/gpurun_out/r05ze_prof_$tag.log 2>&1); }
for i in 1 2; do
  prof xcd_$i SFMX_X=0 || exit 3
  prof plain_$i SFMX_LIB_NAME=libsfmx_diag.so SFMX_SIFT_XCD=0 || exit 4
done
echo done
