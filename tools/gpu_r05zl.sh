#!/bin/bash
# r05zl: the default bench command under rocprofv3 --kernel-trace --stats (the headline kernel's average
# duration from the same command whose line reports it); the printed line kept beside the trace.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && SFMX_BENCH_DETAIL=$R/gpurun_out/r05zl_bench_detail.json timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zl_bench -o bench -- python3 $R/bench.py > $R/gpurun_out/r05zl_bench.log 2>&1) || exit 2
echo done
