#!/bin/bash
# r05a: the default bench line with the compact (<= 8 KB) print and the BA parity sample; detail side file.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
SFMX_BENCH_DETAIL=$R/gpurun_out/r05a_bench_detail.json timeout -k 10 600 python -u bench.py > $R/gpurun_out/r05a_bench.log 2>&1 || exit 4
tail -c 9000 $R/gpurun_out/r05a_bench.log
echo done
