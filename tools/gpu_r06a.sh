#!/bin/bash
# r06a: the bench launcher on the box: `bench.py --gpus 2` with no WORLD_SIZE starts two ranks itself
# (SFMX_BENCH_REHEARSE=1: both on cuda:0, collectives over gloo), strong + weak BA; then the 1-GPU BA leg.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
SFMX_BENCH_DETAIL=$R/gpurun_out/r06a_rehearse_detail.json SFMX_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06a_rehearse_2rank.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r06a_ba.log 2>&1 || exit 3
tail -c 3000 $R/gpurun_out/r06a_rehearse_2rank.log
echo done
