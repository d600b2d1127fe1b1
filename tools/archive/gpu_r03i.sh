#!/bin/bash
# r03i: BA phase stamps (diagnostic stamp builds) of the current and the r03-base kernels
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ba_stamps.py > gpurun_out/r03i_stamps_new.txt 2>&1 || exit 1
SFMX_LIB_NAME=libsfmx_stamps_base.so timeout -k 10 300 python -u tools/ba_stamps.py > gpurun_out/r03i_stamps_base.txt 2>&1 || exit 2
echo done
