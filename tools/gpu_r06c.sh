#!/bin/bash
# r06c: chol_factor timeline at C5 (diagnostic library, tools/chol_trace.py)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
SFMX_LIB_NAME=libsfmx_diag.so timeout -k 10 300 python -u tools/chol_trace.py > $R/gpurun_out/r06c_chol_trace.txt 2>&1 || exit 2
cat $R/gpurun_out/r06c_chol_trace.txt
