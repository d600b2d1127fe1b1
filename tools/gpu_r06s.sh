#!/bin/bash
# r06s: ba_finalize phase stamps (stamp library)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ba_stamps.py > $R/gpurun_out/r06s_ba_stamps.txt 2>&1 || exit 4
cat $R/gpurun_out/r06s_ba_stamps.txt
