#!/bin/bash
# r05zw: counters of the BA per-step reduction kernels (ba_camred, ba_finalize, ba_assemble), to explain
# ba_camred's 17.7 us (r05zt / r05zu: neither unrolling nor LDS-staged slot lists changed it).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
export TMPDIR=/tmp
OUT=gpurun_out/pmc_r05zw
mkdir -p $OUT
B="python3 bench.py --only-ba --no-cpu-baseline --no-ba-calls"
run() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "ba_camred|ba_finalize|ba_assemble" --output-format csv -d $OUT -o $name -- $B > $OUT/$name.log 2>&1; }
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS && \
run p2 FETCH_SIZE && run p3 TCC_HIT_sum TCC_MISS_sum && run p4 GRBM_GUI_ACTIVE GRBM_COUNT || exit 2
echo done
