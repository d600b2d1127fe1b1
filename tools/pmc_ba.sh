#!/bin/bash
# PMC passes over the BA bench leg (one counter group per rocprofv3 run; no trace domains with --pmc).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ba_${1:-r01}
mkdir -p $OUT
B="python bench.py --only-ba --no-cpu-baseline"
run() { name=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex "ba_|chol_" --output-format csv -d $OUT -o $name -- $B > $OUT/$name.log 2>&1; }
run p1 FETCH_SIZE && \
run p2 WRITE_SIZE && \
run p3 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS
echo pmc_rc=$?
