#!/bin/bash
# PMC passes over the BA bench leg (one counter group per rocprofv3 run; no trace domains with --pmc).
# -> gpurun_out/pmc_ba_<tag>/p*_counter_collection.csv ; summarise with tools/pmc_summary.py
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ba_${1:-r02}
mkdir -p $OUT
B="python3 bench.py --only-ba --no-cpu-baseline --no-ba-calls"
run() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "ba_|chol_" --output-format csv -d $OUT -o $name -- $B > $OUT/$name.log 2>&1; }
run p1 FETCH_SIZE && \
run p2 WRITE_SIZE && \
run p3 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS && \
run p4 SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT
echo pmc_rc=$?
