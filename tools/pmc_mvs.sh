#!/bin/bash
# PMC passes on the undistortion kernel (one counter group per rocprofv3 run).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mvs_${1:-r01}
mkdir -p $OUT
run() { name=$1; shift; timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-include-regex 'undistort|map_kernel' --output-format csv -d $OUT -o $name -- python3 tools/prof_mvs.py > $OUT/$name.log 2>&1; }
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU && \
run p2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_WR && \
run p3 FETCH_SIZE && \
run p4 WRITE_SIZE && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- python3 tools/prof_mvs.py > $OUT/trace.log 2>&1
echo pmc_rc=$?
python3 tools/pmc_csv_summary.py $OUT > $OUT/summary.json
