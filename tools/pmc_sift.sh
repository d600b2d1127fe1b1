#!/bin/bash
# PMC passes on the SIFT 2-NN kernel (one counter group per rocprofv3 run; no trace domains with --pmc).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-r01}
mkdir -p $OUT
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
run() { name=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex "sift_knn2" --output-format csv -d $OUT -o $name -- $B > $OUT/$name.log 2>&1; }
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS && \
run p2 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM && \
run p3 FETCH_SIZE && \
run p4 WRITE_SIZE && \
run p5 TCC_HIT_sum TCC_MISS_sum
echo pmc_rc=$?
