#!/bin/bash
# PMC passes on the SIFT 2-NN kernels of the config-2 leg: the two-pass path's screen + pass-2 kernels
# (one counter group per rocprofv3 run; no trace domains with --pmc).
# usage: tools/pmc_sift.sh TAG   (SFMX_SIFT_VARIANT selects the kernel variant)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-r01}
mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features"
run() { name=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex "sift_knn2|sift_screen" --output-format csv -d $OUT -o $name -- $B > $OUT/$name.log 2>&1; }
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS && \
run p2 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES && \
run p3 FETCH_SIZE && \
run p4 WRITE_SIZE && \
run p5 SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU
echo pmc_rc=$?
