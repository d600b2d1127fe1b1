#!/bin/bash
# PMC passes on a matching 2-NN kernel (one counter group per rocprofv3 run; no trace domains with --pmc).
# usage: tools/pmc_match.sh sift|orb TAG   (-> tools/pmc_csv_summary.py; bench.py PMC_FILES takes per-launch sums)
set -o pipefail
export TMPDIR=/tmp
KIND=${1:-sift}
OUT=gpurun_out/pmc_${KIND}_${2:-r01}
mkdir -p $OUT
if [ "$KIND" = orb ]; then RE="orb_screen|orb_subset|orb_settle"; else RE="sift_screen|sift_subset|sift_settle"; fi
B="python bench.py --workload $KIND --steps 2 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
run() { name=$1; shift; timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" --output-format csv -d $OUT -o $name -- $B > $OUT/$name.log 2>&1; }
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS && \
run p2 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES && \
run p3 FETCH_SIZE && \
run p4 WRITE_SIZE
echo pmc_rc=$?
