#!/bin/bash
# r02 PMC passes on the ORB 2-NN kernels (screen + subset pass 2 + settle) of the config-4 leg;
# summary: python tools/pmc_csv_summary.py OUTDIR > profiles/r02_pmc_orb_c4.json
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_orb2}
mkdir -p $OUT
B="bench.py --workload orb --steps 2 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
run() { name=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "orb_screen16|orb_subset|orb_settle" --output-format csv -d $OUT -o $name -- python3 $B > $OUT/$name.log 2>&1; }
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS && \
run p2 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU && \
run p3 FETCH_SIZE && \
run p4 WRITE_SIZE || { echo pmc_failed; exit 1; }
echo pmc_rc=0
