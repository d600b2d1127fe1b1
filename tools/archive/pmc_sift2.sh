#!/bin/bash
# r02 PMC passes on the SIFT 2-NN kernels (screen + subset pass 2 + settle) of the config-2 leg and,
# with --only-c3, of the config-3 leg: one counter group per rocprofv3 run, no trace domains with
# --pmc.  Summaries: python tools/pmc_csv_summary.py DIR > profiles/r02_pmc_sift_{c2,c3}.json
# usage: tools/pmc_sift2.sh OUTDIR
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_sift2}
mkdir -p $OUT/c2 $OUT/c3
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
B3="bench.py --steps 2 --warmup 1 --no-cpu-baseline --only-c3"
run() { d=$1; name=$2; shift 2; timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "sift_screen16|sift_subset|sift_settle" --output-format csv -d $OUT/$d -o $name -- python3 $ARGS > $OUT/$d/$name.log 2>&1; }
for d in c2 c3; do
  if [ $d = c2 ]; then ARGS=$B; else ARGS=$B3; fi
  run $d p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS && \
  run $d p2 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU && \
  run $d p3 FETCH_SIZE && \
  run $d p4 WRITE_SIZE || { echo pmc_failed_$d; exit 1; }
done
echo pmc_rc=0
