#!/bin/bash
# Instruction / wait / LDS counters of the ORB extraction kernels (tools/orb_prof.py, one stream), one
# counter group per rocprofv3 run (no trace domains with --pmc) -> gpurun_out/pmc_orbk_<tag>/;
# summarise with tools/pmc_csv_summary.py.  (tooling)
set -o pipefail
export TMPDIR=/tmp
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/pmc_orbk_${1:-r04}
mkdir -p $OUT
run() { name=$1; shift; (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $@ --kernel-include-regex "orb_" --output-format csv -d $OUT -o $name -- python3 $R/tools/orb_prof.py 16 > $OUT/$name.log 2>&1); }
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE && \
run b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU && \
run f FETCH_SIZE && \
run w WRITE_SIZE
echo pmc_rc=$?
