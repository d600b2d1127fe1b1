#!/bin/bash
# r04b: the round's profiles on the product defaults (one-launch two-pass screens, chol_factor, LDS inner
# sweep, batched ORB extraction): the BA leg vs the r03 library, a C2-only kernel trace of the default
# bench leg (sift_screen16_kernel's average vs roofline.kernel_ms_per_launch), the ORB
# extraction on one stream under a kernel trace (per-kernel breakdown), then the PMC passes -- SIFT C2 and
# ORB C4 2-NN kernels, the extraction legs, the BA leg -- each counter group in its own rocprofv3 run.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--only-ba --no-cpu-baseline --no-ba-calls"
M="--no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/r04b_ba_new_$i.log 2>&1 || exit 1
  SFMX_LIB_NAME=libsfmx_r03.so timeout -k 10 300 python -u bench.py $B > gpurun_out/r04b_ba_r03_$i.log 2>&1 || exit 2
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04b_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py $M > $GRAFT_REPO_ROOT/gpurun_out/r04b_prof_c2.log 2>&1 || exit 3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04b_orb1 -o orb1 -- python3 $GRAFT_REPO_ROOT/tools/orb_prof.py 32 > $GRAFT_REPO_ROOT/gpurun_out/r04b_prof_orb1.log 2>&1 || exit 4
cd $GRAFT_REPO_ROOT
timeout -k 10 600 bash tools/pmc_match.sh sift r04 > gpurun_out/r04b_pmc_sift.log 2>&1 || exit 5
timeout -k 10 600 bash tools/pmc_match.sh orb r04 > gpurun_out/r04b_pmc_orb.log 2>&1 || exit 6
timeout -k 10 800 bash tools/pmc_feat.sh r04 > gpurun_out/r04b_pmc_feat.log 2>&1 || exit 7
timeout -k 10 600 bash tools/pmc_ba.sh r04 > gpurun_out/r04b_pmc_ba.log 2>&1 || exit 8
echo done
