#!/bin/bash
# r04b: the round's PMC passes on the current kernels: SIFT C2 and ORB C4
# 2-NN kernels (FETCH_SIZE / WRITE_SIZE + MFMA busy), the extraction legs and the BA leg, each counter
# group in its own rocprofv3 run (no trace domains with --pmc); first the chol tile micro-benchmark (phase stamps
# of one 64 x 64 diagonal-tile inverse, tools/micro/chol_tile.hip, prebuilt in-tree).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 tools/micro/chol_tile > gpurun_out/r04b_chol_tile.txt 2>&1 || exit 9
timeout -k 10 600 bash tools/pmc_match.sh sift r04 > gpurun_out/r04b_pmc_sift.log 2>&1 || exit 1
timeout -k 10 600 bash tools/pmc_match.sh orb r04 > gpurun_out/r04b_pmc_orb.log 2>&1 || exit 2
timeout -k 10 800 bash tools/pmc_feat.sh r04 > gpurun_out/r04b_pmc_feat.log 2>&1 || exit 3
timeout -k 10 600 bash tools/pmc_ba.sh r04 > gpurun_out/r04b_pmc_ba.log 2>&1 || exit 4
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04b_orbf -o orbf -- python3 $GRAFT_REPO_ROOT/bench.py --only-orb-features --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r04b_prof_orbf.log 2>&1 || exit 5
echo done
