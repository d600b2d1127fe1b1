#!/bin/bash
# r02: ORB subset-restricted pass 2 (default, SFMX_ORB_VARIANT=0) vs the r01 512-query pass 2 (12):
# parity (match tests + C4 all pairs + ORB CLI replay), then the config-4 launch A/B, 2 rounds.
set -o pipefail
OUT=gpurun_out/ab_orb_subset
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fullsize.py tests/test_gpu_cli.py -m gpu -x -v --timeout 200 --timeout-method thread -k "not c5 and not c2_all" > $OUT/parity.log 2>&1 || { echo parity_failed; exit 1; }
B="python bench.py --workload orb --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
for r in 1 2; do for v in 12 0; do
  SFMX_ORB_VARIANT=$v timeout -k 10 200 $B > $OUT/v${v}_$r.log 2>&1 || exit 1
done; done
echo ab_done
