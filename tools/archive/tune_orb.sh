#!/bin/bash
# ORB FP4-MFMA kernel variants on BASELINE config 4 (tuning only; results -> gpurun_out/tune_orb.txt).
# VARIANTS (default "0 5 8"): 0 = two-pass (16x16x128 screen + 512-query pass-2 items),
# 5/6 = single-pass 16x16x128, 8/2-4 = single-pass 32x32x64.  Each variant's
# ORB parity tests run first (the variant is read once per process).
set -o pipefail
out=gpurun_out/tune_orb.txt
: > $out
for v in ${VARIANTS:-0 5 8}; do
  SFMX_ORB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q -k orb --timeout 120 --timeout-method thread > gpurun_out/tune_orb_parity_$v.log 2>&1 || exit 1
done
for r in 1 2; do for v in ${VARIANTS:-0 5 8}; do
  SFMX_ORB_VARIANT=$v timeout -k 10 200 python bench.py --workload orb --no-ba --no-cpu-baseline --steps 5 > gpurun_out/tune_orb_$v.log 2>&1 || exit 1
  python -c "
import json,sys
l=[x for x in open('gpurun_out/tune_orb_$v.log') if x.startswith('{')][-1]; d=json.loads(l)
print('variant $v', round(d['roofline']['kernel_ms_per_launch'],3), 'ms', round(d['roofline']['frac'],3), d['matches'])" >> $out
done; done
cat $out
