#!/bin/bash
# ORB FP4-MFMA kernel variants on BASELINE config 4 (tuning only; results -> gpurun_out/tune_orb.txt)
set -e
out=gpurun_out/tune_orb.txt
: > $out
for v in 0 2 3 4; do
  SFMX_ORB_VARIANT=$v timeout -k 10 120 python bench.py --workload orb --no-ba --no-cpu-baseline --steps 5 > gpurun_out/tune_orb_$v.log 2>&1
  python -c "
import json,sys
l=[x for x in open('gpurun_out/tune_orb_$v.log') if x.startswith('{')][-1]; d=json.loads(l)
print('variant $v', round(d['roofline']['kernel_ms_per_launch'],3), 'ms', round(d['roofline']['frac'],3), d['matches'])" >> $out
done
cat $out
