#!/bin/bash
# Feature-extraction leg under different GPU_MAX_HW_QUEUES (HIP hardware queues per process), alternating.
set -o pipefail
F="--steps 3 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs"
for r in 1 2; do
  for q in ${QS:-4 8 16}; do
    GPU_MAX_HW_QUEUES=$q SFMX_FEAT_STREAMS=${S:-8} timeout -k 10 200 python -u bench.py $F > gpurun_out/hwq_${q}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/hwq_${q}_$r.log') if l.startswith('{')][-1]; f=d['features']; print('hwq', $q, $r, round(f['value'],1), f['streams'], f.get('bit_exact_vs_oracle'), 'match_ms', round(d['ms_per_step'],3))"
  done
done
