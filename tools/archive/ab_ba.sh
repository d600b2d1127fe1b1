#!/bin/bash
# A/B of BA builds, alternating, one box: tools/ab_ba.sh libA.so libB.so [reps]
set -o pipefail
A=$1; B=$2; N=${3:-3}
mkdir -p gpurun_out/ab_ba
for r in $(seq 1 $N); do
  for lib in $A $B; do
    SFMX_LIB_NAME=$lib timeout -k 10 200 python -u bench.py --only-ba --no-cpu-baseline > gpurun_out/ab_ba/${lib%.so}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_ba/${lib%.so}_$r.log') if l.startswith('{')][-1]; print('$lib', $r, round(d['value'],4), {k: round(v,3) for k,v in d['phase_ms_rank0'].items()})"
  done
done
