# ORB extraction leg: worker-stream count sweep (SFMX_FEAT_STREAMS)
set -o pipefail
mkdir -p gpurun_out/ab_os
for r in 1 2; do
  for n in 8 16 32; do
    SFMX_FEAT_STREAMS=$n timeout -k 10 300 python -u bench.py --only-orb-features > gpurun_out/ab_os/n${n}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_os/n${n}_$r.log') if l.startswith('{')][-1]; print('streams $n run $r', round(d['value'],1), d['unit'], d.get('bit_exact_vs_oracle'))"
  done
done
