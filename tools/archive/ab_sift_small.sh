# A/B of the fused small-octave launch (SFMX_SIFT_SMALL=1, default) vs per-octave launches on the SIFT extraction leg
set -o pipefail
F="--steps 3 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-orb-features"
mkdir -p gpurun_out/ab_ss
for r in 1 2 3; do
  for v in 0 1; do
    SFMX_SIFT_SMALL=$v timeout -k 10 300 python -u bench.py $F > gpurun_out/ab_ss/s${v}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_ss/s${v}_$r.log') if l.startswith('{')][-1]['features']; print('small $v run $r', round(d['value'],1), d['unit'], d.get('bit_exact_vs_oracle'), round(d['roofline']['frac'],4))"
  done
done
