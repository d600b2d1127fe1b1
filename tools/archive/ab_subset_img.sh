# A/B of the SIFT subset pass 2 per (pair, subset) (SFMX_SUBSET_IMG=0) vs per (train image, subset) on the C2 step
set -o pipefail
F="--steps 10 --warmup 3 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
mkdir -p gpurun_out/ab_si
for r in 1 2 3; do
  for w in 0 1; do
    SFMX_SUBSET_IMG=$w timeout -k 10 200 python -u bench.py $F > gpurun_out/ab_si/i${w}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_si/i${w}_$r.log') if l.startswith('{')][-1]; r=d['roofline']; print('per_img $w run $r', round(d['ms_per_step'],3), round(r['kernel_ms_per_launch'],3), round(r['screen_only']['kernel_ms_per_launch'],3), d['matches'], round(r['frac'],4))"
  done
done
