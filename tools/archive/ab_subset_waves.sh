# A/B of the SIFT subset pass-2 workgroup size (SFMX_SUBSET_WAVES 4 / 2) on the C2 step, alternating, one box
set -o pipefail
F="--steps 10 --warmup 3 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features"
mkdir -p gpurun_out/ab_sw
for r in 1 2 3; do
  for w in 4 2; do
    SFMX_SUBSET_WAVES=$w timeout -k 10 200 python -u bench.py $F > gpurun_out/ab_sw/w${w}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_sw/w${w}_$r.log') if l.startswith('{')][-1]; r=d['roofline']; print('waves $w run $r', round(d['ms_per_step'],3), round(r['kernel_ms_per_launch'],3), round(r['screen_only']['kernel_ms_per_launch'],3), d['matches'])"
  done
done
