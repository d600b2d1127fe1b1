# extraction legs: 8 vs 16 worker streams (SFMX_FEAT_STREAMS), alternating, SIFT (features) and ORB (features_orb)
set -o pipefail
F="--steps 3 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs"
mkdir -p gpurun_out/ab_fs
for r in 1 2 3; do
  for n in 8 16; do
    SFMX_FEAT_STREAMS=$n timeout -k 10 300 python -u bench.py $F > gpurun_out/ab_fs/n${n}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_fs/n${n}_$r.log') if l.startswith('{')][-1]; print('streams $n run $r sift', round(d['features']['value'],1), 'orb', round(d['features_orb']['value'],1), d['features']['bit_exact_vs_oracle'], d['features_orb']['bit_exact_vs_oracle'])"
  done
done
