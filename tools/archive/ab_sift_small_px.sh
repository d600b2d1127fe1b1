# fused small-octave launch: the size limit sweep (SFMX_SIFT_SMALL_PX) against per-octave launches
set -o pipefail
F="--steps 3 --warmup 1 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-orb-features"
mkdir -p gpurun_out/ab_sp
for r in 1 2; do
  for px in 0 512 2048 8192; do
    if [ $px = 0 ]; then v=0; else v=1; fi
    SFMX_SIFT_SMALL=$v SFMX_SIFT_SMALL_PX=$px timeout -k 10 300 python -u bench.py $F > gpurun_out/ab_sp/p${px}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_sp/p${px}_$r.log') if l.startswith('{')][-1]['features']; print('small_px $px run $r', round(d['value'],1), d['unit'])"
  done
done
