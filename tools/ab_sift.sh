for r in 1 2; do for v in 0 6 8; do
SFMX_SIFT_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography > gpurun_out/ab_${v}_$r.log 2>&1 || exit 1
done; done
