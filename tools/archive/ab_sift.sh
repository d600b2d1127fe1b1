# A/B of SIFT kernel variants on the C2 matching step (argument: variant list)
V=${@:-"0 96"}
for r in 1 2; do for v in $V; do
SFMX_SIFT_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features > gpurun_out/ab_${v}_$r.log 2>&1 || exit 1
done; done
