# A/B of the host-judged (SFMX_BA_SPEC=0) and the speculative device-judged LM on the C5 bench leg, alternating;
# AR1=1: through the multi-rank all-reduce callbacks (torch / RCCL) on a world of one
set -o pipefail
TAG=$1
AR1=${2:-0}
mkdir -p gpurun_out/$TAG
for i in 1 2 3; do
  for m in 0 1; do
    SFMX_BENCH_BA_AR1=$AR1 SFMX_BA_SPEC=$m timeout -k 10 200 python bench.py --only-ba --no-cpu-baseline > gpurun_out/$TAG/spec$m.$i.log 2>&1 || exit 1
    echo "ar1=$AR1 spec=$m run=$i $(grep -o '"value": [0-9.]*' gpurun_out/$TAG/spec$m.$i.log)" >> gpurun_out/$TAG/ab.txt
  done
done
cat gpurun_out/$TAG/ab.txt
