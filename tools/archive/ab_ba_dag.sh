# A/B of the per-level factorization launches (SFMX_BA_DAG=0) and chol_factor (the whole factorization in one
# launch, SFMX_BA_DAG=1) on the C5 bench leg, alternating; first the bit-identity test of every solve form
set -o pipefail
TAG=$1
mkdir -p gpurun_out/$TAG
timeout -k 10 200 python -u -m pytest tests/test_gpu_ba.py -k "bit_identical_to_r02_forms" -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.txt 2>&1 || exit 1
for i in 1 2 3; do
  for m in 0 1; do
    SFMX_BA_DAG=$m timeout -k 10 200 python bench.py --only-ba --no-cpu-baseline > gpurun_out/$TAG/dag$m.$i.log 2>&1 || exit 1
    echo "dag=$m run=$i $(grep -o '"value": [0-9.]*' gpurun_out/$TAG/dag$m.$i.log | head -1)" >> gpurun_out/$TAG/ab.txt
  done
done
cat gpurun_out/$TAG/ab.txt
