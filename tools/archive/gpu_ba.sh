set -o pipefail
TAG=$1
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_fullsize.py -k "ba or c5" -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_ba.txt 2>&1 && \
timeout -k 10 300 python bench.py --only-ba --no-cpu-baseline > gpurun_out/$TAG/bench_ba.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof_ba -o run -- python bench.py --only-ba --no-cpu-baseline > gpurun_out/$TAG/prof_ba.log 2>&1 && \
bash tools/pmc_ba.sh $TAG
echo rc=$?
