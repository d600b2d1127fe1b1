# SIFT matching: the GPU parity tests (match + full-size C2) and the kernel stats of the matching-only bench
set -o pipefail
TAG=$1
mkdir -p gpurun_out/$TAG
F="--no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-orb-features --no-features"
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fullsize.py -k "not c4_all and not c5" -x -v --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.txt 2>&1 && \
timeout -k 10 300 python bench.py $F > gpurun_out/$TAG/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python bench.py $F > gpurun_out/$TAG/prof.log 2>&1
echo rc=$?
