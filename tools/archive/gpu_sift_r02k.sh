set -o pipefail
mkdir -p gpurun_out/r02k
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fullsize.py tests/test_gpu_adapter.py tests/test_gpu_cli.py -m gpu -x -v --timeout 200 --timeout-method thread -k "not c5" > gpurun_out/r02k/pytest_match.txt 2>&1 && \
bash tools/pmc_sift2.sh gpurun_out/r02k/pmc && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02k/prof -o sift -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ba --no-orb --no-homography --no-f4 --no-mvs --no-features --no-orb-features > gpurun_out/r02k/prof_bench.log 2>&1
echo rc=$?
