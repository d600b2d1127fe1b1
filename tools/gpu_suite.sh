set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02a/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/r02a/bench.log 2>&1
echo rc=$?
