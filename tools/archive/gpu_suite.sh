set -o pipefail
OUT=${1:-gpurun_out/r02a}
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
echo rc=$?
