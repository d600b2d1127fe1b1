#!/bin/bash
# BA tests + BA bench + rocprofv3 kernel stats of the BA leg (GPU box; tooling)
TAG=${1:-r02}
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_ba.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --only-ba --steps 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_ba.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o ba -- python3 bench.py --only-ba --steps 3 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
