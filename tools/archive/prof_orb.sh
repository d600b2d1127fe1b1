#!/bin/bash
# ORB extraction: GPU tests, CLI replay, ORB bench leg + rocprofv3 kernel stats (GPU box; tooling)
TAG=${1:-r02}
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_cli.py -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_orb_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only-orb-features --steps 10 > gpurun_out/${TAG}_bench_orb.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o orb -- python3 bench.py --only-orb-features --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_prof_orb.log 2>&1
