#!/bin/bash
# r03n: round-3 closing measurements on one GPU: full GPU suite + smoke, the default bench line, kernel
# stats of the whole bench, BA PMC traffic, 2-rank rehearsal (both ranks on cuda:0, gloo collectives)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r03n_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03n_smoke.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > gpurun_out/r03n_bench.log 2>&1 || exit 3
bash tools/pmc_ba.sh r03n > gpurun_out/r03n_pmc_ba.log 2>&1 || exit 4
SFMX_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03n_rehearse_2rank.log 2>&1 || exit 5
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03n -o all -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r03n_prof.log 2>&1 || exit 6
echo done
