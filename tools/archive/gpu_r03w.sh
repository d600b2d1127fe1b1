#!/bin/bash
# r03w: ORB extraction with retainBest on the device (one host wait per image): ORB parity suite vs
# the oracle, smoke, the ORB extraction bench leg (r03n: 4485 images/s), its kernel stats
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_orb.py > gpurun_out/r03w_orb.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03w_smoke.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features > gpurun_out/r03w_bench_orbf_$i.log 2>&1 || exit 3
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03w -o orbf -- python3 $GRAFT_REPO_ROOT/bench.py --only-orb-features --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r03w_prof.log 2>&1 || exit 4
echo done
