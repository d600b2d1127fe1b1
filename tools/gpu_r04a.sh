#!/bin/bash
# r04a: first GPU session of round 4: the whole GPU suite (new: tiny point groups after other solves,
# native RCCL world of one, refused update, 2-rank multi-camera sharding; landed r03 patches: chol
# inner sweep by cross-lane moves + ba_glin padding rows, ORB retainBest on the device), smoke, the
# default bench line, a C2-only kernel trace, and A/Bs of the BA and ORB-extraction legs vs r03's library
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r04a_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a_smoke.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > gpurun_out/r04a_bench.log 2>&1 || exit 3
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r04a_bench_ba_new_$i.log 2>&1 || exit 4
  SFMX_LIB_NAME=libsfmx_r03.so timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline --no-ba-calls > gpurun_out/r04a_bench_ba_r03_$i.log 2>&1 || exit 5
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > gpurun_out/r04a_bench_orbf_new_$i.log 2>&1 || exit 6
  SFMX_LIB_NAME=libsfmx_r03.so timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > gpurun_out/r04a_bench_orbf_r03_$i.log 2>&1 || exit 7
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04a_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-ba --no-orb --no-c3 --no-homography --no-f4 --no-mvs --no-features --no-orb-features > $GRAFT_REPO_ROOT/gpurun_out/r04a_prof_c2.log 2>&1 || exit 8
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04a_ba -o ba -- python3 $GRAFT_REPO_ROOT/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $GRAFT_REPO_ROOT/gpurun_out/r04a_prof_ba.log 2>&1 || exit 9
echo done
