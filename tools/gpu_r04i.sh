#!/bin/bash
# r04i: ORB FAST scores from sliding arc minima (+ angle by v_dot4, rBRIEF LDS windows, tiled resize) / maxima on 64 x 32 tiles, blur row sums by v_dot4 from
# aligned words: GPU ORB suite, features_orb, one-stream trace, the PMC instruction counters; the BA host
# setup's phase times on the box's CPU (incremental update 199 -> 200 cameras, diagnostic library);
# then the whole GPU suite, smoke and the default bench line.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r04i_pytest_orb.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04i_orbf.log 2>&1 || exit 2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04i_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r04i_prof_orb1.log 2>&1) || exit 3
timeout -k 10 600 bash tools/pmc_orb_kernels.sh r04i > $R/gpurun_out/r04i_pmc_orbk.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/ba_host_phases.py 8 > $R/gpurun_out/r04i_ba_host_phases.log 2>&1 || exit 5
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $R/gpurun_out/r04i_pytest_gpu.log 2>&1 || exit 6
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r04i_smoke.log 2>&1 || exit 7
timeout -k 10 600 python -u bench.py > $R/gpurun_out/r04i_bench.log 2>&1 || exit 8
echo done
