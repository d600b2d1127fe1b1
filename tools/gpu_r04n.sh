#!/bin/bash
# r04n: ORB resize on 128 x 32 tiles (two rows per thread), FAST pre-test over rows x lanes: GPU ORB suite,
# features_orb twice, one-stream trace, extraction traffic PMC (for the bench line); then the whole GPU suite,
# smoke and the default bench line on the round's final libraries.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_orb.py -m gpu > $R/gpurun_out/r04n_pytest_orb.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-orb-features --no-cpu-baseline > $R/gpurun_out/r04n_orbf_$i.log 2>&1 || exit 2
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04n_orb1 -o orb1 -- python3 $R/tools/orb_prof.py 32 > $R/gpurun_out/r04n_prof_orb1.log 2>&1) || exit 3
timeout -k 10 800 bash tools/pmc_feat.sh r04n > $R/gpurun_out/r04n_pmc_feat.log 2>&1 || exit 4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $R/gpurun_out/r04n_pytest_gpu.log 2>&1 || exit 5
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r04n_smoke.log 2>&1 || exit 6
timeout -k 10 600 python -u bench.py > $R/gpurun_out/r04n_bench.log 2>&1 || exit 7
echo done
