#!/bin/bash
# r05zg: BA steps on the unscaled iteration-0 records scale what they read (no ba_gschur<SCALEJ> write-back):
# the BA GPU suite and the C5 oracle test, the BA leg x 2, one BA kernel trace, FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_adapter.py "tests/test_gpu_fullsize.py::test_c5_full_ba_matches_oracle" > $R/gpurun_out/r05zg_pytest_ba.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r05zg_ba_$i.log 2>&1 || exit 3
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05zg_ba -o ba -- python3 $R/bench.py --only-ba --no-cpu-baseline --no-ba-calls > $R/gpurun_out/r05zg_prof_ba.log 2>&1) || exit 4
OUT=gpurun_out/pmc_ba_r05zg
mkdir -p $OUT
B="python3 bench.py --only-ba --no-cpu-baseline --no-ba-calls"
run() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "ba_|chol_" --output-format csv -d $OUT -o $name -- $B > $OUT/$name.log 2>&1; }
run p1 FETCH_SIZE && run p2 WRITE_SIZE || exit 5
echo done
