#!/bin/bash
# r05d: the box's CPU share, and the BA call replay under host-pool settings (threads, spin) and the
# pieced get (A/B of the r05 host setup knobs; product defaults: 16 threads, 3000 us spin, 4 pieces).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$R/gpurun_out/r05d_env.txt
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; lscpu | head -20; } > $O 2>&1
for cfg in "16 3000 4" "16 0 4" "12 3000 4" "8 3000 4" "16 3000 1" "16 300 1"; do
  set -- $cfg
  SFMX_HOST_THREADS=$1 SFMX_HOST_SPIN_US=$2 SFMX_BA_GET_PIECES=$3 timeout -k 10 300 python -u bench.py --only-ba --no-cpu-baseline > $R/gpurun_out/r05d_ba_t$1_s$2_g$3.log 2>&1 || exit 3
done
echo done
