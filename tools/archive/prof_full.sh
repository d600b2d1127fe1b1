set -o pipefail
TAG=$1
mkdir -p gpurun_out/$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof_full -o run -- python3 bench.py > gpurun_out/$TAG/prof_full_bench.log 2>&1
echo rc=$?
