set -o pipefail
TAG=$1
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/$TAG/prof_hip -o run -- python bench.py --only-ba --no-cpu-baseline > gpurun_out/$TAG/prof_hip.log 2>&1
echo rc=$?
