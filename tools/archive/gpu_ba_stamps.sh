set -o pipefail
mkdir -p gpurun_out/$1
timeout -k 10 300 python tools/ba_stamps.py > gpurun_out/$1/ba_stamps.txt 2>&1
echo rc=$?
