set -o pipefail
bash tools/pmc_orb2.sh gpurun_out/r02m/pmc_orb && \
bash tools/gpu_suite.sh gpurun_out/r02m
