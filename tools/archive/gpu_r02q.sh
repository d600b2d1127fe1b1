# r02q verification: full GPU suite, smoke, bench, a 2-rank one-GPU rehearsal of every bench leg, and the
# rocprofv3 kernel stats of the bench command
set -o pipefail
OUT=gpurun_out/r02q
mkdir -p $OUT
bash tools/gpu_suite.sh $OUT && \
SFMX_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/rehearse_2rank.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline > $OUT/bench_profiled.log 2>&1
echo rc=$?
