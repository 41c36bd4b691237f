set -e
timeout -k 10 300 python bench.py --no-cpu-baseline --ba-calls 0 > gpurun_out/bench_now.log 2>&1
echo bench ok
OUT=gpurun_out/pmc_now BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --ba-calls 0" bash tools/pmc_kernel.sh
