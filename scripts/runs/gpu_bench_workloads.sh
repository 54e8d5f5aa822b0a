#!/bin/bash
# Bench lines for the non-default workloads (config E fewSamples at 512
# scenes per GPU, config D batch K=32 x 8) with their rocprofv3 kernel
# statistics.  Every GPU step has its own time limit; the chain stops at the
# first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-w1}
timeout -k 10 300 python bench.py --workload E_L64 --scenes 512 --steps 3 --warmup 1 --no-traffic > gpurun_out/bench_E_$TAG.log 2>&1 || { echo "bench E failed"; tail -30 gpurun_out/bench_E_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_E_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profE_$TAG -o kt --output-format csv -- python bench.py --workload E_L64 --scenes 512 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/profE_$TAG.log 2>&1 || { echo "rocprof E failed"; tail -30 gpurun_out/profE_$TAG.log; exit 1; }
timeout -k 10 300 python bench.py --workload D --scenes 1 --steps 3 --warmup 1 > gpurun_out/bench_D_$TAG.log 2>&1 || { echo "bench D failed"; tail -30 gpurun_out/bench_D_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_D_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profD_$TAG -o kt --output-format csv -- python bench.py --workload D --scenes 1 --steps 1 --warmup 1 > gpurun_out/profD_$TAG.log 2>&1 || { echo "rocprof D failed"; tail -30 gpurun_out/profD_$TAG.log; exit 1; }
echo done
