#!/bin/bash
# GPU round: parity tests, bench (default workload), rocprofv3 kernel stats of
# the same bench, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) for the
# update kernel's HBM traffic.  Every GPU step has its own time limit and the
# chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r1}
BENCH_ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -2 gpurun_out/bench_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof kt failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-graph --no-traffic > gpurun_out/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -30 gpurun_out/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-graph --no-traffic > gpurun_out/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed"; tail -30 gpurun_out/pmc_write_$TAG.log; exit 1; }
find gpurun_out -name "*.csv" | head -50
echo done
