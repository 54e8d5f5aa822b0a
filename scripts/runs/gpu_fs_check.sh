#!/bin/bash
# fewSamples path check: T(z) / config-E parity tests, then the E_L64 bench
# and its rocprofv3 kernel statistics.  Steps chained with &&, each time-limited.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-fs}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "online_E or tz" > gpurun_out/pytest_gpu_$TAG.log 2>&1 && tail -2 gpurun_out/pytest_gpu_$TAG.log && \
timeout -k 10 300 python bench.py --workload E_L64 --scenes 512 --steps 3 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/bench_E_$TAG.log 2>&1 && tail -1 gpurun_out/bench_E_$TAG.log | cut -c1-200 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profE_$TAG -o kt --output-format csv -- python bench.py --workload E_L64 --scenes 512 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/profE_$TAG.log 2>&1 && echo done
