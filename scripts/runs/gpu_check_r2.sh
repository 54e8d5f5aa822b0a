#!/bin/bash
# GPU check: parity suite, then a short config-B bench and its rocprofv3
# kernel statistics.  Every GPU step is time-limited; the chain stops at the
# first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -3
grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head -20
[ "$rc" = "0" ] || [ -n "$BENCH_ANYWAY" ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs head -8 | cut -d, -f1-6
exit $rc
