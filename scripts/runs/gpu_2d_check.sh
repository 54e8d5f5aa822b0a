#!/bin/bash
# GPU check of the two-dimensional GEVD solver: full -m gpu suite, then
# rocprofv3 kernel statistics of the N2 (online K=32x8, D=39) and D (batch
# K=32x8) workloads.  Every GPU step is time-limited; the chain stops at the
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
for W in N2 D; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof${W}_$TAG -o kt --output-format csv -- python bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-traffic --no-extra > gpurun_out/prof${W}_$TAG.log 2>&1 || { tail -20 gpurun_out/prof${W}_$TAG.log; exit 1; }
  tail -1 gpurun_out/prof${W}_$TAG.log | cut -c1-300
  find gpurun_out/prof${W}_$TAG -name "*kernel_stats.csv" | head -1 | xargs head -5 | cut -d, -f1-6
done
exit $rc
