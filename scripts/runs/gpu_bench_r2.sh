#!/bin/bash
# Full default bench line (B at S=31 + the single-WASN B and N2 lines, PMC
# traffic passes and CPU baselines), then rocprofv3 kernel statistics of the
# N2 workload alone.  Optional PYTEST_K runs a GPU test selection first.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2}
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "$PYTEST_K" > gpurun_out/pytest_sel_$TAG.log 2>&1 || { grep -E "passed|failed|Error" gpurun_out/pytest_sel_$TAG.log | tail -5; exit 1; }
  grep -E "passed|failed" gpurun_out/pytest_sel_$TAG.log | tail -2
fi
timeout -k 10 900 python bench.py > gpurun_out/bench_full_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_full_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_full_$TAG.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profN2_$TAG -o kt --output-format csv -- python bench.py --workload N2 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/profN2_$TAG.log 2>&1 || { tail -20 gpurun_out/profN2_$TAG.log; exit 1; }
find gpurun_out/profN2_$TAG -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -d, -f1-6
