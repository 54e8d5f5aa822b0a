#!/bin/bash
# Round-2 closing GPU check: the whole -m gpu suite, the default bench line
# (B + B at S=1 + N2, PMC traffic passes, CPU baselines), the config C
# (CohDrift) workload line, and rocprofv3 kernel statistics of B, N2 and C.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -2
grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head -20
[ "$rc" = "0" ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench_full_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_full_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_full_$TAG.log | cut -c1-300
timeout -k 10 600 python bench.py --workload C --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_C_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_C_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_C_$TAG.log | cut -c1-300
for W in B N2 C; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof${W}_$TAG -o kt --output-format csv -- python bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-traffic --no-extra > gpurun_out/prof${W}_$TAG.log 2>&1 || { tail -20 gpurun_out/prof${W}_$TAG.log; exit 1; }
  find gpurun_out/prof${W}_$TAG -name "*kernel_stats.csv" | head -1 | xargs head -4 | cut -d, -f1-4
done
exit 0
