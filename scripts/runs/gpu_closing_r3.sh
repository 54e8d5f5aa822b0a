#!/bin/bash
# Round-3 closing evidence (second pass): smoke, the whole -m gpu suite, the
# default bench line, config C (CohDrift) and C_dxcp lines, kernel statistics.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3y}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -2
grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head -10
[ "$rc" -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_full_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_full_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_full_$TAG.log | cut -c1-200
timeout -k 10 300 python bench.py --workload C_dxcp --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_Cdxcp_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_Cdxcp_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_Cdxcp_$TAG.log | cut -c1-200
timeout -k 10 300 python bench.py --workload C --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_C_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_C_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_C_$TAG.log | cut -c1-200
for W in B N2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof${W}_$TAG -o kt --output-format csv -- python bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-traffic --no-extra > gpurun_out/prof${W}_$TAG.log 2>&1 || { tail -20 gpurun_out/prof${W}_$TAG.log; exit 1; }
done
exit $rc
