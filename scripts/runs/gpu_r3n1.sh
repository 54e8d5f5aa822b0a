#!/bin/bash
# Round-3 N1 check: the resident engine's GPU tests, the default bench line
# (B, B at S=1 launch-per-round / grid / resident, N2) and rocprofv3 kernel
# statistics of the resident single-WASN run.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3n1}
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_modes.py -m gpu -v -s -x -k "resident" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_res_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_res_$TAG.log | tail -2
grep -E "resident w|FAILED|Error" gpurun_out/pytest_res_$TAG.log | head -10
[ "$rc" -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload B --scenes 1 --resident --no-extra --no-cpu-baseline --no-traffic --steps 5 --warmup 2 > gpurun_out/bench_res_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_res_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_res_$TAG.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profres_$TAG -o kt --output-format csv -- python bench.py --workload B --scenes 1 --resident --no-extra --no-cpu-baseline --no-traffic --steps 2 --warmup 1 > gpurun_out/profres_$TAG.log 2>&1 || { tail -20 gpurun_out/profres_$TAG.log; exit 1; }
find gpurun_out/profres_$TAG -name "*kernel_stats.csv" | head -1 | xargs head -8 | cut -d, -f1-4
timeout -k 10 900 python bench.py > gpurun_out/bench_full_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_full_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_full_$TAG.log | cut -c1-300
exit $rc
