#!/bin/bash
# pytest -m gpu, bench (S=16), rocprofv3 kernel-trace stats of the same bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit 0
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --scenes 16 --cpu-seconds 10 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.log
[ $rc -eq 0 ] || exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof -o b16 --output-format csv -- python bench.py --steps 1 --warmup 1 --scenes 16 --no-cpu-baseline > gpurun_out/prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof.log
exit 0
