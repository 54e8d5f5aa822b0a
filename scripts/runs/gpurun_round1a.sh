#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 --scenes 4 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
  echo "bench rc=$?" >> gpurun_out/bench.log
fi
exit 0
