#!/bin/bash
# Whole -m gpu suite and smoke() on the current tree.
mkdir -p gpurun_out
TAG=${TAG:-suite}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -2
grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head -20
exit $rc
