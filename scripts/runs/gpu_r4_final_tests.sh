#!/bin/bash
# round 4 closing: the whole GPU test suite on HEAD
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4final
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 1100 --timeout-method thread > gpurun_out/r4final/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/r4final/pytest_gpu.log | tail -8
exit $rc
