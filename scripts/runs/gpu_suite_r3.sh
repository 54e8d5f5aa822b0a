#!/bin/bash
# Round-3 GPU check: smoke() and the whole -m gpu suite.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_SEL:-} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -2
grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head -20
exit $rc
