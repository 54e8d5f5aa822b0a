#!/bin/bash
# GPU parity suite (all -m gpu tests), one process, time-limited.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu_$TAG.log
exit $rc
