#!/bin/bash
# GPU parity tests only (pytest -m gpu), optional -k filter in $K.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-t}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider "${KARG[@]}" > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu_$TAG.log
exit $rc
