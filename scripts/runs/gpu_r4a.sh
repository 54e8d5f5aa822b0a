#!/bin/bash
# round 4, first GPU call: hipGraph replay check + dist / engine-mode tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/graph_replay_check.py > gpurun_out/graph_replay_r4a.log 2>&1 || { echo "graph check failed rc=$?"; tail -20 gpurun_out/graph_replay_r4a.log; exit 1; }
cat gpurun_out/graph_replay_r4a.log | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_engine_modes.py -k "rccl or sharded or resident or condition" > gpurun_out/pytest_r4a.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_r4a.log
exit $rc
