#!/bin/bash
# round 4: hipGraph replay check, dist / resident / condition-number / DXCP
# (config C K = 16 x 4) tests, and the fewSamples step lists (E battery cells)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/graph_replay_check.py > gpurun_out/graph_replay_r4c.log 2>&1 || { echo "graph check failed rc=$?"; tail -20 gpurun_out/graph_replay_r4c.log; exit 1; }
grep -v amdgpu.ids gpurun_out/graph_replay_r4c.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "online_E or fs" > gpurun_out/pytest_E_r4c.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_E_r4c.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1200 python -u -m pytest -v -s --timeout 900 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_engine_modes.py tests/test_gpu_dxcp.py -k "rccl or sharded or resident or condition or dxcp or keep_history" > gpurun_out/pytest_r4c.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|DXCP|pair|config C|cond error" gpurun_out/pytest_r4c.log | tail -40
exit $rc
