#!/bin/bash
# round 4: hipGraph replay check (memset nodes vs the fill kernel), dist /
# resident / condition-number tests, config C with DXCP at K = 16 x 4
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/graph_replay_check.py > gpurun_out/graph_replay_r4b.log 2>&1 || { echo "graph check failed rc=$?"; tail -20 gpurun_out/graph_replay_r4b.log; exit 1; }
grep -v amdgpu.ids gpurun_out/graph_replay_r4b.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_engine_modes.py tests/test_gpu_dxcp.py -k "rccl or sharded or resident or condition or dxcp" > gpurun_out/pytest_r4b.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|DXCP|pair|config C|cond error" gpurun_out/pytest_r4b.log | tail -40
exit $rc
