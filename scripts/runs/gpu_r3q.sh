#!/bin/bash
# quick check: condition numbers (default path), split solves on B (parity + speed)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_engine_modes.py -m gpu -q -s -k "condition" --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cond_r3q.log 2>&1
rc=$?; grep -E "passed|failed|cond error" gpurun_out/pytest_cond_r3q.log | tail -3; [ $rc -eq 0 ] || exit $rc
DANSE_LANE_SPLIT=1 timeout -k 10 250 python -u -m pytest tests/test_gpu_engine_modes.py -m gpu -q -s -x -k "config_B_shape or headline" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_split_r3q.log 2>&1
rc=$?; grep -E "passed|failed|online_" gpurun_out/pytest_split_r3q.log | tail -6; [ $rc -eq 0 ] || exit $rc
DANSE_LANE_SPLIT=1 timeout -k 10 200 python bench.py --workload B --no-cpu-baseline --no-traffic --no-extra > gpurun_out/bench_split_r3q.log 2>&1 || exit 1
DANSE_LANE_SPLIT=1 timeout -k 10 200 python bench.py --workload N2 --no-cpu-baseline --no-traffic --no-extra > gpurun_out/bench_N2split_r3q.log 2>&1 || exit 1
for f in gpurun_out/bench_split_r3q.log gpurun_out/bench_N2split_r3q.log; do tail -1 $f | cut -c1-160; done
