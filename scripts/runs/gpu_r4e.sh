#!/bin/bash
# round 4: warm-started rank-1 Lanczos on the lane-grid GEVD classes --
# parity of every 2d-class case (incl. the N2 headline K = 32 x 8), then N2
# timing with and without the warm start, and the rocprof kernel statistics
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py -k "headline or 2d or grid or shape or kat or online_engine or filter_update" > gpurun_out/r4e/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed| w \{" gpurun_out/r4e/pytest.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload N2 --steps 5 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4e/bench_N2_warm.log 2>&1 || { echo "bench warm failed"; tail -5 gpurun_out/r4e/bench_N2_warm.log; exit 1; }
tail -1 gpurun_out/r4e/bench_N2_warm.log
DANSE_NO_WARM=1 timeout -k 10 300 python -u bench.py --workload N2 --steps 5 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4e/bench_N2_nowarm.log 2>&1 || { echo "bench nowarm failed"; exit 1; }
tail -1 gpurun_out/r4e/bench_N2_nowarm.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e/profN2 -o kt -- python -u bench.py --workload N2 --steps 3 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4e/profN2.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/r4e/profN2.log; exit 1; }
find gpurun_out/r4e/profN2 -name "*kernel_stats.csv" | head -1 | xargs head -6
