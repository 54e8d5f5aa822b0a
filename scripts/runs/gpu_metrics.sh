#!/bin/bash
# Device metrics parity (fwSNRseg / SNR / get_metrics vs the reference fixtures
# and the oracle), then the E workload at the battery's 200 ppm SRO setting.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_metrics.py -m gpu > gpurun_out/metrics_tests.log 2>&1
timeout -k 10 400 python -u bench.py --workload E_L64_sro200 --scenes 512 --steps 3 --warmup 1 > gpurun_out/bench_E_sro200.log 2>&1
