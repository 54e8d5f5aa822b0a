#!/bin/bash
# Device metrics parity (fwSNRseg / SNR vs the reference fixtures and the oracle)
# and the batch node-sharding tests.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_metrics.py -m gpu > gpurun_out/metrics_tests.log 2>&1
