#!/bin/bash
# Node-sharded batch DANSE: parity of the sharded engines vs the full run,
# the existing batch tests, and a config-D bench line (N=1, unchanged path).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "batch" > gpurun_out/batch_shard_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload D --steps 3 --warmup 1 > gpurun_out/batch_shard_benchD.log 2>&1
