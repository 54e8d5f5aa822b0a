#!/bin/bash
# Selected GPU tests (PYTEST_K), then one SQ-counter pass over the config-B
# bench (update kernel instruction mix / wave cycles).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2}
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "$PYTEST_K" > gpurun_out/pytest_sel_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_sel_$TAG.log | tail -2
grep -E "^FAILED" gpurun_out/pytest_sel_$TAG.log | head
[ "$rc" = "0" ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/pmcB_$TAG -o pmc --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-traffic --no-extra > gpurun_out/pmcB_$TAG.log 2>&1 || { tail -5 gpurun_out/pmcB_$TAG.log; exit 1; }
python scripts/pmc_sq.py gpurun_out/pmcB_$TAG/pmc_counter_collection.csv update_kernel
