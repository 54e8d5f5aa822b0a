#!/bin/bash
# Round-3 check: new-feature GPU tests, then the E battery bench grid.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3c}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_metrics.py tests/test_gpu_dxcp.py tests/test_gpu_scene.py -m gpu -v -s \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${PYTEST_K:-sro_nocomp or L256 or stoi or end_to_end or cl_dxcp or tdoa or dxcp or get_metrics or scene}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_$TAG.log | tail -2
grep -E "^FAILED" gpurun_out/pytest_$TAG.log | head -20
[ "$rc" = "0" ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
for spec in "E_noComp 64" "E_compNoFlags 64" "E_comp 64" "E_comp 32" "E_comp 128" "E_comp 256"; do
  set -- $spec
  timeout -k 10 300 python bench.py --workload $1 --L $2 --scenes 512 --steps 2 --warmup 1 --cpu-seconds 8 --no-traffic \
    > gpurun_out/bench_${1}_L$2_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_${1}_L$2_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_${1}_L$2_$TAG.log | cut -c1-200
done
exit 0
