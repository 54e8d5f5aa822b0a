#!/bin/bash
# round 4: warm-started rank-1 Lanczos (lane-grid classes + resident engine)
# parity, then N2 / B / resident timing and the N2 rocprof statistics
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py -k "headline or 2d or grid or shape or kat or online_engine or filter_update or resident" > gpurun_out/r4f/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed| w \{|resident w" gpurun_out/r4f/pytest.log | tail -60
[ $rc -ne 0 ] && exit $rc
for v in warm nowarm; do
  if [ $v = nowarm ]; then export DANSE_NO_WARM=1; else unset DANSE_NO_WARM; fi
  timeout -k 10 300 python -u bench.py --workload N2 --steps 5 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4f/bench_N2_$v.log 2>&1 || { echo "bench N2 $v failed"; tail -5 gpurun_out/r4f/bench_N2_$v.log; exit 1; }
  echo "N2 $v: $(tail -1 gpurun_out/r4f/bench_N2_$v.log | cut -c1-400)"
done
unset DANSE_NO_WARM
timeout -k 10 400 python -u bench.py --workload B --steps 10 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4f/bench_B.log 2>&1 || { echo "bench B failed"; tail -5 gpurun_out/r4f/bench_B.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r4f/bench_B.log').read().strip().splitlines()[-1])
print('B', d['value'] / 1e6, 'M FU/s', d['ms_per_step'], 'ms; roofline', d.get('roofline'))
for k, v in (d.get('extra') or {}).items():
    print(' ', k, round(v.get('value', 0) / 1e6, 1), 'M FU/s', v.get('ms_per_step'))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4f/profN2 -o kt -- python -u bench.py --workload N2 --steps 3 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4f/profN2.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/r4f/profN2.log; exit 1; }
find gpurun_out/r4f/profN2 -name "*kernel_stats.csv" | head -1 | xargs head -6
