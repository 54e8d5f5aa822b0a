#!/bin/bash
# round 4: packed bin-major SCM storage on the grid / row classes -- parity
# over the online engine files, N2 / C / B-resident timing, N2 kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py > gpurun_out/r4h/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4h/pytest.log | tail -15
[ $rc -ne 0 ] && exit $rc
for W in N2 C; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r4h/bench_${W}.log 2>&1 || { echo "bench $W failed"; tail -5 gpurun_out/r4h/bench_${W}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4h/bench_${W}.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'], 'traffic', r.get('traffic'), r.get('traffic_detail'))"
done
timeout -k 10 300 python -u bench.py --workload B --scenes 1 --resident --steps 5 --warmup 2 --no-extra --no-traffic --no-cpu-baseline > gpurun_out/r4h/bench_Bres.log 2>&1 || { echo "bench Bres failed"; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4h/bench_Bres.log').read().strip().splitlines()[-1]); print('B S1 resident', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],2), 'ms')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h/ktN2 -o kt -- python bench.py --workload N2 --steps 2 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4h/ktN2.log 2>&1 || { echo "kt failed"; exit 1; }
head -4 $(find gpurun_out/r4h/ktN2 -name "*kernel_stats.csv" | head -1)
