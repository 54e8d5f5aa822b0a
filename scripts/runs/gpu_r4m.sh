#!/bin/bash
# round 4: 8-wave broadcast workgroups for small grids (S K <= 128) -- engine
# parity, dist, then N2 / C timing and the default bench line (B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4m
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py tests/test_gpu_dist.py > gpurun_out/r4m/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4m/pytest.log | tail -6
[ $rc -ne 0 ] && exit $rc
for W in N2 C; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4m/bench_${W}.log 2>&1 || { echo "bench $W failed"; tail -5 gpurun_out/r4m/bench_${W}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4m/bench_${W}.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
done
timeout -k 10 600 python -u bench.py > gpurun_out/r4m/bench_default.log 2>&1 || { echo "default bench failed"; tail -5 gpurun_out/r4m/bench_default.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4m/bench_default.log').read().strip().splitlines()[-1]); r=d['roofline']; print('default', d['config'].get('workload'), round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us frac', r['frac'], 'traffic', r.get('traffic')); [print('  ', k, round(v['value']/1e6,1), round(v['ms_per_step'],2)) for k, v in (d.get('extra_lines') or {}).items()]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4m/ktN2 -o kt -- python bench.py --workload N2 --steps 2 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4m/ktN2.log 2>&1 || { echo "kt failed"; exit 1; }
head -5 $(find gpurun_out/r4m/ktN2 -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
