#!/bin/bash
# round 4: recursion-only update variants for rounds without a solver item
# (UpdateArgs.noSolve) -- parity, N2 / B with and without (DANSE_NO_RO),
# B at 31 scenes on the 4 x 4 grid class
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4o
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py -k "online or large_D or headline or shape or resident or keep_history or sharded" > gpurun_out/r4o/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4o/pytest.log | tail -6
[ $rc -ne 0 ] && exit $rc
for v in ro noro; do
  if [ $v = noro ]; then export DANSE_NO_RO=1; else unset DANSE_NO_RO; fi
  timeout -k 10 300 python -u bench.py --workload N2 --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4o/bench_N2_$v.log 2>&1 || { echo "bench N2 $v failed"; tail -5 gpurun_out/r4o/bench_N2_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4o/bench_N2_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('N2 $v', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
  timeout -k 10 400 python -u bench.py --workload B --no-extra --no-cpu-baseline --no-traffic --steps 10 --warmup 2 > gpurun_out/r4o/bench_B_$v.log 2>&1 || { echo "bench B $v failed"; tail -5 gpurun_out/r4o/bench_B_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4o/bench_B_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('B $v', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us frac', r['frac'])"
done
unset DANSE_NO_RO
timeout -k 10 400 python -u bench.py --workload B --no-extra --no-cpu-baseline --no-traffic --steps 10 --warmup 2 --small-grid > gpurun_out/r4o/bench_B_grid.log 2>&1 || { echo "bench B grid failed"; tail -5 gpurun_out/r4o/bench_B_grid.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4o/bench_B_grid.log').read().strip().splitlines()[-1]); r=d['roofline']; print('B grid', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us frac', r['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4o/ktB -o kt -- python bench.py --workload B --no-extra --no-cpu-baseline --no-traffic --steps 2 --warmup 1 > gpurun_out/r4o/ktB.log 2>&1 || { echo "kt failed"; exit 1; }
head -8 $(find gpurun_out/r4o/ktB -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
