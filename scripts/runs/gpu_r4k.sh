#!/bin/bash
# round 4: rank-one updates of the float64 factor record (li_rank1_2d) --
# parity of the grid classes, N2 / C timing with and without (DANSE_NO_R1),
# E kernel trace (the E line's drop since round 2)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py -k "large_D or headline or shape or resident or online_engine_vs_oracle" > gpurun_out/r4k/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4k/pytest.log | tail -8
grep -E "headline|C_shape|D27|D51|D20|B_shape" gpurun_out/r4k/pytest.log | grep " w " | cut -c1-200 | head -12
[ $rc -ne 0 ] && exit $rc
for W in N2 C; do for v in r1 nor1; do
  if [ $v = nor1 ]; then export DANSE_NO_R1=1; else unset DANSE_NO_R1; fi
  timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4k/bench_${W}_$v.log 2>&1 || { echo "bench $W $v failed"; tail -5 gpurun_out/r4k/bench_${W}_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4k/bench_${W}_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W $v', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
done; done
unset DANSE_NO_R1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4k/ktE -o kt -- python bench.py --workload E_comp --L 64 --scenes 512 --scene-gen device --steps 2 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4k/ktE.log 2>&1 || { echo "ktE failed"; tail -5 gpurun_out/r4k/ktE.log; exit 1; }
head -12 $(find gpurun_out/r4k/ktE -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
