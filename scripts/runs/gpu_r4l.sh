#!/bin/bash
# round 4: rank-one factor updates v2 (shuffle scans) -- grid-class parity,
# N2 / C timing with and without; E at round 2's DANSE-only setting
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4l
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py -k "large_D or headline or C_shape or kat_gevd" > gpurun_out/r4l/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4l/pytest.log | tail -6
grep -E "headline|C_shape|D27|D51" gpurun_out/r4l/pytest.log | grep " w " | cut -c1-200 | head -8
[ $rc -ne 0 ] && exit $rc
for W in N2 C; do for v in r1 nor1; do
  if [ $v = nor1 ]; then export DANSE_NO_R1=1; else unset DANSE_NO_R1; fi
  timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4l/bench_${W}_$v.log 2>&1 || { echo "bench $W $v failed"; tail -5 gpurun_out/r4l/bench_${W}_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4l/bench_${W}_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W $v', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
done; done
unset DANSE_NO_R1
timeout -k 10 300 python -u bench.py --workload E_L64_sro200 --scenes 512 --scene-gen device --steps 4 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4l/bench_E_sro200.log 2>&1 || { echo "bench E failed"; tail -5 gpurun_out/r4l/bench_E_sro200.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4l/bench_E_sro200.log').read().strip().splitlines()[-1]); r=d['roofline']; print('E_L64_sro200', round(d['value']/1e9,3), 'G FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
