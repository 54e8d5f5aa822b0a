#!/bin/bash
# round 4: split broadcast (one wave per analysis + the synthesis launch) on
# small grids -- parity + dist, N2 / C timing with and without (DANSE_NO_BSPLIT)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4p
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py tests/test_gpu_dist.py -k "online or large_D or headline or shape or resident or keep_history or sharded or dist or rccl or gate" > gpurun_out/r4p/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4p/pytest.log | tail -6
[ $rc -ne 0 ] && exit $rc
for W in N2 C; do for v in split nosplit; do
  if [ $v = nosplit ]; then export DANSE_NO_BSPLIT=1; else unset DANSE_NO_BSPLIT; fi
  timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4p/bench_${W}_$v.log 2>&1 || { echo "bench $W $v failed"; tail -5 gpurun_out/r4p/bench_${W}_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4p/bench_${W}_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W $v', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
done; done
unset DANSE_NO_BSPLIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4p/ktN2 -o kt -- python bench.py --workload N2 --steps 2 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4p/ktN2.log 2>&1 || { echo "kt failed"; exit 1; }
head -6 $(find gpurun_out/r4p/ktN2 -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
