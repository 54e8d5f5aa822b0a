#!/bin/bash
# round 4: staged observation loads (lane kernels), SCM blocks loaded before the stores (2D kernels)
# -- the whole GPU suite, then B / N2 / C / E comp timing and kernel statistics
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4s
timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r4s/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4s/pytest.log | tail -6
[ $rc -ne 0 ] && exit $rc
for W in B N2 C E_comp; do for v in new; do
  if [ $v = base ]; then export DANSE_LIB=$PWD/danse_amd/libdanse_base.so; else unset DANSE_LIB; fi
  timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4s/bench_${W}_$v.log 2>&1 || { echo "bench $W $v failed"; tail -5 gpurun_out/r4s/bench_${W}_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4s/bench_${W}_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W $v', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
done; done
unset DANSE_LIB
for W in B N2; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s/kt$W -o kt -- python bench.py --workload $W --steps 2 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4s/kt$W.log 2>&1 || { echo "kt failed"; exit 1; }
head -6 $(find gpurun_out/r4s/kt$W -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
done
