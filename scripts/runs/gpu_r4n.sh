#!/bin/bash
# round 4: config B at 31 scenes on the lane kernel vs the 4 x 4 grid class
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n
for v in lane grid; do
  extra=""; [ $v = grid ] && extra="--small-grid"
  timeout -k 10 400 python -u bench.py --workload B --no-extra --no-cpu-baseline --steps 10 --warmup 2 $extra > gpurun_out/r4n/bench_B_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r4n/bench_B_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4n/bench_B_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('B $v', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us frac', r['frac'], 'traffic', r.get('traffic'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n/ktB -o kt -- python bench.py --workload B --no-extra --no-cpu-baseline --no-traffic --steps 2 --warmup 1 > gpurun_out/r4n/ktB.log 2>&1 || { echo "kt failed"; exit 1; }
head -8 $(find gpurun_out/r4n/ktB -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
