#!/bin/bash
# round 4 closing: smoke, the default bench line, kernel statistics of B / N2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4final
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r4final/smoke.log; exit 1; }
tail -2 gpurun_out/r4final/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4final/bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4final/bench_default.log; exit 1; }
tail -1 gpurun_out/r4final/bench_default.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final/ktB -o kt -- python bench.py --no-extra --no-traffic --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r4final/ktB.log 2>&1 || { echo "ktB failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final/ktN2 -o kt -- python bench.py --workload N2 --no-traffic --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r4final/ktN2.log 2>&1 || { echo "ktN2 failed"; exit 1; }
for w in B N2; do head -4 $(find gpurun_out/r4final/kt$w -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4; done
# A/B: the N2 class compiled for 3 waves per EU (danse_amd/exp build)
DANSE_LIB=$PWD/danse_amd/exp/libdanse_mi355x.so timeout -k 10 300 python -u bench.py --workload N2 --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4final/bench_N2_w3.log 2>&1 || { echo "bench w3 failed"; tail -5 gpurun_out/r4final/bench_N2_w3.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4final/bench_N2_w3.log').read().strip().splitlines()[-1]); r=d['roofline']; print('N2 w3', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
