#!/bin/bash
# round 4: rank-one factor path reads each block row before its stores, DXCP
# state / tables, T(z) IR waves and chunk staging, wide triangular solves -- the whole GPU
# suite, then B / N2 / C / E comp timing (B also with eight-wave broadcasts;
# B and E comp also without the broadcast's pre-FFT weight loads: DANSE_LIB)
# and the kernel statistics of C and E comp
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4t
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r4t/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4t/pytest.log | tail -6
[ $rc -ne 0 ] && exit $rc
for W in B N2 C E_comp; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4t/bench_$W.log 2>&1 || { echo "bench $W failed"; tail -5 gpurun_out/r4t/bench_$W.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4t/bench_$W.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
done
DANSE_BCAST_WAVES=8 timeout -k 10 300 python -u bench.py --workload B --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4t/bench_B_w8.log 2>&1 || { echo "bench B w8 failed"; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4t/bench_B_w8.log').read().strip().splitlines()[-1]); print('B bcast8', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms')"
for W in B E_comp; do
DANSE_LIB=$PWD/danse_amd/libdanse_base.so timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4t/bench_${W}_nowpre.log 2>&1 || { echo "bench $W nowpre failed"; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4t/bench_${W}_nowpre.log').read().strip().splitlines()[-1]); print('$W no-weight-prefetch', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms')"
done
for W in C E_comp; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4t/kt$W -o kt -- python bench.py --workload $W --steps 2 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/r4t/kt$W.log 2>&1 || { echo "kt failed"; exit 1; }
python - "$(find gpurun_out/r4t/kt$W -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(r['Name'][:70], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 2), 'ms', round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
