#!/bin/bash
# round 4 closing, second pass (after the held-load-run kernels): smoke, the
# default bench line, kernel statistics of B / N2 on HEAD
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4close2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4close2/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r4close2/smoke.log; exit 1; }
tail -2 gpurun_out/r4close2/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4close2/bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4close2/bench_default.log; exit 1; }
tail -1 gpurun_out/r4close2/bench_default.log | cut -c1-700
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4close2/ktB -o kt -- python bench.py --no-extra --no-traffic --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r4close2/ktB.log 2>&1 || { echo "ktB failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4close2/ktN2 -o kt -- python bench.py --workload N2 --no-traffic --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r4close2/ktN2.log 2>&1 || { echo "ktN2 failed"; exit 1; }
for w in B N2; do
python - "$(find gpurun_out/r4close2/kt$w -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:5]:
    print(r['Name'][:70], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 2), 'ms', round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
