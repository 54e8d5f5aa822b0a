#!/bin/bash
# round 4 closing on HEAD (the broadcast weight prefetch reverted): the whole
# GPU suite, smoke, the default bench line, kernel statistics of B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4close3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -6
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktB -o kt -- python bench.py --no-extra --steps 2 --warmup 1 --no-traffic --no-cpu-baseline > $O/ktB.log 2>&1 || { echo "kt B failed"; exit 1; }
python - "$(find $O/ktB -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:4]:
    print(r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 2), 'ms', round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
