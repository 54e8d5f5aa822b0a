#!/bin/bash
# round 4: broadcast jobs reordered (the fused-spectrum frames first on every
# wave, then wave 0's z chain beside the other waves' update-frame analyses)
# -- the whole GPU suite, smoke, the default bench line, B / N2 against the
# previous library (DANSE_LIB=libdanse_base.so), kernel statistics of B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -6
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
line() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r.get('kernel'), r.get('frac'))" "$1" "$2"; }
for W in B N2; do for v in new base; do
  if [ $v = base ]; then export DANSE_LIB=$PWD/danse_amd/libdanse_base.so; else unset DANSE_LIB; fi
  timeout -k 10 200 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > $O/bench_${W}_$v.log 2>&1 || { echo "bench $W $v failed"; tail -5 $O/bench_${W}_$v.log; exit 1; }
  line $O/bench_${W}_$v.log "$W $v"
done; done
unset DANSE_LIB
for W in B; do
  X=""; [ $W = B ] && X="--no-extra"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$W -o kt -- python bench.py --workload $W $X --steps 2 --warmup 1 --no-traffic --no-cpu-baseline > $O/kt$W.log 2>&1 || { echo "kt $W failed"; exit 1; }
  python - "$(find $O/kt$W -name '*kernel_stats.csv' | head -1)" $W <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:4]:
    print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 2), 'ms', round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
