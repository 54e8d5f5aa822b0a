#!/bin/bash
# One GPU session on the MI355X box, as a list of steps (replaces the one-off
# command files of rounds 1-4, which stay in the git history):
#
#   bash scripts/gpu_session.sh TAG STEP [STEP ...]
#
# Steps (outputs under gpurun_out/TAG/):
#   suite                 the whole `pytest -m gpu` suite
#   tests:EXPR            `pytest -m gpu -k EXPR`
#   smoke                 __graft_entry__.smoke()
#   bench                 the default `python bench.py` line (driver settings: --steps 20 --warmup 5)
#   wl:W[:ARGS]           bench.py --workload W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline ARGS
#                         (ARGS: comma-separated extra flags, e.g. wl:B:--no-extra,--scenes,62)
#   kt:W                  rocprofv3 --kernel-trace --stats of a 2-step bench of W (kernel statistics)
#   pmc:W:CNT[,CNT...]    one rocprofv3 --pmc pass of the un-graphed bench pass of W (counters of one
#                         pass only: at most 8 SQ_, 4 TCC_ (FETCH_SIZE uses 3), 2 TA_/TD_/GRBM_)
# Every GPU step runs under its own timeout; the session stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
NT=0
summary() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get('roofline') or {}
print(sys.argv[2], round(d['value'] / 1e6, 1), 'M FU/s', round(d['ms_per_step'], 2), 'ms/step', r.get('kernel'),
      'avg', r.get('avg_launch_ms'), 'frac', r.get('frac'), 'lanczos', r.get('lanczos'))
for k, e in (d.get('extra_lines') or {}).items():
    rr = e.get('roofline') or {}
    print('  ', k, round(e['value'] / 1e6, 1), 'M FU/s', round(e['ms_per_step'], 2), 'ms/step', rr.get('kernel'),
          'avg', rr.get('avg_launch_ms'), 'frac', rr.get('frac'), 'x cpu', e.get('gpu_over_cpu'))
PY
}
for step in "$@"; do
  IFS=: read -r kind a1 a2 <<< "$step"
  case $kind in
    suite)
      timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests \
        > "$O/pytest_gpu.log" 2>&1 || { echo "suite failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
      grep -E "passed|failed" "$O/pytest_gpu.log" | tail -2 ;;
    tests)
      NT=$((NT + 1))
      timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests -k "$a1" \
        > "$O/pytest_k$NT.log" 2>&1 || { echo "tests failed"; tail -40 "$O/pytest_k$NT.log"; exit 1; }
      grep -E "passed|failed" "$O/pytest_k$NT.log" | tail -2 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -5 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > "$O/bench_default.log" 2>&1 \
        || { echo "bench failed"; tail -20 "$O/bench_default.log"; exit 1; }
      summary "$O/bench_default.log" default ;;
    wl)
      X=${a2//,/ }
      timeout -k 10 300 python -u bench.py --workload "$a1" --steps 4 --warmup 2 --no-traffic --no-cpu-baseline $X \
        > "$O/bench_$a1.log" 2>&1 || { echo "bench $a1 failed"; tail -20 "$O/bench_$a1.log"; exit 1; }
      summary "$O/bench_$a1.log" "$a1" ;;
    kt)
      X=""; [ "$a1" = B ] && X="--no-extra"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt$a1" -o kt -- \
        python bench.py --workload "$a1" $X --steps 2 --warmup 1 --no-traffic --no-cpu-baseline \
        > "$O/kt$a1.log" 2>&1 || { echo "kt $a1 failed"; tail -5 "$O/kt$a1.log"; exit 1; }
      python - "$(find "$O/kt$a1" -name '*kernel_stats.csv' | head -1)" "$a1" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(sys.argv[2], r['Name'][:70], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 2), 'ms',
          round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
      ;;
    pmc)
      timeout -s KILL 120 rocprofv3 --pmc ${a2//,/ } --kernel-trace --output-format csv -d "$O/pmc_${a1}_${a2//,/_}" \
        -o pmc -- python bench.py --pmc-child --workload "$a1" > "$O/pmc_${a1}.log" 2>&1 \
        || { echo "pmc $a1 $a2 failed"; tail -5 "$O/pmc_${a1}.log"; exit 1; }
      echo "pmc $a1 $a2 done" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
