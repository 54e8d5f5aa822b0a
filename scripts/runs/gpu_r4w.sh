#!/bin/bash
# round 4, last: refreshed lines for config D (batch), C with DXCP-PhaT
# estimation, and E_L64_sro200 on HEAD (after the held-load-run kernels)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4w
mkdir -p $O
line() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r.get('kernel'), r.get('frac'))" "$1" "$2"; }
for W in D C_dxcp E_L64_sro200; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 3 --warmup 1 --no-traffic --no-cpu-baseline > $O/bench_$W.log 2>&1 || { echo "bench $W failed"; tail -5 $O/bench_$W.log; exit 1; }
  line $O/bench_$W.log $W
done
