#!/bin/bash
# bench sweep over scenes per GPU (no CPU baseline), one line per S
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-sweep}
for S in ${SCENES:-15 16 31}; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --scenes $S --no-cpu-baseline --no-traffic > gpurun_out/bench_${TAG}_S$S.log 2>&1 || { echo "bench S=$S failed"; tail -20 gpurun_out/bench_${TAG}_S$S.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_S$S.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('S', $S, 'value %.3e' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'upd ms %.4f' % d['roofline']['avg_launch_ms'], 'frac %.3f' % d['roofline']['frac'])"
done
